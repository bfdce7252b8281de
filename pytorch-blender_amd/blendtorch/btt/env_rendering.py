"""Image viewers for ``RemoteEnv.render('human')``.

Reference: pkg_pytorch/blendtorch/btt/env_rendering.py -- a registry of
backends looked up in the order ``['openai', 'matplotlib']``; each backend
registers only when importable.  A 'null' backend (records the last frame,
displays nothing) is always available for headless use.
"""
RENDER_BACKENDS = {}
LOOKUP_ORDER = ['openai', 'matplotlib', 'null']


def create_renderer(backend=None, **kwargs):
    """Instantiate the named backend, or the first available one."""
    if backend is None:
        avail = [RENDER_BACKENDS[n] for n in LOOKUP_ORDER if n in RENDER_BACKENDS]
        assert len(avail) > 0, 'No render backends available.'
        return avail[0](**kwargs)
    assert backend in RENDER_BACKENDS, f'Render backend {backend} not found.'
    return RENDER_BACKENDS[backend](**kwargs)


class NullRenderer:
    """Keeps the last image; for headless runs and tests."""

    def __init__(self, **kwargs):
        self.last = None
        self.shown = 0

    def imshow(self, rgb):
        self.last = rgb
        self.shown += 1

    def close(self):
        self.last = None


RENDER_BACKENDS['null'] = NullRenderer

try:
    import matplotlib
    import matplotlib.pyplot as plt

    class MatplotlibRenderer:
        def __init__(self, **kwargs):
            self.fig, self.ax = plt.subplots(1, 1)
            self.img = None

        def imshow(self, rgb):
            if self.img is None:
                self.img = self.ax.imshow(rgb)
                plt.show(block=False)
                self.fig.canvas.draw()
            else:
                self.img.set_data(rgb)
                self.fig.canvas.draw_idle()
                self.fig.canvas.flush_events()

        def close(self):
            if self.fig is not None:
                plt.close(self.fig)
                self.fig = None

        def __del__(self):
            self.close()

    RENDER_BACKENDS['matplotlib'] = MatplotlibRenderer
except ImportError:
    pass

try:
    from gym.envs.classic_control import rendering as _gym_rendering

    class OpenAIGymRenderer:
        def __init__(self, **kwargs):
            self._viewer = _gym_rendering.SimpleImageViewer(**kwargs)

        def imshow(self, rgb):
            self._viewer.imshow(rgb)

        def close(self):
            if self._viewer:
                self._viewer.close()
                self._viewer = None

        def __del__(self):
            self.close()

    RENDER_BACKENDS['openai'] = OpenAIGymRenderer
except ImportError:
    pass
