"""Image viewers for ``RemoteEnv.render('human')``.

Contract (reference: pkg_pytorch/blendtorch/btt/env_rendering.py:1-78): a
registry of named backends with the lookup order ``['openai', 'matplotlib']``
-- the gym viewer first, else a matplotlib window -- and a backend only
counts when its library imports.  Every viewer has ``imshow(rgb)`` and
``close()``.

Here each backend is a small factory that imports its library on first use
(so importing ``btt`` never pulls in matplotlib or gym), and a ``'null'``
backend, last in the order, keeps the frames for headless runs and tests.
"""
import importlib.util

LOOKUP_ORDER = ['openai', 'matplotlib', 'null']
RENDER_BACKENDS = {}


def _installed(package):
    """Is ``package`` installed?  (Checked without importing it.)"""
    try:
        return importlib.util.find_spec(package) is not None
    except (ImportError, ValueError):
        return False


def register_backend(name, factory, requires=None):
    """Add a viewer factory; ``requires`` names a package that must be installed."""
    if requires is None or _installed(requires):
        RENDER_BACKENDS[name] = factory


def create_renderer(backend=None, **kwargs):
    """Instantiate ``backend`` (a registered name), or the first registered
    backend in :data:`LOOKUP_ORDER`."""
    if backend is not None:
        if backend not in RENDER_BACKENDS:
            raise AssertionError(f'Render backend {backend} not found.')
        return RENDER_BACKENDS[backend](**kwargs)
    for name in LOOKUP_ORDER:
        if name in RENDER_BACKENDS:
            return RENDER_BACKENDS[name](**kwargs)
    raise AssertionError('No render backends available.')


class NullRenderer:
    """Displays nothing; remembers the last frame and counts frames."""

    def __init__(self, **kwargs):
        self.last, self.shown = None, 0

    def imshow(self, rgb):
        self.last, self.shown = rgb, self.shown + 1

    def close(self):
        self.last = None


class _FigureViewer:
    """One matplotlib figure whose image is updated in place."""

    def __init__(self, **kwargs):
        import matplotlib.pyplot as plt
        self._plt = plt
        self.fig, ax = plt.subplots(1, 1)
        self._ax, self._artist = ax, None

    def imshow(self, rgb):
        if self._artist is not None:
            self._artist.set_data(rgb)
            self.fig.canvas.draw_idle()
            self.fig.canvas.flush_events()
            return
        self._artist = self._ax.imshow(rgb)
        self._plt.show(block=False)
        self.fig.canvas.draw()

    def close(self):
        fig, self.fig = self.fig, None
        if fig is not None:
            self._plt.close(fig)

    def __del__(self):
        self.close()


class _GymViewer:
    """gym's ``SimpleImageViewer`` (classic-control rendering)."""

    def __init__(self, **kwargs):
        from gym.envs.classic_control import rendering
        self._viewer = rendering.SimpleImageViewer(**kwargs)

    def imshow(self, rgb):
        self._viewer.imshow(rgb)

    def close(self):
        viewer, self._viewer = self._viewer, None
        if viewer is not None:
            viewer.close()

    def __del__(self):
        self.close()


# reference names, kept importable
MatplotlibRenderer = _FigureViewer
OpenAIGymRenderer = _GymViewer

register_backend('null', NullRenderer)
register_backend('matplotlib', _FigureViewer, requires='matplotlib')
register_backend('openai', _GymViewer, requires='gym')
