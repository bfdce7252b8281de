"""Supershape producer, Blender side (needs the external ``supershape``
package inside Blender; contract of the reference's
examples/densityopt/supershape.blend.py).  Headless stand-in:
``blendtorch/bin/supershapesim``.

The PyTorch side sends batches ``{'shape_params': N x 2 x 6, 'shape_ids': N}``
over the duplex channel.  Each frame polls it without blocking; a batch
replaces whatever is being rendered, and while a batch lasts every frame
morphs the mesh to its next shape and publishes the 64 x 64 gamma-corrected
render with that shape's id.
"""
import bpy  # noqa: F401  (Blender context for the renderer)
from blendtorch import btb

import supershape as sshape

UV_SHAPE = (100, 100)


class ShapeStream:
    """Works through the latest parameter batch, one shape per frame."""

    def __init__(self, duplex, publisher):
        self.duplex, self.publisher = duplex, publisher
        self.mesh = sshape.make_bpy_mesh(UV_SHAPE)
        self.queue = None          # iterator over (params, id) of the current batch
        self.current = None        # id of the shape shown in this frame
        self.renderer = btb.OffScreenRenderer(camera=btb.Camera(), mode='rgb', gamma_coeff=2.2)
        self.renderer.set_render_style(shading='SOLID', overlays=False)

    def before_frame(self):
        batch = self.duplex.recv(timeoutms=0)
        if batch is not None:
            self.queue = iter(zip(batch['shape_params'], batch['shape_ids']))
        if self.queue is None:
            return
        nxt = next(self.queue, None)
        if nxt is None:
            self.queue = self.current = None
            return
        params, self.current = nxt
        sshape.update_bpy_mesh(*sshape.supercoords(params, shape=UV_SHAPE), self.mesh)

    def after_frame(self):
        if self.queue is not None:
            self.publisher.publish(image=self.renderer.render(), shape_id=self.current)


if __name__ == '__main__':
    btargs, _ = btb.parse_blendtorch_args()
    stream = ShapeStream(btb.DuplexChannel(btargs.btsockets['CTRL'], btargs.btid),
                         btb.DataPublisher(btargs.btsockets['DATA'], btargs.btid))
    loop = btb.AnimationController()
    loop.pre_frame.add(stream.before_frame)
    loop.post_frame.add(stream.after_frame)
    loop.play(frame_range=(0, 10000), num_episodes=-1)
