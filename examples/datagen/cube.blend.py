"""Cube producer, Blender side (scene: cube.blend; the message contract of
the reference's examples/datagen/cube.blend.py).

Every frame the cube gets a random orientation; after the frame the producer
publishes ``{'btid', 'image': H x W x 3 render, 'xy': 8 x 2 projected cube
corners, 'frameid'}``.  Runs inside Blender, or headless under
``blendtorch.btb.headless`` (scene preset 'cube').  ``bench.py`` uses the
native stand-in ``blendtorch/bin/cubesim`` with the same contract.
"""
import bpy
import numpy as np
from blendtorch import btb


class CubeProducer:
    """Randomise before a frame, publish after it."""

    def __init__(self, args):
        self.rng = np.random.RandomState(args.btseed)
        self.cube = bpy.data.objects['Cube']
        self.camera = btb.Camera()
        self.renderer = btb.OffScreenRenderer(camera=self.camera, mode='rgb')
        self.renderer.set_render_style(shading='RENDERED', overlays=False)
        self.publisher = btb.DataPublisher(args.btsockets['DATA'], args.btid)
        self.loop = btb.AnimationController()
        self.loop.pre_frame.add(self.randomize)
        self.loop.post_frame.add(self.publish)

    def randomize(self):
        self.cube.rotation_euler = self.rng.uniform(0.0, np.pi, size=3)

    def publish(self):
        self.publisher.publish(image=self.renderer.render(), xy=self.camera.object_to_pixel(self.cube),
                               frameid=self.loop.frameid)

    def run(self):
        # interactive Blender: timer-driven playback; --background: blocking loop
        self.loop.play(frame_range=(0, 100), num_episodes=-1, use_animation=not bpy.app.background)


if __name__ == '__main__':
    btargs, _ = btb.parse_blendtorch_args()
    CubeProducer(btargs).run()
