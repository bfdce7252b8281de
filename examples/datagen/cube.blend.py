"""Cube producer (Blender side): random cube rotation per frame; publishes the
render, the projected cube vertices and the frame id.  Runs in Blender with
cube.blend, or headless (`blendtorch.btb.headless`, scene preset 'cube').
The native C++ equivalent used by bench.py is blendtorch/bin/cubesim."""
import bpy
import numpy as np
from blendtorch import btb


def main():
    btargs, remainder = btb.parse_blendtorch_args()
    np.random.seed(btargs.btseed)
    cube = bpy.data.objects['Cube']

    def pre_frame():
        cube.rotation_euler = np.random.uniform(0, np.pi, size=3)

    def post_frame(off, pub, anim, cam):
        pub.publish(image=off.render(), xy=cam.object_to_pixel(cube), frameid=anim.frameid)

    pub = btb.DataPublisher(btargs.btsockets['DATA'], btargs.btid)
    cam = btb.Camera()
    off = btb.OffScreenRenderer(camera=cam, mode='rgb')
    off.set_render_style(shading='RENDERED', overlays=False)
    anim = btb.AnimationController()
    anim.pre_frame.add(pre_frame)
    anim.post_frame.add(post_frame, off, pub, anim, cam)
    anim.play(frame_range=(0, 100), num_episodes=-1, use_animation=not bpy.app.background)


main()
