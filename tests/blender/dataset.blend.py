"""Streams a 64x64 zero image per frame, frames 1..3 forever."""
import bpy
import numpy as np
from blendtorch import btb

btargs, remainder = btb.parse_blendtorch_args()
pub = btb.DataPublisher(btargs.btsockets['DATA'], btargs.btid, lingerms=5000)


def post_frame(pub, anim):
    pub.publish(frameid=anim.frameid, img=np.zeros((64, 64), dtype=np.uint8))


anim = btb.AnimationController()
anim.post_frame.add(post_frame, pub, anim)
anim.play(frame_range=(1, 3), num_episodes=-1, use_animation=not bpy.app.background)
