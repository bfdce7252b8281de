"""Records the callback order of two episodes over frames 1..3 and publishes it."""
import bpy
from blendtorch import btb

btargs, remainder = btb.parse_blendtorch_args()
seq = []
pub = btb.DataPublisher(btargs.btsockets['DATA'], btargs.btid, lingerms=5000)
anim = btb.AnimationController()
for name in ('pre_play', 'pre_animation', 'pre_frame', 'post_frame', 'post_animation'):
    getattr(anim, name).add(lambda n=name: seq.extend([n, anim.frameid]))


def post_play():
    seq.extend(['post_play', anim.frameid])
    pub.publish(seq=seq)


anim.post_play.add(post_play)
anim.play(frame_range=(1, 3), num_episodes=2, use_animation=not bpy.app.background)
