"""Blender-side supershape producer (runs inside Blender with the external
``supershape`` package, see the reference example's readme).  The headless
native equivalent is ``blendtorch/bin/supershapesim``.

Per frame: poll the duplex channel without blocking; a new message starts a
generator over its (shape_params, shape_ids); while it runs, each frame
updates the mesh and publishes the 64x64 gamma-corrected render with its id.
"""
import bpy  # noqa: F401
from blendtorch import btb

import supershape as sshape


def generate_supershape(msg, shape=(100, 100)):
    for params, shape_id in zip(msg['shape_params'], msg['shape_ids']):
        yield params, shape_id, sshape.supercoords(params, shape=shape)


def main():
    btargs, remainder = btb.parse_blendtorch_args()
    uvshape = (100, 100)
    obj = sshape.make_bpy_mesh(uvshape)
    state = {'gen': None, 'idx': None}

    def pre_frame(duplex):
        msg = duplex.recv(timeoutms=0)
        if msg is not None:
            state['gen'] = generate_supershape(msg, shape=uvshape)
        if state['gen'] is not None:
            try:
                _, state['idx'], coords = next(state['gen'])
                sshape.update_bpy_mesh(*coords, obj)
            except StopIteration:
                state['gen'] = None

    def post_frame(off, pub):
        if state['gen'] is not None:
            pub.publish(image=off.render(), shape_id=state['idx'])

    pub = btb.DataPublisher(btargs.btsockets['DATA'], btargs.btid)
    duplex = btb.DuplexChannel(btargs.btsockets['CTRL'], btargs.btid)
    off = btb.OffScreenRenderer(camera=btb.Camera(), mode='rgb', gamma_coeff=2.2)
    off.set_render_style(shading='SOLID', overlays=False)
    anim = btb.AnimationController()
    anim.pre_frame.add(pre_frame, duplex)
    anim.post_frame.add(post_frame, off, pub)
    anim.play(frame_range=(0, 10000), num_episodes=-1)


main()
