"""Blender-side cart-pole env (needs cartpole.blend with Bullet rigid bodies).
The native stand-in blendtorch/bin/cartpolesim implements the same env."""
import argparse

import bpy
import numpy as np
from blendtorch import btb


class CartpoleEnv(btb.env.BaseEnv):
    def __init__(self, agent):
        super().__init__(agent)
        self.cart = bpy.data.objects['Cart']
        self.pole = bpy.data.objects['Pole']
        self.polerot = bpy.data.objects['PoleRotHelp']
        self.motor = bpy.data.objects['Motor'].rigid_body_constraint
        self.fps = bpy.context.scene.render.fps   # physics must run at the same rate
        self.total_mass = self.cart.rigid_body.mass + self.pole.rigid_body.mass

    def _env_reset(self):
        self.motor.motor_lin_target_velocity = 0.
        self.cart.location = (0.0, 0, 1.2)
        self.polerot.rotation_euler[1] = np.random.uniform(-0.6, 0.6)

    def _env_prepare_step(self, action):
        # constant acceleration between steps: v(t+1) = v(t) + (f/m) dt
        self.motor.motor_lin_target_velocity += action / self.total_mass / self.fps

    def _env_post_step(self):
        c = self.cart.matrix_world.translation[0]
        p = self.pole.matrix_world.translation[0]
        a = self.pole.matrix_world.to_euler('XYZ')[1]
        return dict(obs=(c, p, a), reward=0., done=bool(abs(a) > 0.6 or abs(c) > 4.0))


def main():
    args, remainder = btb.parse_blendtorch_args()
    parser = argparse.ArgumentParser()
    parser.add_argument('--render-every', default=None, type=int)
    parser.add_argument('--real-time', dest='realtime', action='store_true')
    parser.add_argument('--no-real-time', dest='realtime', action='store_false')
    envargs = parser.parse_args(remainder)
    agent = btb.env.RemoteControlledAgent(args.btsockets['GYM'], real_time=envargs.realtime)
    env = CartpoleEnv(agent)
    if envargs.render_every:
        env.attach_default_renderer(every_nth=envargs.render_every)
    env.run(frame_range=(1, 10000), use_animation=True)


main()
