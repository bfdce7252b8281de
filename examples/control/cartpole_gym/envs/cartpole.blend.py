"""Cart-pole environment, Blender side (scene: cartpole.blend with Bullet
rigid bodies; contract of the reference's
examples/control/cartpole_gym/envs/cartpole.blend.py).

Action: a force on the cart, applied as a change of the slider motor's target
velocity over one frame (dv = F / m_total / fps).  Observation: (cart x, pole
x, pole angle); reward 0; the episode is done once the pole tilts past 0.6
rad or the cart leaves [-4, 4].  The native stand-in
``blendtorch/bin/cartpolesim`` implements the same env without Blender.
"""
import argparse

import bpy
import numpy as np
from blendtorch import btb

MAX_ANGLE, MAX_OFFSET = 0.6, 4.0


class CartpoleEnv(btb.env.BaseEnv):
    def __init__(self, agent):
        super().__init__(agent)
        objs = bpy.data.objects
        self.cart, self.pole, self.hinge = objs['Cart'], objs['Pole'], objs['PoleRotHelp']
        self.motor = objs['Motor'].rigid_body_constraint
        # velocity change per unit force in one frame (physics runs at the scene fps)
        self.dv_per_force = 1.0 / ((self.cart.rigid_body.mass + self.pole.rigid_body.mass)
                                   * bpy.context.scene.render.fps)

    def _env_reset(self):
        self.motor.motor_lin_target_velocity = 0.0
        self.cart.location = (0.0, 0.0, 1.2)
        self.hinge.rotation_euler[1] = np.random.uniform(-MAX_ANGLE, MAX_ANGLE)

    def _env_prepare_step(self, action):
        self.motor.motor_lin_target_velocity += action * self.dv_per_force

    def _env_post_step(self):
        cart_x = self.cart.matrix_world.translation[0]
        pole_x = self.pole.matrix_world.translation[0]
        angle = self.pole.matrix_world.to_euler('XYZ')[1]
        return {'obs': (cart_x, pole_x, angle), 'reward': 0.0,
                'done': bool(abs(angle) > MAX_ANGLE or abs(cart_x) > MAX_OFFSET)}


def env_options(argv):
    p = argparse.ArgumentParser()
    p.add_argument('--render-every', type=int, default=None)
    p.add_argument('--real-time', dest='realtime', action='store_true')
    p.add_argument('--no-real-time', dest='realtime', action='store_false')
    return p.parse_args(argv)


if __name__ == '__main__':
    btargs, rest = btb.parse_blendtorch_args()
    opts = env_options(rest)
    env = CartpoleEnv(btb.env.RemoteControlledAgent(btargs.btsockets['GYM'], real_time=opts.realtime))
    if opts.render_every:
        env.attach_default_renderer(every_nth=opts.render_every)
    env.run(frame_range=(1, 10000), use_animation=True)
