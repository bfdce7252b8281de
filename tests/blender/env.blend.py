"""Scene script for tests/test_env.py: a minimal remote environment.

The action sets the cube's rotation about z. The observation is that angle,
the reward is 1 once the angle exceeds 0.5 in magnitude, and the episode ends
after ``--done-after`` frames. ``count`` reports how many steps the env has
taken since its last reset, which pins down the reply-lag protocol.
"""
import argparse

import bpy
from blendtorch import btb


class RotateCubeEnv(btb.env.BaseEnv):
    def __init__(self, agent, done_after):
        super().__init__(agent)
        self.cube = bpy.data.objects['Cube']
        self.done_after = done_after
        self.steps = 0

    def _env_reset(self):
        self.steps = 0
        self.cube.rotation_euler[2] = 0.0

    def _env_prepare_step(self, action):
        self.cube.rotation_euler[2] = action

    def _env_post_step(self):
        self.steps += 1
        z = self.cube.rotation_euler[2]
        return {'obs': z, 'reward': float(abs(z) > 0.5), 'count': self.steps,
                'done': self.events.frameid > self.done_after}


def script_args(argv):
    p = argparse.ArgumentParser()
    p.add_argument('--done-after', type=int, default=10)
    p.add_argument('--render-every', type=int, default=0)
    p.add_argument('--real-time', dest='real_time', action='store_true')
    p.add_argument('--no-real-time', dest='real_time', action='store_false')
    return p.parse_args(argv)


btargs, remainder = btb.parse_blendtorch_args()
opts = script_args(remainder)
env = RotateCubeEnv(btb.env.RemoteControlledAgent(btargs.btsockets['GYM'], real_time=opts.real_time),
                    done_after=opts.done_after)
if opts.render_every > 0 or not bpy.app.background:
    env.attach_default_renderer(every_nth=max(1, opts.render_every))
env.run(frame_range=(1, 10000), use_animation=not bpy.app.background)
