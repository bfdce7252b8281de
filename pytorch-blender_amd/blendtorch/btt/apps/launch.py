"""``blendtorch-launch``: start producer instances from a JSON spec and
publish how to reach them.

Same command line as pkg_pytorch/blendtorch/btt/apps/launch.py:26-41::

    blendtorch-launch [--out-launch-info launch_info.json] spec.json

``spec.json`` holds :class:`~blendtorch.btt.BlenderLauncher` keyword
arguments, e.g. ``{"script": "tests/blender/launcher.blend.py",
"num_instances": 2, "named_sockets": ["DATA", "GYM"], "background": true,
"bind_addr": "primaryip"}``.  Once the instances run, their addresses and
commands go to the launch-info file -- the hand-over to consumers in other
processes or on other hosts (``LaunchInfo.load_json``) -- and the command
then waits for the instances to exit.
"""
import argparse
import json

from ..launch_info import LaunchInfo
from ..launcher import BlenderLauncher


def _cli():
    p = argparse.ArgumentParser('blendtorch-launch', description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument('--out-launch-info', default='launch_info.json',
                   help='where to write the addresses and commands of the instances')
    p.add_argument('jsonargs', help='JSON file with BlenderLauncher keyword arguments')
    return p


def main(inargs=None):
    opts = _cli().parse_args(inargs)
    with open(opts.jsonargs) as f:
        spec = json.load(f)
    with BlenderLauncher(**spec) as launcher:
        LaunchInfo.save_json(opts.out_launch_info, launcher.launch_info)
        launcher.wait()


if __name__ == '__main__':
    main()
