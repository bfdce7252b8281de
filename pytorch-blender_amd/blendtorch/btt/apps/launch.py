"""``blendtorch-launch``: launch producer instances from a JSON spec.

Reference: pkg_pytorch/blendtorch/btt/apps/launch.py:26-41.  The JSON file
holds ``BlenderLauncher`` keyword arguments, e.g.::

    {"scene": "", "script": "tests/blender/launcher.blend.py",
     "num_instances": 2, "named_sockets": ["DATA", "GYM"],
     "background": true, "seed": 10}

The launcher starts the instances, writes the LaunchInfo (addresses and
commands) to ``--out-launch-info`` so other processes or hosts can connect,
and waits for the instances to exit.
"""
import argparse
import json

from ..launch_info import LaunchInfo
from ..launcher import BlenderLauncher


def main(inargs=None):
    parser = argparse.ArgumentParser('Blender Launcher', description=__doc__,
                                     formatter_class=argparse.RawTextHelpFormatter)
    parser.add_argument('--out-launch-info', help='Path to save connection info to.', default='launch_info.json')
    parser.add_argument('jsonargs', type=str, help='JSON Dict of arguments for blendtorch.btt.BlenderLauncher')
    args = parser.parse_args(inargs)
    with open(args.jsonargs, 'r') as fp:
        launch_args = json.load(fp)
    with BlenderLauncher(**launch_args) as bl:
        LaunchInfo.save_json(args.out_launch_info, bl.launch_info)
        bl.wait()


if __name__ == '__main__':
    main()
