"""Instance arguments handed to producer scripts by ``btt.BlenderLauncher``.

Reference: pkg_blender/blendtorch/btb/arguments.py:5-47.  Everything after
the ``--`` separator of Blender's command line belongs to the script;
``-btid``, ``-btseed`` and ``-btsockets NAME=ADDRESS ...`` are consumed here
and the rest is returned for the script's own argparse.
"""
import argparse
import sys


def _name_address(text):
    name, sep, addr = text.partition('=')
    if not sep:
        raise argparse.ArgumentTypeError(f'expected NAME=ADDRESS, got {text!r}')
    return name, addr


def parse_blendtorch_args(argv=None):
    """Return ``(args, remainder)``; ``args.btsockets`` is a name->address dict.

    Raises ValueError when the command line has no ``--`` separator.
    """
    argv = argv or sys.argv
    if '--' not in argv:
        raise ValueError('No script arguments found; missing `--`?')
    argv = argv[argv.index('--') + 1:]
    parser = argparse.ArgumentParser()
    parser.add_argument('-btid', type=int, help='Identifier for this Blender instance')
    parser.add_argument('-btseed', type=int, help='Random number seed')
    parser.add_argument('-btsockets', metavar='NAME=ADDRESS', nargs='*', type=_name_address,
                        help='Set a number of named address pairs.')
    args, remainder = parser.parse_known_args(argv)
    args.btsockets = dict(args.btsockets or [])
    return args, remainder
