"""Locate a usable Blender executable.

Reference: pkg_pytorch/blendtorch/btt/finder.py:16-71.  The binary is looked
up on PATH (optionally extended), its ``--version`` banner parsed with
``Blender X.Y``, and a probe script that imports the message transport is run
in the background with ``--python-exit-code 255`` to check that blendtorch's
Blender-side requirements are importable.
"""
import logging
import os
import re
import shutil
import subprocess
import tempfile
from pathlib import Path

logger = logging.getLogger('blendtorch')

_VERSION_RE = re.compile(r'Blender\s(\d+)\.(\d+)', re.IGNORECASE)

# Blender ships its own Python; the probe checks that a ZMTP transport is
# importable there (real pyzmq, or blendtorch's native engine).
_PROBE = r'''
try:
    import zmq  # noqa: F401
except ImportError:
    from blendtorch.transport import zmq  # noqa: F401
'''


def discover_blender(additional_blender_paths=None):
    """Return ``{'path', 'major', 'minor'}`` for a working Blender, else None."""
    env = os.environ.copy()
    if additional_blender_paths is not None:
        env['PATH'] = str(additional_blender_paths) + os.pathsep + env.get('PATH', '')
    found = shutil.which('blender', path=env['PATH'])
    if found is None:
        logger.warning('Could not find Blender.')
        return None
    bpath = Path(found).resolve()
    logger.debug(f'Discovered Blender in {bpath}')

    try:
        r = subprocess.run([str(bpath), '--version'], capture_output=True, env=env, timeout=120)
    except (OSError, subprocess.TimeoutExpired):
        logger.warning('Failed to run Blender --version.')
        return None
    m = _VERSION_RE.search(r.stdout.decode(errors='replace'))
    if r.returncode != 0 or m is None:
        logger.warning('Failed to parse Blender version.')
        return None

    with tempfile.NamedTemporaryFile('w', suffix='.py', delete=False) as fp:
        fp.write(_PROBE)
    try:
        r = subprocess.run([str(bpath), '--background', '--python-use-system-env', '--python-exit-code', '255',
                            '--python', fp.name], capture_output=True, env=env, timeout=300)
    except (OSError, subprocess.TimeoutExpired):
        r = None
    finally:
        os.remove(fp.name)
    if r is None or r.returncode != 0:
        logger.warning('Failed to run minimal Blender script; ensure Python requirements are installed.')
        return None
    return {'path': bpath, 'major': int(m[1]), 'minor': int(m[2])}


def _main():
    print(discover_blender())


if __name__ == '__main__':
    _main()
