"""Install the Blender-side package (``blendtorch.btb``) into Blender's Python.

Run ONCE through Blender:

    blender --background --python scripts/install_btb.py [-- --no-native] [-- --no-pyzmq]

Same job as the reference's ``scripts/install_btb.py:22-43`` (ensurepip, then
an editable pip install of the Blender package into Blender's bundled
interpreter), adapted to this repository:

* the interpreter is ``sys.executable`` -- ``bpy.app.binary_path_python`` (used
  by the reference, ``install_btb.py:23,34``) was removed in Blender 2.91;
* one package (``pytorch-blender_amd``) carries both ``btb`` and ``btt``; the
  Blender side imports only ``blendtorch.btb`` (+ the transport);
* the native ZMTP transport (``blendtorch/_native*.so``) is a CPython extension,
  so it is rebuilt for Blender's Python version (needs ``g++`` and pybind11,
  installed here with pip); without it, ``btb`` uses pyzmq
  (``BLENDTORCH_TRANSPORT=pyzmq``), which this script also tries to install.
  Both speak the same ZMTP/3.0 wire protocol as the PyTorch side.
"""
import subprocess
import sys
from pathlib import Path

THISDIR = Path(__file__).resolve().parent
PKG = THISDIR.parent / 'pytorch-blender_amd'


def run(cmd, check=True):
    print('+', ' '.join(str(c) for c in cmd), flush=True)
    try:
        out = subprocess.check_output([str(c) for c in cmd], stderr=subprocess.STDOUT)
        print(out.decode(errors='replace'))
        return True
    except subprocess.CalledProcessError as e:
        print(e.output.decode(errors='replace'))
        if check:
            sys.exit(1)
        return False


def pip(*args, check=True):
    return run([sys.executable, '-m', 'pip', 'install', '--upgrade', '--user', *args], check=check)


def main(argv):
    no_native = '--no-native' in argv
    no_pyzmq = '--no-pyzmq' in argv
    run([sys.executable, '-m', 'ensurepip', '--upgrade', '--user'], check=False)
    pip('numpy')
    pip('-e', str(PKG), '--no-deps')
    if not no_pyzmq:
        pip('pyzmq', check=False)
    if not no_native:
        pip('pybind11', check=False)
        # C++ transport for this interpreter; the HIP extension is PyTorch-side only
        run([sys.executable, '-m', 'blendtorch._build', '--no-hip'], check=False)
    run([sys.executable, '-c', 'import blendtorch.btb as btb; print("blendtorch.btb", btb.__version__)'])


if __name__ == '__main__':
    argv = sys.argv[sys.argv.index('--') + 1:] if '--' in sys.argv else []
    main(argv)
