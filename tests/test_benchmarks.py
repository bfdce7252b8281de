"""The reference-harness benchmark (benchmarks/benchmark.py, mirroring the
reference's benchmarks/benchmark.py:7-47) runs end to end on the CPU path, and
the Blender install helpers are well-formed."""
import json
import subprocess
import sys

import pytest

from helpers import ROOT


@pytest.mark.parametrize('scene,producer', [('cube', 'cubesim'), ('falling_cubes', 'cubesim'), ('cube', 'blender')])
def test_reference_harness_cpu(free_port, scene, producer):
    r = subprocess.run([sys.executable, str(ROOT / 'benchmarks' / 'benchmark.py'), '--path', 'cpu', '--scene', scene,
                        '--producer', producer, '--instances', '2', '--workers', '2', '--items', '32', '--sleep', '0',
                        '--start-port', str(free_port), '--json'],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d['shape'] == [8, 480, 640, 3] and d['sec_per_image'] > 0 and d['sec_per_batch'] > 0


def test_install_scripts_parse():
    subprocess.run(['bash', '-n', str(ROOT / 'scripts' / 'install_blender.sh')], check=True)
    subprocess.run([sys.executable, '-m', 'py_compile', str(ROOT / 'scripts' / 'install_btb.py')], check=True)
