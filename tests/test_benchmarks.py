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


def test_sweep_rows_carry_reference_and_producers(monkeypatch, capsys):
    """benchmarks/sweep.py: one JSON row per (mode, producer count) with the
    matching reference row (Readme.md:88-93) and the producer caveat."""
    import importlib.util
    import json
    from helpers import ROOT
    spec = importlib.util.spec_from_file_location('sweep', ROOT / 'benchmarks' / 'sweep.py')
    sweep = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sweep)

    def fake(mode, n, steps, warmup, extra):
        return {'producer': 'cubesim (stand-in)', 'config': {'cpus_per_gpu': 16}, 'n_gpus': 1,
                'value': 1000.0 * n, 'sec_per_image': 1 / (1000.0 * n), 'sec_per_batch': 8 / (1000.0 * n),
                'steps': steps}
    monkeypatch.setattr(sweep, 'run_row', fake)
    sweep.main(['--producers', '1,5,8', '--modes', 'rgb,rgba', '--steps', '3'])
    rows = [json.loads(l) for l in capsys.readouterr().out.splitlines()]
    assert [(r['mode'], r['producers']) for r in rows] == [('rgb', 1), ('rgb', 5), ('rgb', 8),
                                                          ('rgba', 1), ('rgba', 5), ('rgba', 8)]
    r5 = rows[1]
    assert r5['reference_row']['sec_per_image'] == 0.011 and r5['reference_row']['note'] == 'no UI refresh'
    assert r5['ratio_vs_reference_row'] == round(0.011 * 5000, 1)
    assert rows[2]['reference_row'] is None and rows[0]['cpus'] == 16 and 'stand-in' in rows[0]['producer']


def test_bench_cli_fleet_and_jitter_flags():
    """bench.py's mixed-fleet and colour-jitter switches parse (the GPU runs
    are in profiles/r6/), and the loader gives every TCP pipe its own receive
    thread while ipc:// loaders keep at most 4."""
    import importlib.util
    from helpers import ROOT
    spec = importlib.util.spec_from_file_location('bench_cli', ROOT / 'bench.py')
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    a = mod.parse_args(['--producers', '6', '--inline-producers', '3', '--color-jitter'])
    assert a.inline_producers == 3 and a.color_jitter and a.shm > 0
    from blendtorch.btt.gpu import _default_io_threads
    assert _default_io_threads(['ipc:///tmp/a'] * 8) == 4
    assert _default_io_threads(['ipc:///tmp/a']) == 1
    import os
    cpus = len(os.sched_getaffinity(0))
    assert _default_io_threads(['tcp://127.0.0.1:5000'] * 8) == min(8, max(4, cpus - 2))
