"""Self-launch of N ranks (blendtorch/parallel/launch.py, bench.py --gpus N).

CPU-only: the ranks run a tiny gloo program, so the spawn / relay / exit-code
logic is pinned without a GPU."""
import json
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

from blendtorch.parallel import launch

ROOT = Path(__file__).resolve().parent.parent

RANK_PROG = textwrap.dedent('''
    import json, os, sys
    import torch, torch.distributed as dist
    dist.init_process_group('gloo')
    r, w = dist.get_rank(), dist.get_world_size()
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    info = [None] * w
    dist.all_gather_object(info, {'rank': r, 'local': int(os.environ['LOCAL_RANK'])})
    if r == 0:
        print(json.dumps({'world': w, 'sum': t.item(), 'ranks': info}), flush=True)
    dist.destroy_process_group()
    sys.exit(int(os.environ.get('FAIL_RANK', '-1')) == r and 7 or 0)
''')


def _run_supervisor(tmp_path, world, extra_env=None, timeout_s=None):
    prog = tmp_path / 'rank.py'
    prog.write_text(RANK_PROG)
    sup = textwrap.dedent(f'''
        import sys, os
        sys.path.insert(0, {str(ROOT / 'pytorch-blender_amd')!r})
        from blendtorch.parallel.launch import spawn_ranks
        env = dict(os.environ)
        env.update({extra_env or {}!r})
        codes, rc = spawn_ranks([sys.executable, {str(prog)!r}], {world}, env=env, grace_s=5,
                                timeout_s={timeout_s!r})
        print('CODES', codes, flush=True)
        sys.exit(rc)
    ''')
    return subprocess.run([sys.executable, '-c', sup], capture_output=True, text=True, timeout=180)


def test_rank_env_contract():
    env = launch.rank_env(1, 4, 29500, base={})
    assert env['RANK'] == '1' and env['LOCAL_RANK'] == '1'
    assert env['WORLD_SIZE'] == '4' and env['LOCAL_WORLD_SIZE'] == '4'
    assert env['MASTER_ADDR'] == '127.0.0.1' and env['MASTER_PORT'] == '29500'
    assert env['HSA_ENABLE_IPC_MODE_LEGACY'] == '0'


def test_worst_rc():
    assert launch.worst_rc([0, 0]) == 0
    assert launch.worst_rc([0, 3, 1]) == 3
    assert launch.worst_rc([-15, 0]) == 143
    assert launch.worst_rc([None]) == 1


def test_spawn_two_gloo_ranks_relays_rank0(tmp_path):
    r = _run_supervisor(tmp_path, 2)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1                       # only rank 0 prints, and it reaches the parent's stdout
    out = json.loads(lines[0])
    assert out['world'] == 2 and out['sum'] == 3.0
    assert sorted(x['rank'] for x in out['ranks']) == [0, 1]
    assert sorted(x['local'] for x in out['ranks']) == [0, 1]
    assert 'CODES [0, 0]' in r.stdout


def test_failing_rank_sets_exit_code(tmp_path):
    r = _run_supervisor(tmp_path, 2, extra_env={'FAIL_RANK': '1'})
    assert r.returncode == 7, (r.stdout, r.stderr)


def test_hung_rank_is_stopped(tmp_path):
    prog = tmp_path / 'hang.py'
    prog.write_text('import time\nwhile True: time.sleep(1)\n')
    codes, rc = launch.spawn_ranks([sys.executable, str(prog)], 2, grace_s=2, timeout_s=1.0)
    assert rc == 124
    assert all(c is not None and c != 0 for c in codes)


def test_bench_refuses_missing_gpus():
    """No GPU in this container: --gpus 2 over RCCL must fail loudly, never
    fall back to a single rank."""
    r = subprocess.run([sys.executable, str(ROOT / 'bench.py'), '--gpus', '2', '--steps', '1', '--warmup', '0'],
                       capture_output=True, text=True, timeout=600,
                       env={k: v for k, v in __import__('os').environ.items()
                            if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')})
    assert r.returncode == 3, (r.stdout, r.stderr)
    assert 'needs 2 visible GPUs' in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith('{')]
