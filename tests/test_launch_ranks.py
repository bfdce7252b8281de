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
    if int(os.environ.get('FAIL_RANK', '-1')) == r:
        print(f'rank {r} says: simulated RCCL failure', file=sys.stderr, flush=True)
        sys.exit(7)
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
    # the supervisor names the failed rank and repeats the tail of its stderr
    assert '[launch] rank 1 exited with 7 [failed first]' in r.stderr, r.stderr
    assert '[launch]   rank 1| rank 1 says: simulated RCCL failure' in r.stderr


def test_failure_report_format():
    text = launch.failure_report([0, -15, 3], [['ok'], ['stopped'], ['Traceback', 'RuntimeError: boom']], first=2)
    assert 'rank 0' not in text
    assert 'rank 1 exited with -15 (signal 15)' in text
    assert 'rank 2 exited with 3 [failed first]' in text and 'rank 2| RuntimeError: boom' in text


@pytest.mark.parametrize('mode', ['shard', 'pool', 'scatter'])
def test_eight_rank_resource_plan_small_node(tmp_path, mode):
    """8 ranks on a node whose cgroup allows 16 CPUs (of 256 visible) and a
    256 MiB /dev/shm: every rank gets >= 1 producer, disjoint CPU slices and
    port blocks, and the rings of all ranks fit /dev/shm together."""
    from blendtorch.parallel import plan_rank_resources
    allowed = list(range(256))
    frame = 640 * 480 * 4
    shm_free = 256 << 20
    plans = [plan_rank_resources(r, r, 8, 8, allowed, budget=16, pin=False, dist_mode=mode, shm_slots=48,
                                 shm_free_bytes=shm_free, frame_bytes=frame, bus_ids=[None] * 8, sysfs=tmp_path)
             for r in range(8)]
    assert all(p['producers'] >= 1 for p in plans)
    if mode == 'scatter':
        assert sum(p['producers'] for p in plans) >= 8
    blocks = [range(p['start_port'], p['start_port'] + p['port_span']) for p in plans]
    for i in range(8):
        for j in range(i + 1, 8):
            assert not set(blocks[i]) & set(blocks[j]), (i, j)
    for i in range(8):
        for j in range(i + 1, 8):
            assert not set(plans[i]['cpus']) & set(plans[j]['cpus'])
    used = sum(p['producers'] * p['shm_slots'] * frame for p in plans)
    assert used <= shm_free
    assert all(p['shm_slots'] == 0 or p['shm_slots'] >= 8 for p in plans)
    # a roomy /dev/shm keeps the requested ring depth
    big = plan_rank_resources(0, 0, 8, 8, allowed, 16, False, dist_mode=mode, shm_slots=48,
                              shm_free_bytes=64 << 30, frame_bytes=frame, bus_ids=[None] * 8, sysfs=tmp_path)
    assert big['shm_slots'] == 48


def test_eight_rank_plan_pinned_quota():
    """Pinned producers (the quota covers most of the affinity mask): every
    producer gets one core of its own rank's slice."""
    from blendtorch.parallel import plan_rank_resources
    from blendtorch.parallel.topology import producers_for_share
    plans = [plan_rank_resources(r, r, 8, 8, list(range(64)), budget=64, pin=True, bus_ids=[None] * 8,
                                 sysfs=Path('/nonexistent')) for r in range(8)]
    for p in plans:
        # 8 CPUs per rank: the link, not the CPU, is the bound (producers_for_share)
        assert p['producers'] == producers_for_share(8) and all(len(a) == 1 and a[0] in p['cpus']
                                                                for a in p['affinity'])


def test_eight_ranks_under_16_cpu_quota_get_cost_justified_producers(tmp_path):
    """8 ranks under a 16-CPU quota (2 CPUs each): at the measured costs of
    ~65 us of producer CPU and ~20 us of consumer-process CPU per frame
    (profiles/r4/cpu_per_frame.md) a rank sustains 2e6 / 85 = 23.5k
    frames/s, for which its producers need 1.53 cores: 2 producers each (the
    round-2 ``share - 3`` rule gave 1, i.e. ~12k frames/s per rank).  One
    rank with all 16 CPUs is link-bound (42k RGBA frames/s need 2.7
    producer cores): 5 with the 1.5x margin."""
    from blendtorch.parallel import plan_rank_resources
    from blendtorch.parallel.topology import producers_for_share, CONSUMER_US_PER_FRAME, PRODUCER_US_PER_FRAME
    frame = 640 * 480 * 4
    plans = [plan_rank_resources(r, r, 8, 8, list(range(256)), budget=16, pin=False, shm_slots=48,
                                 shm_free_bytes=64 << 30, frame_bytes=frame, bus_ids=[None] * 8, sysfs=tmp_path)
             for r in range(8)]
    rate = 2 * 1e6 / (PRODUCER_US_PER_FRAME + CONSUMER_US_PER_FRAME)
    want = -(-rate * PRODUCER_US_PER_FRAME / 1e6 // 1)
    assert want == 2 and all(p['producers'] == want for p in plans)
    one = plan_rank_resources(0, 0, 1, 1, list(range(16)), budget=16, pin=True, shm_slots=48,
                              shm_free_bytes=64 << 30, frame_bytes=frame, bus_ids=[None], sysfs=tmp_path)
    assert one['producers'] == 5
    # more CPU per frame in the consumer leaves fewer cores to producers
    assert producers_for_share(2, frame, consumer_us=150.0) == 1
    # the costs follow the frame size: exact at the headline frame, per-message
    # part fixed (a 4x larger frame needs more producer cores on the same share)
    from blendtorch.parallel.topology import frame_costs_us
    assert frame_costs_us(frame) == (PRODUCER_US_PER_FRAME, CONSUMER_US_PER_FRAME)
    big, small = frame_costs_us(4 * frame), frame_costs_us(64 * 64 * 3)
    assert big[0] > 3 * PRODUCER_US_PER_FRAME and 10.0 <= small[0] < 11.0
    # 4 CPUs, 4x frames: link-bound at 10.5k frames/s x 230 us = 2.4 cores, x1.5 -> 4
    assert producers_for_share(4, 4 * frame) == 4


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
