"""densityopt (reference: examples/densityopt/densityopt.py:257-331) on the
device-resident iteration (blendtorch.models.densityopt.DensityOptStep):
gating semantics against a direct transcription of the reference rules, and
data parallelism over gloo with 2 ranks (identical ProbModel and
discriminator on both).  The GPU variant (bf16 MFMA discriminator, HIP graph,
RCCL) runs in tests/test_gpu_consumer.py and profiles/r3/."""
import importlib.util
import json
import os
import socket
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _example():
    spec = importlib.util.spec_from_file_location('densityopt_example', ROOT / 'examples' / 'densityopt' /
                                                  'densityopt.py')
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_step_matches_reference_rules_cpu():
    """Eager CPU iterations of DensityOptStep against the reference's host
    logic (D step iff D_real - D_sim < 0.7; S step unless first and not yet
    separated; baseline = first errS mean, then an EMA).  Every other
    iteration runs its real-batch half ahead through prefetch()."""
    from blendtorch.models import Discriminator, ProbModel
    from blendtorch.models.densityopt import DensityOptStep
    import torch.nn as nn
    B = 8
    torch.manual_seed(0)
    netA, netB = Discriminator(), Discriminator()
    netB.load_state_dict(netA.state_dict())
    pmA, pmB = ProbModel([1.2, 3.0], [0.4, 0.4]), ProbModel([1.2, 3.0], [0.4, 0.4])
    g = torch.Generator().manual_seed(1)
    real = torch.rand(B, 3, 64, 64, generator=g) * 2 - 1
    step = DensityOptStep(netA, pmA, real.clone(), B, graph=False)
    step.start()
    optD = torch.optim.Adam(netB.parameters(), lr=5e-5, betas=(0.5, 0.999))
    optS = torch.optim.Adam(pmB.parameters(), lr=5e-2, betas=(0.7, 0.999))
    crit = nn.BCELoss(reduction='none')
    b, first = 0.7, True
    for it in range(6):
        samples = {'m1': step.samples[0].clone(), 'm2': step.samples[1].clone()}
        sim = torch.rand(B, 3, 64, 64, generator=g) * 2 - 1
        sid = torch.randperm(B, generator=g)
        if it % 2:
            step.prefetch()     # the real half enqueued ahead (while producers render): same iteration
        step(sim, sid)
        # reference transcription (densityopt.py:257-316)
        netB.zero_grad()
        out = netB(real)
        crit(out, torch.ones(B)).mean().backward()
        d_real = out.mean().item()
        out = netB(sim)
        crit(out, torch.zeros(B)).mean().backward()
        d_sim = out.mean().item()
        if d_real - d_sim < 0.7:
            optD.step()
        assert float(step.gate_d) == float(d_real - d_sim < 0.7)
        if not first or d_real - d_sim >= 0.7:
            optS.zero_grad()
            with torch.no_grad():
                errS = crit(netB(sim), torch.ones(B))
            loss = pmB.log_prob(samples)[sid] * (errS - b)
            loss.mean().backward()
            optS.step()
            b = errS.mean() if first else 0.9 * errS.mean() + 0.1 * b
            first = False
            assert float(step.gate_s) == 1.0
        else:
            assert float(step.gate_s) == 0.0
        torch.testing.assert_close(step.b.reshape(()), torch.as_tensor(b, dtype=torch.float32).reshape(()),
                                   rtol=1e-5, atol=1e-6)
        for pa, pb in zip(pmA.parameters(), pmB.parameters()):
            torch.testing.assert_close(pa, pb, rtol=1e-4, atol=1e-5)
        for pa, pb in zip(netA.parameters(), netB.parameters()):
            torch.testing.assert_close(pa, pb, rtol=1e-4, atol=1e-5)


@pytest.mark.background
def test_densityopt_example_cpu(free_port, tmp_path):
    """The example runs end to end on the CPU path and writes the reference's
    outputs (densityopt.py:321-331, 350-354): the parameter history as text,
    one row per epoch plus the target as the last row, and image grids of
    the target and simulated batch every 5 epochs."""
    import numpy as np
    from blendtorch.utils.images import read_png
    mod = _example()
    res = mod.main(['--device', 'cpu', '--num-epochs', '5', '--instances', '2', '--batch', '16',
                    '--start-port', str(free_port), '--out-dir', str(tmp_path), '--steady-skip', '1'])
    assert res['iterations'] == 6 and res['world'] == 1 and res['dtype'] == 'fp32'
    assert all(d == d for d in res['abs_diff'])           # finite
    # the reference passes its note as savetxt's comments= (the header's
    # prefix, not a comment line): mirrored byte for byte, so skip that line
    hist = np.loadtxt(res['history_file'], skiprows=1)
    assert hist.shape == (7, 4) and res['history_rows'] == 7
    np.testing.assert_allclose(hist[-1], res['target'], rtol=1e-6)
    np.testing.assert_allclose(hist[-2], res['final_params'], rtol=1e-5)
    head = Path(res['history_file']).read_text().splitlines()
    assert head[0] == 'last entry corresponds to target paramsmu_m1, mu_m2, std_m1, std_m2'
    # 16 images of 64x64 in rows of 8 with 2-pixel padding: 2 x 8 tiles
    for name in ('real_005.png', 'sim_samples_005.png'):
        img = read_png(tmp_path / name)
        assert img.shape == (2 * 66 + 2, 8 * 66 + 2, 3) and img.max() > img.min()
    st = res['steady']
    assert st['iterations'] >= 1 and st['iterations_per_s'] > 0
    assert set(st['ms_per_iteration']) >= {'sim_wait', 'step_enqueue', 'fetch', 'send'}


def _rank(rank, world, port, prod_port, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        mod = _example()
        res = mod.main(['--device', 'cpu', '--backend', 'gloo', '--num-epochs', '3', '--instances', '2',
                        '--batch', '8', '--start-port', str(prod_port), '--seed', str(rank), '--out-dir', ''])
        Path(out).write_text(json.dumps(res))
    except Exception:
        import traceback
        Path(out).write_text(json.dumps({'error': traceback.format_exc()}))


@pytest.mark.background
def test_densityopt_data_parallel_gloo_world2(tmp_path):
    """2 ranks, each with its own producers; rank 0's samples are broadcast,
    gradients / gate statistics averaged: ProbModel and discriminator end
    bit-identical on both ranks (different seeds would diverge them)."""
    ctx = mp.get_context('spawn')
    port = _free_port()
    prod = 38000 + (os.getpid() % 400) * 10
    outs = [tmp_path / f'r{r}.json' for r in range(2)]
    procs = [ctx.Process(target=_rank, args=(r, 2, port, prod, str(outs[r]))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    res = [json.loads(o.read_text()) for o in outs]
    for r in res:
        assert 'error' not in r, r.get('error')
    assert res[0]['world'] == 2 and res[0]['collectives'] == 'gloo'
    assert res[0]['weights_sha'] == res[1]['weights_sha']
    assert res[0]['final_params'] == res[1]['final_params']
    assert res[0]['d_steps'] == res[1]['d_steps'] and res[0]['s_steps'] == res[1]['s_steps']


def test_sstep_reference_matches_probmodel_autograd_cpu():
    """The fused S step's closed-form gradient (models.densityopt.sstep_reference:
    the arithmetic of csrc/gpu/dopt.hip's dopt_sstep_kernel) against autograd
    through the PyTorch ProbModel on the reference's loss
    ``(log_probs[shape_id] * (errS - b)).mean()`` (densityopt.py:290-300),
    including out-of-order shape ids and saturated probabilities (the BCE's
    -100 clamp)."""
    from blendtorch.models import ProbModel
    from blendtorch.models.densityopt import sstep_reference
    g = torch.Generator().manual_seed(3)
    B, N = 16, 48
    pm = ProbModel([1.2, 3.0], [0.4, 0.3])
    with torch.no_grad():
        pm.m1m2_mean.add_(torch.randn(2, generator=g) * 0.1)
    torch.manual_seed(5)
    s = pm.sample(N)
    samples = torch.stack([s['m1'], s['m2']])
    sid = torch.randperm(N, generator=g)[:B]
    logit = torch.randn(B, generator=g) * 3
    logit[0] = -200.0                                  # log(sigmoid) below -100: clamped
    b = 0.55
    out = sstep_reference(logit, sid, samples, pm.m1m2_mean.detach(), pm.m1m2_log_std.detach(), b)
    p = torch.sigmoid(logit)
    err = torch.nn.functional.binary_cross_entropy(p, torch.ones_like(p), reduction='none')
    log_probs = pm.log_prob({'m1': samples[0], 'm2': samples[1]})
    loss = (log_probs[sid] * (err - b)).mean()
    loss.backward()
    torch.testing.assert_close(out[0], err.mean(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(out[1:3], pm.m1m2_mean.grad, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(out[3:5], pm.m1m2_log_std.grad, rtol=1e-5, atol=1e-6)
