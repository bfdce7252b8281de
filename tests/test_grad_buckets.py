"""parallel.GradBuckets: persistent flat gradient storage (CPU; the gfx950
kernels writing straight into the buckets are covered in
tests/test_gpu_consumer.py), and the data-parallel CapturedStep on it over
gloo with 2 ranks."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from blendtorch import ops, parallel


def _net():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 4, 2, 1, bias=False), torch.nn.BatchNorm2d(8), torch.nn.LeakyReLU(0.2),
                               torch.nn.Conv2d(8, 4, 3), torch.nn.Flatten(), torch.nn.Linear(4 * 6 * 6, 1))


def test_views_alias_buckets_with_param_strides():
    m = _net().to(memory_format=torch.channels_last)
    gb = parallel.GradBuckets(m.parameters())
    assert gb.attached() and len(gb.buckets) == 1
    base = gb.buckets[0].data_ptr()
    for p in m.parameters():
        assert p.grad is not None and p.grad.stride() == p.stride() and p.grad.shape == p.shape
        off = p.grad.data_ptr() - base
        assert off % 256 == 0 and 0 <= off < gb.buckets[0].numel() * 4
        assert ops.grad_sink(p) is p.grad
    # reverse parameter order: the last layer's gradient is at the front
    assert list(m.parameters())[-1].grad.data_ptr() == base


def test_backward_accumulates_into_buckets_like_plain_autograd():
    a, b = _net(), _net()
    gb = parallel.GradBuckets(a.parameters(), bucket_mb=1e-3)     # tiny: several buckets
    assert len(gb.buckets) > 1
    x1, x2 = torch.randn(2, 3, 16, 16), torch.randn(2, 3, 16, 16)
    for _ in range(2):
        gb.zero_()
        b.zero_grad(set_to_none=True)
        a(x1).sum().backward()
        a(x2).pow(2).sum().backward()        # second backward of the step accumulates
        b(x1).sum().backward()
        b(x2).pow(2).sum().backward()
        for pa, pb in zip(a.parameters(), b.parameters()):
            torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-6, atol=1e-6)
    assert gb.attached()


def test_detached_grads_are_detected():
    m = _net()
    gb = parallel.GradBuckets(m.parameters())
    m.zero_grad(set_to_none=True)
    with pytest.raises(RuntimeError, match='replaced'):
        gb.zero_()
    gb.detach()
    assert ops.grad_sink(next(m.parameters())) is None


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, q, overlap=False):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from blendtorch.parallel.step import CapturedStep
        parallel.init_distributed(backend='gloo')
        m = _net()
        opt = ops.FusedAdam(m.parameters(), lr=1e-2)
        step = CapturedStep(m, opt, lambda mod, x: mod(x).pow(2).mean(), graph=False, overlap=overlap)
        ok_scale = opt.grad_scale == 1.0 / world and step.grads is not None and not step.comm.native
        xs = [torch.randn(4, 3, 16, 16, generator=torch.Generator().manual_seed(10 * r + i))
              for r in range(world) for i in range(3)]
        for i in range(3):
            step(xs[3 * rank + i])
        # reference: single process, full batch of both ranks' data, mean of the per-rank losses
        ref = _net()
        ropt = torch.optim.Adam(ref.parameters(), lr=1e-2)
        for i in range(3):
            ropt.zero_grad()
            loss = sum(ref(xs[3 * r + i]).pow(2).mean() for r in range(world)) / world
            loss.backward()
            ropt.step()
        w = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
        allw = [torch.empty_like(w) for _ in range(world)]
        torch.distributed.all_gather(allw, w)
        ok_sync = all(torch.equal(allw[0], x) for x in allw) and step.collectives == len(step.grads.buckets)
        wr = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
        ok_ref = torch.allclose(w, wr, rtol=1e-4, atol=1e-5)
        q.put((rank, ok_scale, ok_sync, ok_ref))
        torch.distributed.destroy_process_group()
    except Exception as e:  # surface failures to the parent
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize('overlap', [False, True])
def test_bucketed_dp_step_gloo_world2(overlap):
    """CapturedStep on GradBuckets + FusedAdam(grad_scale=1/world): weights
    stay bit-identical across ranks and equal single-process training on the
    union of the ranks' batches -- also with two buckets reduced as soon as
    they are complete (overlap)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q, overlap)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1:] == (True, True, True), r


def test_armed_buckets_reduce_as_soon_as_complete():
    """GradBuckets.arm: a bucket's all-reduce is enqueued the moment the last
    of its gradients is reported written (ops._GRAD_DONE, as the gfx950
    backward kernels do), the rest at finish(); a second contribution into a
    bucket already reduced raises."""
    m = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.Linear(64, 256), torch.nn.Linear(256, 8))
    gb = parallel.GradBuckets(m.parameters(), n_buckets=2)
    assert len(gb.buckets) == 2
    first = {id(p) for p in gb._members[0]}
    # reverse order, 70 % of the bytes: the last two layers
    assert first == {id(p) for p in list(m[2].parameters()) + list(m[1].parameters())}

    class Comm:
        calls = []

        def all_reduce_(self, t, op):
            self.calls.append(t.data_ptr())

    c = Comm()
    gb.zero_()
    gb.arm(c)
    for p in m[2].parameters():
        ops._grad_done(p)
    assert c.calls == []                      # bucket 0 still has m[1]'s gradients to come
    ops._grad_done(m[1].weight)
    ops._grad_done(m[1].bias)
    assert c.calls == [gb.buckets[0].data_ptr()]
    ops._grad_done(m[1].bias)                 # reported twice: no second collective
    assert len(c.calls) == 1
    with pytest.raises(RuntimeError, match='after its bucket'):
        ops._GRAD_LATE(m[2].weight)
    ops._GRAD_LATE(m[0].weight)               # bucket 1 not reduced yet: fine
    assert gb.finish() == 2 and c.calls[1] == gb.buckets[1].data_ptr()
    assert ops._GRAD_DONE is None and ops._GRAD_LATE is None


def test_reduce_claim_stays_off_the_cpu_path():
    """FusedAdam.attach_reduce (the update summing the backward's last weight-
    gradient slice reduce) is a GPU-only handshake: on CPU parameters it does
    not attach, a CapturedStep leaves no claim behind, and flushing with no
    claim is a no-op."""
    m = _net()
    opt = ops.FusedAdam(m.parameters(), lr=1e-3)
    assert opt.attach_reduce() is False
    assert ops._REDUCE_CLAIM is None
    ops._claim_flush()
    from blendtorch.parallel.step import CapturedStep
    st = CapturedStep(m, opt, lambda mm, x: mm(x).pow(2).mean(), graph=False, allreduce=False)
    for _ in range(2):
        st(torch.randn(2, 3, 16, 16))
    assert ops._REDUCE_CLAIM is None
    opt.detach_reduce()
    assert ops._REDUCE_CLAIM is None
