"""Child process of tests/test_gpu_consumer.py::test_rccl_direct_one_rank_process_group:
a 1-rank RCCL process group exercising parallel.DeviceComm (direct RCCL on the
compute stream) and the graphed data-parallel step.  Writes JSON to argv[1]."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / 'pytorch-blender_amd'))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from blendtorch import ops  # noqa: E402
from blendtorch.models import Discriminator  # noqa: E402
from blendtorch.parallel import DeviceComm  # noqa: E402
from blendtorch.parallel.step import CapturedStep  # noqa: E402


def main(path):
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', device_id=dev)
    comm = DeviceComm()
    res = {'native': comm.native, 'selfcheck': comm.selfcheck(nbytes=1 << 16, timeout_s=60)}
    t = torch.arange(1000, dtype=torch.float32, device=dev)
    comm.all_reduce_(t, 'avg')
    res['allreduce_avg_ok'] = bool(torch.equal(t, torch.arange(1000, dtype=torch.float32, device=dev)))
    b = torch.arange(77, dtype=torch.int64, device=dev)
    comm.broadcast_(b, 0)
    res['broadcast_ok'] = bool(torch.equal(b, torch.arange(77, device=dev)))
    src = torch.randint(0, 255, (3, 17), dtype=torch.uint8, device=dev)
    dst = torch.zeros_like(src)
    comm.p2p([(True, src, 0), (False, dst, 0)])
    torch.cuda.synchronize()
    res['p2p_self_ok'] = bool(torch.equal(src, dst))

    g = torch.Generator(device=dev).manual_seed(3)
    xs = [torch.rand(4, 4, 96, 128, device=dev, generator=g).to(torch.bfloat16)
          .contiguous(memory_format=torch.channels_last) for _ in range(5)]
    nets = []
    for pg in (False, True, 'overlap'):
        torch.manual_seed(0)
        m = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
        opt = ops.FusedAdam(m.parameters(), lr=2e-4)
        step = CapturedStep(m, opt, lambda mod, x: mod.bce_loss_bf16(x, 1.0), warmup=2,
                            allreduce='always' if pg else False, comm=comm if pg else None, overlap=pg == 'overlap')
        w0 = ops.KERNEL_CALLS.get('conv_wgrad', 0)
        for x in xs:
            step(x)
        torch.cuda.synchronize()
        nets.append(m)
        if pg is True:
            res['collectives'] = step.collectives
            res['state'] = step.state
            res['error'] = step.error
        elif pg == 'overlap':
            # (bucket, weight-gradient launches before its all-reduce) of the captured step
            res['overlap'] = {'collectives': step.collectives, 'state': step.state, 'error': step.error,
                              'order': [(i, n - w0) for i, n in step.grads.order],
                              'first_bucket_params': len(step.grads._members[0]),
                              'max_abs_diff': max(float((p - q).abs().max())
                                                  for p, q in zip(nets[0].parameters(), m.parameters()))}
    res['max_abs_diff'] = max(float((p - q).abs().max()) for p, q in zip(nets[0].parameters(), nets[1].parameters()))
    d = torch.cat([(p - q).detach().abs().flatten() for p, q in zip(nets[0].parameters(), nets[1].parameters())])
    res['mean_abs_diff'] = float(d.mean())
    res['frac_above_half_lr'] = float((d > 1e-4).float().mean())
    Path(path).write_text(json.dumps(res))
    dist.destroy_process_group()


if __name__ == '__main__':
    main(sys.argv[1])
