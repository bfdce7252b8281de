"""Per-thread CPU of a streaming consumer process, phase by phase: torch idle,
native loader started without producers, streaming, stream paused with the
loader alive, loader stopped.  Finds runtime threads that spin (a thread
whose CPU equals the window length is busy-waiting).  GPU box only."""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / 'pytorch-blender_amd'))
import torch  # noqa: E402
from blendtorch import btt, ops  # noqa: E402
from blendtorch.btt.gpu import DeviceLoader  # noqa: E402


def threads():
    out = {}
    for tid in os.listdir('/proc/self/task'):
        try:
            st = open(f'/proc/self/task/{tid}/stat').read()
        except OSError:
            continue
        rest = st[st.rindex(')') + 2:].split()
        out[int(tid)] = (st[st.index('(') + 1:st.rindex(')')], int(rest[11]) + int(rest[12]))
    return out


def report(label, a, b, secs, worker=None):
    tick = os.sysconf('SC_CLK_TCK')
    busy = sorted(((round((b[t][1] - a.get(t, ('', 0))[1]) / tick, 3),
                    ('worker' if t == worker else b[t][0]) + f':{t - os.getpid()}') for t in b), reverse=True)
    print(json.dumps({'phase': label, 'secs': round(secs, 3), 'nthreads': len(b),
                      'busy': [[n, c] for c, n in busy if c > 0]}), flush=True)


def idle(label, secs=1.0, worker=None):
    a, t = threads(), time.perf_counter()
    time.sleep(secs)
    report(label, a, threads(), time.perf_counter() - t, worker)


def main():
    dev = torch.device('cuda', 0)
    torch.ones(8, device=dev).sum().item()
    idle('torch idle')
    dec = ops.DecodeConfig.unit(channels='rgba', gamma=2.2)
    probe = DeviceLoader(['tcp://127.0.0.1:9'], batch_size=8, device=dev, decode=dec)
    ld = probe._make()
    ld.start()
    time.sleep(0.3)
    idle('loader started, no producer', worker=ld.stats().get('worker_tid'))
    ld.stop()
    idle('loader stopped')
    port = 24000 + os.getpid() % 1000
    with btt.BlenderLauncher(producer='cubesim', num_instances=4, named_sockets=['DATA'], start_port=port,
                             instance_args=[['--mode', 'rgba', '--shm', '64']] * 4) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, device=dev, decode=dec, timeoutms=60000)
        it = iter(dl)
        for _ in range(50):
            next(it)
        torch.cuda.synchronize()
        a, t = threads(), time.perf_counter()
        for _ in range(1000):
            next(it)
        torch.cuda.synchronize()
        wt = dl._live.stats().get('worker_tid')
        report('streaming 1000 batches', a, threads(), time.perf_counter() - t, wt)
        idle('stream paused (loader alive, buffers full)', worker=wt)
        it.close()
        idle('after close')


if __name__ == '__main__':
    main()
