"""Per-kernel floor on the device: N tiny kernels back to back, eager and in
one HIP graph (device time per kernel from events around graph replays).

    python scripts/launch_floor.py
"""
import json
import torch

dev = torch.device('cuda', 0)
x = torch.zeros(1, device=dev)
big = torch.zeros(8 << 20, device=dev)   # 32 MB


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


out = {}
N = 200
out['eager_tiny_us'] = timed(lambda: [x.add_(1) for _ in range(N)]) / N
mid = torch.zeros(1 << 20, device=dev)   # 4 MB


def pair():
    mid.add_(1)
    x.add_(1)


for name, op in (('tiny', lambda: x.add_(1)), ('32MB', lambda: big.add_(1)), ('4MB', lambda: mid.add_(1)),
                 ('4MB+tiny', pair)):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(N):
            op()
    out[f'graph_{name}_us'] = timed(g.replay) / N
print(json.dumps({k: round(v, 3) for k, v in out.items()}))
