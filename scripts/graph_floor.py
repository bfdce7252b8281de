"""Per-kernel cost inside one HIP graph: a serial chain vs the same kernels
split over parallel branches (fork/join captured from side streams).

    python scripts/graph_floor.py [--n 240]

Prints one JSON line: device time per kernel (events around graph replays)
for tiny (1-element), 4 MB and 32 MB elementwise kernels, serial and over
2 / 4 branches.  The serial tiny number is the floor a consumer step pays
per kernel; the branch numbers say how much of it parallel graph branches
hide.
"""
import argparse
import json

import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


def capture(ops_per_branch, branches):
    """One graph: ``branches`` parallel chains, chain b running ops_per_branch[b]."""
    main = torch.cuda.Stream()
    side = [torch.cuda.Stream() for _ in range(branches)]
    main.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=main):
        for s in side:
            s.wait_stream(main)
        for s, ops in zip(side, ops_per_branch):
            with torch.cuda.stream(s):
                for op in ops:
                    op()
        for s in side:
            main.wait_stream(s)
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=240)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    N = a.n
    out = {'n_kernels': N}
    sizes = {'tiny': 1, '4MB': 1 << 20, '32MB': 8 << 20}
    for name, numel in sizes.items():
        for br in (1, 2, 4):
            bufs = [torch.zeros(numel, device=dev) for _ in range(br)]
            ops = [[(lambda t=bufs[b]: t.add_(1)) for _ in range(N // br)] for b in range(br)]
            g = capture(ops, br)
            out[f'{name}_b{br}_us_per_kernel'] = round(timed(g.replay) / N, 3)
            del g
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
