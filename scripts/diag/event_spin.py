"""Which HIP usage pattern keeps a runtime thread busy: each phase repeats one
pattern for ~0.4 s on cuda:0 and reports the per-thread CPU (see
threads_cpu.py).  GPU box only."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import torch  # noqa: E402
from threads_cpu import threads, report  # noqa: E402

dev = torch.device('cuda', 0)
a = torch.ones(1 << 20, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
torch.cuda.synchronize()


def phase(label, body, secs=0.4):
    t0 = time.perf_counter()
    th0 = threads()
    n = 0
    while time.perf_counter() - t0 < secs:
        body()
        n += 1
    torch.cuda.synchronize()
    report(f'{label} (x{n})', th0, threads(), time.perf_counter() - t0)


def kernels():
    with torch.cuda.stream(s1):
        a.add_(1.0)
    time.sleep(50e-6)


def ev_destroy_pending():
    with torch.cuda.stream(s1):
        a.add_(1.0)
        e = torch.cuda.Event()
        e.record(s1)
    del e
    time.sleep(50e-6)


evs = [torch.cuda.Event() for _ in range(64)]
k = [0]


def ev_reuse():
    with torch.cuda.stream(s1):
        a.add_(1.0)
        evs[k[0] % 64].record(s1)
    k[0] += 1
    time.sleep(50e-6)


def ev_wait_cross():
    with torch.cuda.stream(s1):
        a.add_(1.0)
        e = evs[k[0] % 64]
        e.record(s1)
    s2.wait_event(e)
    with torch.cuda.stream(s2):
        a.mul_(1.0)
    k[0] += 1
    time.sleep(50e-6)


def ev_query():
    with torch.cuda.stream(s1):
        a.add_(1.0)
        e = evs[k[0] % 64]
        e.record(s1)
    while not e.query():
        time.sleep(10e-6)
    k[0] += 1


def idle():
    time.sleep(1e-3)


# a captured graph of 20 small kernels, replayed like the disc consumer's step
gs = torch.cuda.Stream(dev)
gs.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(gs):
    for _ in range(3):
        for _ in range(20):
            a.add_(1.0)
torch.cuda.current_stream().wait_stream(gs)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    for _ in range(20):
        a.add_(1.0)


def graph_replay():
    graph.replay()
    time.sleep(200e-6)


def graph_replay_sync():
    graph.replay()
    torch.cuda.current_stream().synchronize()


for label, body in [('idle', idle), ('kernels', kernels), ('event record+destroy while pending', ev_destroy_pending),
                    ('event reuse', ev_reuse), ('cross-stream wait', ev_wait_cross), ('event query poll', ev_query),
                    ('graph replay', graph_replay), ('graph replay + stream sync', graph_replay_sync),
                    ('idle again', idle)]:
    phase(label, body)
