"""Host-side cost of the HIP calls a stream loader makes per batch (event
record, cross-stream wait, pinned H2D copy), alone and interleaved, while the
GPU is busy with a long-running kernel sequence.  Prints one JSON line.

    python scripts/hip_api_cost.py
"""
import json
import time

import torch


def per_call(fn, n=200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    dev = torch.device('cuda', 0)
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    side2 = torch.cuda.Stream()
    src = torch.empty(1228800, dtype=torch.uint8).pin_memory()
    dst = torch.empty(1228800, dtype=torch.uint8, device=dev)
    busy = torch.randn(4096, 4096, device=dev)
    out = {}
    done = torch.cuda.Event()
    done.record()
    torch.cuda.synchronize()

    def keep_busy():   # ~ms of queued GEMMs so every call below finds the GPU busy
        for _ in range(20):
            busy.matmul(busy)

    keep_busy()
    out['event_record_us'] = per_call(lambda: torch.cuda.Event().record())
    keep_busy()
    out['wait_completed_event_us'] = per_call(lambda: side.wait_event(done))
    keep_busy()

    def wait_fresh():
        e = torch.cuda.Event()
        e.record(main_s)
        side2.wait_event(e)
    out['record_plus_cross_wait_us'] = per_call(wait_fresh)
    torch.cuda.synchronize()
    keep_busy()

    def copy():
        with torch.cuda.stream(side):
            dst.copy_(src, non_blocking=True)
    out['h2d_copy_1_2MB_us'] = per_call(copy, 100)
    torch.cuda.synchronize()
    keep_busy()

    def wait_then_copy():
        e = torch.cuda.Event()
        e.record(main_s)
        with torch.cuda.stream(side):
            torch.cuda.current_stream().wait_event(e)
            dst.copy_(src, non_blocking=True)
    out['record_wait_copy_us'] = per_call(wait_then_copy, 100)
    torch.cuda.synchronize()
    keep_busy()

    def wait_old_then_copy():
        with torch.cuda.stream(side):
            torch.cuda.current_stream().wait_event(done)
            dst.copy_(src, non_blocking=True)
    out['wait_completed_then_copy_us'] = per_call(wait_old_then_copy, 100)
    torch.cuda.synchronize()
    out['query_completed_event_us'] = per_call(lambda: done.query())
    print(json.dumps({k: round(v, 2) for k, v in out.items()}), flush=True)


if __name__ == '__main__':
    main()
