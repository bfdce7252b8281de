#!/usr/bin/env python
"""The reference's published table, row by row, as JSON lines.

The reference reports sec/image and sec/batch for 1, 2, 4 and 5 Blender
instances on the 640x480 Cube scene, batch 8 (Readme.md:86-93).
This sweep runs ``bench.py`` once per (frame format, producer count) and
prints one JSON line per row with the producer count, the CPU cores the job
may use, the matching reference row and the ratio -- for RGB (what the
reference's cube.blend.py actually renders) and RGBA (what its README says).

    python benchmarks/sweep.py [--producers 1,2,4,5,8] [--modes rgba,rgb]
                               [--steps 2000] [--warmup 50] [--out rows.jsonl]

Every row's producers are ``cubesim`` (the C++ stand-in for Blender/Eevee),
so a ratio against the reference row compares whole pipelines -- rendering
included -- not the streaming framework alone (``bench.py`` says the same in
its ``baseline_note``).
"""
import argparse
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

# reference rows (Readme.md:88-93): instances -> (sec/batch, sec/image, note)
REFERENCE = {
    1: (0.236, 0.030, 'UI refresh'),
    2: (0.14, 0.018, 'UI refresh'),
    4: (0.099, 0.012, 'UI refresh'),
    5: (0.085, 0.011, 'no UI refresh'),
}


def run_row(mode, producers, steps, warmup, extra):
    cmd = [sys.executable, str(ROOT / 'bench.py'), '--mode', mode, '--producers', str(producers),
           '--steps', str(steps), '--warmup', str(warmup)] + list(extra)
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    if r.returncode != 0 or not lines:
        raise RuntimeError(f'{" ".join(cmd)} failed (rc {r.returncode}):\n{r.stderr[-2000:]}')
    return json.loads(lines[-1])


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument('--producers', default='1,2,4,5,8')
    ap.add_argument('--modes', default='rgba,rgb')
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--warmup', type=int, default=50)
    ap.add_argument('--out', default=None, help='also append the rows to this file')
    a, extra = ap.parse_known_args(argv)
    for mode in a.modes.split(','):
        for n in (int(x) for x in a.producers.split(',')):
            d = run_row(mode, n, a.steps, a.warmup, extra)
            ref = REFERENCE.get(n)
            row = {
                'metric': 'images/sec per producer-count row, 640x480 Cube scene, batch=8',
                'mode': mode,
                'producers': n,
                'producer': d.get('producer'),
                'cpus': d['config'].get('cpus_per_gpu'),
                'n_gpus': d['n_gpus'],
                'images_per_s': d['value'],
                'sec_per_image': d['sec_per_image'],
                'sec_per_batch': d['sec_per_batch'],
                'reference_row': ({'instances': n, 'sec_per_batch': ref[0], 'sec_per_image': ref[1],
                                   'images_per_s': round(1 / ref[1], 1), 'note': ref[2]} if ref else None),
                'ratio_vs_reference_row': round(ref[1] / d['sec_per_image'], 1) if ref else None,
                'h2d_gbytes_per_s': d.get('h2d_gbytes_per_s'),
                'producer_frames_per_s': d.get('producer_frames_per_s'),
                'steps': d['steps'],
            }
            line = json.dumps(row)
            print(line, flush=True)
            if a.out:
                with open(a.out, 'a') as f:
                    f.write(line + '\n')


if __name__ == '__main__':
    main()
