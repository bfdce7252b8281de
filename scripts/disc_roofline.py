"""Per-kernel roofline of one disc consumer step (bench.py --consumer disc:
DCGAN discriminator on 8 x 480 x 640 RGBA frames, bf16 NHWC, ndf 32).

Inputs:
  * a kernel trace summary (scripts/step_sequence.py output): kernel names and
    mean durations per position of the graphed step;
  * rocprofv3 --pmc CSV passes of the eager step (scripts/gpurun/
    disc_roofline.sh): counters per dispatch, matched to step positions in
    dispatch order (one step = the position sequence of the trace).

Per position it prints: analytic FLOPs and minimum HBM bytes (every operand
read once, every output written once), measured FETCH_SIZE / WRITE_SIZE per
DISPATCH (KB counters -> MB; FETCH_SIZE doubled, see below), achieved TFLOP/s and TB/s against the MI355X's
dense bf16 peak (2.5 PFLOP/s) and HBM (8 TB/s), VALU and LDS instructions
per MFMA, and LDS bank conflicts as SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
(extra cycles over all LDS-array cycles, MI355X_MICROARCH.md section LDS).

    python scripts/disc_roofline.py SEQ.txt PMC_DIR [--md out.md]
"""
import argparse
import collections
import csv
import glob
import re
import sys

PEAK_TFLOPS = 2500.0
PEAK_TBS = 8.0

B, H, W = 8, 480, 640
A1 = B * 240 * 320 * 32 * 2     # bytes of a bf16 NHWC activation per layer
A2 = B * 120 * 160 * 64 * 2
A3 = B * 60 * 80 * 128 * 2
A4 = B * 30 * 40 * 256 * 2
U8 = B * H * W * 4
G = 2.0 * B * 120 * 160 * 64 * 512          # each of conv2-4 (fwd, dgrad, wgrad): 10.07 GFLOP
G1 = 2.0 * B * 240 * 320 * 32 * 64          # the first layer (4 input channels): 2.52 GFLOP
PARAMS = 4 * (32 * 64 + 64 * 512 + 128 * 1024 + 256 * 2048 + 256 * 16)   # fp32 weights

# (what, FLOPs, minimum bytes) per position of the default step (22 kernels)
MODEL = [
    ('conv1 fwd (u8 decode fused)', G1, U8 + A1),
    ('BN1 apply fwd', 0, 2 * A1),
    ('conv2 fwd', G, A1 + A2),
    ('BN2 apply fwd', 0, 2 * A2),
    ('conv3 fwd', G, A2 + A3),
    ('BN3 apply fwd', 0, 2 * A3),
    ('conv4 fwd', G, A3 + A4),
    ('head fwd (BN4 apply, pool, conv, BCE)', 0, A4),
    ('head bwd', 0, 2 * A4),
    ('BN4 apply bwd', 0, 3 * A4),
    ('conv4 dgrad', G, A4 + A3),
    ('conv4 wgrad', G, A3 + A4),
    ('BN3 apply bwd', 0, 3 * A3),
    ('conv3 dgrad', G, A3 + A2),
    ('conv3 wgrad', G, A2 + A3),
    ('BN2 apply bwd', 0, 3 * A2),
    ('conv2 dgrad (patch)', G, A2 + A1),
    ('conv2 wgrad', G, A1 + A2),
    ('conv1 wgrad (BN1 bwd + u8 decode fused)', G1, U8 + 2 * A1),
    ('wgrad slice reduce', 0, 0),
    ('adam schedule', 0, 0),
    ('adam update', 0, 4 * PARAMS),
]


# the same step with each tap-GEMM layer's data and weight gradient in one launch
# (dgrad_wgrad_kernel, BT_FUSE_DW): 20 kernels
MODEL_FUSED = MODEL[:10] + [
    ('conv4 dgrad + wgrad (one launch)', 2 * G, 2 * (A4 + A3)),
    ('BN3 apply bwd (folds)', 0, 3 * A3),
    ('conv3 dgrad + wgrad (one launch)', 2 * G, 2 * (A3 + A2)),
] + MODEL[15:]
# ... and the 32-channel layer's patch data gradient with its weight gradient (dpatch_wgrad_kernel): 19
MODEL_FUSED2 = MODEL_FUSED[:14] + [('conv2 dgrad (patch) + wgrad (one launch)', 2 * G, 2 * (A2 + A1))] + MODEL_FUSED[16:]


# round 6's step (17 kernels): the head applies the last BN's backward (no BN4 apply), the Adam
# schedule rides in a slice-reduce launch, every tap-GEMM layer's data and weight gradient is one
# launch, the first layer's weight gradient reads a decoded input patch (conv_wgrad_c4p_kernel)
MODEL_R6 = MODEL[:7] + [
    ('head fwd (BN4 apply, pool, conv, BCE, BN4 bwd sums)', 0, A4),
    ('head bwd (+ BN4 bwd apply)', 0, 3 * A4),
    ('conv4 dgrad + wgrad (one launch)', 2 * G, 2 * (A4 + A3)),
    ('BN3 apply bwd', 0, 3 * A3),
    ('conv3 dgrad + wgrad (one launch)', 2 * G, 2 * (A3 + A2)),
    ('BN2 apply bwd', 0, 3 * A2),
    ('conv2 dgrad (patch) + wgrad (one launch)', 2 * G, 2 * (A2 + A1)),
    ('conv1 wgrad (decoded patch, BN1 bwd fused)', G1, U8 + 2 * A1),
    ('wgrad slice reduce (+ Adam schedule)', 0, 0),
    ('adam update', 0, 4 * PARAMS),
]
# ... and its last form (16 kernels): the update launch sums the first layer's weight-gradient
# slices itself (FusedAdam.attach_reduce), the schedule rides in the conv4 pair's launch
MODEL_R6B = MODEL_R6[:15] + [('adam update (+ conv1 wgrad slice reduce)', 0, 4 * PARAMS)]
CLOCK_HZ, CUS = 2.4e9, 256


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('btn::gpu::', '').replace('void ', '')
    return re.sub(r'\(.*$', '', n).strip()


def base(name):
    """Kernel name without template arguments (the eager step's variants of a
    graphed kernel, e.g. conv1_fwd_kernel<32, 2, false> for <32, 2, true>,
    stand in for it: the PMC passes run eager steps)."""
    return name.split('<')[0]


def read_sequence(path):
    seq = []
    with open(path) as f:
        lines = f.read().splitlines()
    i = next(k for k, ln in enumerate(lines) if ln.startswith('mean over'))
    for ln in lines[i + 1:]:
        m = re.match(r'\s*(\d+)\s+([\d.]+) us\s+(.*)$', ln)
        if not m:
            break
        seq.append((short(m.group(3)), float(m.group(2))))
    return seq


def read_pmc(pmc_dir):
    """{dispatch id: (kernel name, {counter: value})} over every pass."""
    out = {}
    for f in sorted(glob.glob(f'{pmc_dir}/pass*.csv')):
        tag = f
        for r in csv.DictReader(open(f)):
            key = (tag, int(r['Dispatch_Id']))
            nm, ctr = out.setdefault(key, (short(r['Kernel_Name']), {}))
            ctr[r['Counter_Name']] = ctr.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    return out


def per_position(seq, pmc):
    """Average counters per step position: in every pass, dispatches in order
    are matched greedily against the position sequence (steps start at the
    first kernel's name; other kernels of the eager step are skipped)."""
    names = [base(n) for n, _ in seq]
    acc = [collections.defaultdict(float) for _ in names]
    cnt = [collections.defaultdict(int) for _ in names]
    by_pass = collections.defaultdict(list)
    for (tag, d), v in pmc.items():
        by_pass[tag].append((d, v))
    for tag, items in by_pass.items():
        items.sort()
        pos = None
        steps = 0
        for _, (nm, ctr) in items:
            nm = base(nm)
            if nm == names[0]:
                pos, steps = 0, steps + 1
            if pos is None or pos >= len(names) or steps < 2:   # first step: warm-up
                if pos is not None and pos < len(names) and nm == names[pos]:
                    pos += 1
                continue
            if nm == names[pos]:
                for k, x in ctr.items():
                    acc[pos][k] += x
                    cnt[pos][k] += 1
                pos += 1
    return [{k: a[k] / c[k] for k in a} for a, c in zip(acc, cnt)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('seq')
    ap.add_argument('pmc')
    ap.add_argument('--md', default=None)
    a = ap.parse_args()
    seq = read_sequence(a.seq)
    ctrs = per_position(seq, read_pmc(a.pmc)) if a.pmc != '-' else [{} for _ in seq]
    model = MODEL_FUSED if any(base(n) == 'dgrad_wgrad_kernel' for n, _ in seq) else MODEL
    if any(base(n) == 'dpatch_wgrad_kernel' for n, _ in seq):
        model = MODEL_FUSED2
    if len(seq) == len(MODEL_R6) and any(base(n) == 'conv_wgrad_c4p_kernel' for n, _ in seq):
        model = MODEL_R6
    if len(seq) == len(MODEL_R6B) and any(base(n) == 'conv_wgrad_c4p_kernel' for n, _ in seq):
        model = MODEL_R6B
    if len(seq) != len(model):
        print(f'warning: {len(seq)} kernels per step, the model has {len(model)}', file=sys.stderr)
    rows = []
    tot = collections.defaultdict(float)
    hdr = ('| # | kernel | what | us | GFLOP | TFLOP/s | % bf16 peak | min MB | fetch MB | write MB | TB/s (meas.) '
           '| % HBM | VALU/MFMA | LDS/MFMA | bank conflict % | conflict cycles % of runtime |')
    rows.append(hdr)
    rows.append('|' + '---|' * 16)
    for i, (nm, us) in enumerate(seq):
        what, fl, mb = model[i] if i < len(model) else ('?', 0, 0)
        c = ctrs[i] if i < len(ctrs) else {}
        # FETCH_SIZE x 2: on this gfx950 / rocprofv3 the counter reads half the
        # bytes a streaming kernel must read (BN1 apply: 18.9 -> 37.8 MB of the
        # 39.3 MB it reads; WRITE_SIZE matches the analytic writes as is)
        fetch = 2.0 * c.get('FETCH_SIZE', 0.0) / 1024.0      # KB -> MB
        write = c.get('WRITE_SIZE', 0.0) / 1024.0
        mf = c.get('SQ_INSTS_MFMA', 0.0)
        lds_act = c.get('SQ_LDS_IDX_ACTIVE', 0.0)
        moved = (fetch + write) if c else mb / 1e6
        tbs = moved * 1e6 / (us * 1e-6) / 1e12 if us else 0.0
        tf = fl / (us * 1e-6) / 1e12 if us else 0.0
        rows.append(f'| {i} | `{nm[:44]}` | {what} | {us:.2f} | {fl / 1e9:.2f} | {tf:.0f} | {100 * tf / PEAK_TFLOPS:.1f} '
                    f'| {mb / 1e6:.1f} | {fetch:.1f} | {write:.1f} | {tbs:.2f} | {100 * tbs / PEAK_TBS:.0f} '
                    f'| {c.get("SQ_INSTS_VALU", 0) / mf if mf else float("nan"):.2f} '
                    f'| {c.get("SQ_INSTS_LDS", 0) / mf if mf else float("nan"):.2f} '
                    f'| {100 * c.get("SQ_LDS_BANK_CONFLICT", 0) / lds_act if lds_act else float("nan"):.1f} '
                    # extra LDS cycles of all CUs over the kernel's CU-cycles (trace duration x clock x CUs)
                    f'| {100 * c.get("SQ_LDS_BANK_CONFLICT", 0) / (us * 1e-6 * CLOCK_HZ * CUS) if (c and us) else float("nan"):.2f} |')
        tot['us'] += us
        tot['fl'] += fl
        tot['mb'] += mb / 1e6
        tot['moved'] += moved
    rows.append(f'| | **step** | | **{tot["us"]:.1f}** | {tot["fl"] / 1e9:.1f} | {tot["fl"] / (tot["us"] * 1e-6) / 1e12:.0f} '
                f'| {100 * tot["fl"] / (tot["us"] * 1e-6) / 1e12 / PEAK_TFLOPS:.1f} | {tot["mb"]:.0f} | | '
                f'| {tot["moved"] * 1e6 / (tot["us"] * 1e-6) / 1e12:.2f} | | | | | |')
    txt = '\n'.join(rows)
    print(txt)
    if a.md:
        with open(a.md, 'w') as f:
            f.write(txt + '\n')


if __name__ == '__main__':
    main()
