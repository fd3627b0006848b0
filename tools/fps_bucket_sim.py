"""FPS pruning by bucket size (numpy simulation, CPU): points streamed per step for buckets of S
consecutive points of a Morton order (64^3 grid by default), with
  * 'flat'  — every bucket keyed by its own max: active iff lb(box) < bucket max;
  * 'two'   — 64-point blocks keyed by their max, split into S-point sub-buckets with their own boxes:
              a sub-bucket is streamed iff lb(sub box) < its OWN max (per-sub max kept);
and optional box quantisation to Q bits per bound relative to the frame bbox (outward rounding).
usage: fps_bucket_sim.py STEPS [S ...]"""
import sys
import numpy as np

rng = np.random.default_rng(1)
N = 65536
M = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
sizes = [int(s) for s in sys.argv[2:]] or [64, 32, 16]
x = rng.uniform(-1, 1, (N, 3)).astype(np.float32)


def spread(v, bits):
    r = np.zeros_like(v)
    for b in range(bits):
        r |= ((v >> b) & 1) << (3 * b)
    return r


def morton(g):
    lo = x.min(0)
    hi = x.max(0)
    c = np.clip(((x - lo) * (g / (hi - lo))).astype(np.int64), 0, g - 1)
    bits = int(np.log2(g))
    return spread(c[:, 0], bits) | (spread(c[:, 1], bits) << 1) | (spread(c[:, 2], bits) << 2)


def quant(bmin, bmax, qbits):
    if not qbits:
        return bmin, bmax
    lo = x.min(0)
    hi = x.max(0)
    s = (hi - lo) / (2 ** qbits - 1)
    return lo + np.floor((bmin - lo) / s) * s, lo + np.ceil((bmax - lo) / s) * s


for g in (16, 64):
    order = np.argsort(morton(g), kind="stable")
    xs = x[order]
    for S in sizes:
        for qbits in (0, 8):
            nb = N // S
            B = xs.reshape(nb, S, 3)
            bmin, bmax = quant(B.min(1), B.max(1), qbits)
            dist = np.full(N, np.inf, np.float32)
            last = 0
            act = 0
            for it in range(1, M):
                q = xs[last]
                gg = np.maximum(np.maximum(bmin - q, q - bmax), 0)
                lb = (gg * gg).sum(1)
                bd = dist.reshape(nb, S).max(1)
                a = lb < bd
                act += int(a.sum())
                d = ((xs - q) ** 2).sum(1).astype(np.float32)
                dist = np.minimum(dist, d)
                last = int(np.argmax(dist))
            print("morton %d^3 S=%d q=%d: active/step %.1f  points/step %.0f  (x64-bucket-equiv %.1f)"
                  % (g, S, qbits, act / (M - 1), act * S / (M - 1), act * S / (M - 1) / 64), flush=True)
