"""The parallel emulation of a sequential fp64 sum (density.hip block_sum_chain),
restated in numpy and checked against the plain sequential loop on adversarial inputs.

The kernel itself is checked on the GPU (tests/test_gpu_tier_r.py: the reference's goldens and
test_preprocess_chain_stress_vs_oracle). This CPU test pins the algorithm the kernel implements:
while the accumulator a stays in one binade with grid u, fl(a + v) = a + u * rint(v / u), unless v / u
is an exact tie; a window of rows is accepted when every partial sum stays inside the binade, and a
violating row is added with one ordinary add."""
import math

import numpy as np
import pytest

TWO44, TWO52, TWO53 = 2.0 ** 44, 2.0 ** 52, 2.0 ** 53


def sequential(vals):
    a = 0.0
    for v in vals:
        a = a + float(v)
    return a


def emulated(vals, window=256, min_run=16, seq_run=32, stats=None):
    """Window-at-a-time emulation with the kernel's acceptance rules (exact integer prefix sums).
    stats (dict, optional) receives the number of rows added one at a time."""
    a, i, n, forced = 0.0, 0, len(vals), 0
    singles = 0
    while i < n:
        if forced > 0 or not (abs(a) >= 2.2250738585072014e-308) or not math.isfinite(a):
            run = min(forced, n - i) if forced > 0 else 1
            for t in range(run):
                a = a + float(vals[i + t])
            singles += run
            i += run
            forced = max(0, forced - run)
            continue
        _, e = math.frexp(a)
        sh = 53 - e
        A = math.ldexp(a, sh)
        seg = np.asarray(vals[i:i + window], dtype=np.float64)
        xs = np.ldexp(seg, sh)
        k = np.rint(xs)
        bad = ~(np.abs(k) <= TWO44) | (np.abs(xs - k) == 0.5)
        k = np.where(bad, 0.0, k)
        P = np.cumsum(k)  # integers below 2^52: exact
        Aj = A + P
        sAj = Aj if a > 0 else -Aj
        viol = bad | ~((sAj > TWO52) & (sAj < TWO53))
        if not viol.any():
            a = math.ldexp(float(Aj[-1]), -sh)
            i += len(seg)
            continue
        j0 = int(np.argmax(viol))
        if j0 > 0:
            a = math.ldexp(float(Aj[j0 - 1]), -sh)
        a = a + float(seg[j0])
        singles += 1
        i += j0 + 1
        if j0 < min_run:
            forced = seq_run
    if stats is not None:
        stats["singles"] = singles
    return a


def _cases():
    rng = np.random.default_rng(7)
    n = 20000
    yield "squares", rng.uniform(-15, 15, n) ** 2
    yield "centred", rng.uniform(-15, 15, n)
    yield "ties_at_grid", 2.0 ** 40 + rng.integers(0, 1000, n) * 0.25
    yield "cancel", np.where(np.arange(n) % 2 == 0, 1e12, -1e12) + rng.uniform(-1, 1, n)
    yield "tiny", rng.uniform(-1e-300, 1e-300, n)
    yield "subnormal_mix", np.concatenate([rng.uniform(0, 1e-310, 100), rng.uniform(0, 1, n)])
    yield "powers", rng.choice([1.0, 1.5, -1.0, -1.5], n) * np.ldexp(1.0, rng.integers(-30, 30, n))
    yield "int_big", rng.integers(-2 ** 40, 2 ** 40, n).astype(np.float64)
    yield "huge_then_small", np.concatenate([[1e300, -1e300], rng.uniform(0, 1, n)])
    yield "inf", np.concatenate([rng.uniform(0, 1, 500), [np.inf], rng.uniform(0, 1, 500)])
    yield "nan", np.concatenate([rng.uniform(0, 1, 500), [np.nan], rng.uniform(0, 1, 500)])


@pytest.mark.parametrize("name,vals", list(_cases()), ids=[c[0] for c in _cases()])
def test_emulation_equals_sequential_sum(name, vals):
    want, got = sequential(vals), emulated(vals)
    assert (math.isnan(want) and math.isnan(got)) or np.float64(want).tobytes() == np.float64(got).tobytes()


def test_emulation_accepts_most_rows_of_a_sum_of_squares():
    """The point of the emulation: a growing accumulator stays in a binade for long runs, so nearly every
    row is accepted inside a window and single adds stay a small share (a centred sum is the opposite
    case, which is why the kernel keeps those chains sequential)."""
    rng = np.random.default_rng(1)
    sq, st = rng.uniform(-15, 15, 65536) ** 2, {}
    assert np.float64(emulated(sq, stats=st)).tobytes() == np.float64(sequential(sq)).tobytes()
    assert st["singles"] < 0.02 * len(sq)
    centred, st2 = rng.uniform(-15, 15, 65536), {}
    emulated(centred, stats=st2)
    assert st2["singles"] > 0.2 * len(centred)
