"""CPU check of the fused SA-MLP kernel's data layout (no GPU needed).

Emulates, lane by lane, what ``sa_group_mlp_kernel`` (csrc/sa_mlp.hip) does with the
weight image built by the library's own host packer ``lidar_mlp_pack_f32``:
v_mfma_f32_32x32x2_f32 semantics (lane l holds A[l&31][l>>5] and B[l>>5][l&31];
D reg r of lane l is row (r&3)+8(r>>2)+4(l>>5), column l&31), the accumulator-as-
operand chaining and the transposed last layer — and compares with the oracle's
plain matrix formulation.  A wrong packing order fails here before any GPU run.
"""
import numpy as np
import pytest

from oracle import tier_n
from lidar_ai_recommendation_software_amd import pointnet2 as pn


def rho(r):
    return (r & 3) + 8 * (r >> 2)


def mfma(acc, a, b):
    """acc (32, 32) += A(32x2) B(2x32) with per-lane operands a, b (64,)."""
    A = np.stack([a[:32], a[32:]], axis=1).astype(np.float64)
    Bm = np.stack([b[:32], b[32:]], axis=0).astype(np.float64)
    return acc + A @ Bm


def regs_of(D):
    """(32,32) tile -> per-lane registers (64, 16) in the D layout."""
    out = np.empty((64, 16))
    for l in range(64):
        for r in range(16):
            out[l, r] = D[rho(r) + 4 * (l >> 5), l & 31]
    return out


def emulate(x_rows, packed, cf, c1, c2, c3):
    """x_rows: (32, 3 + cf) canonical rows [dx, dy, dz, f...] -> (32, c3) last-layer
    outputs (before the max-pool), following the kernel's indexing exactly."""
    s1 = cf // 2 + 2
    s1p = (s1 + 3) // 4 * 4
    T1, T2, T3 = c1 // 32, c2 // 32, c3 // 32
    W1 = packed
    W2 = W1[T1 * s1p * 64:]
    W3 = W2[T2 * (c1 // 2) * 64:]
    B1 = W3[T3 * (c2 // 2) * 64:]
    B2, B3 = B1[c1:], B1[c1 + c2:]
    # layer-1 per-lane B operand
    x1 = np.zeros((64, s1p))
    for l in range(64):
        h, col = l >> 5, l & 31
        row = x_rows[col]
        for q in range(cf // 2):
            x1[l, q] = row[3 + h * (cf // 2) + q]
        x1[l, cf // 2] = row[2] if h else row[0]
        x1[l, cf // 2 + 1] = 0.0 if h else row[1]
    wl = lambda W, t, steps, s: np.array([W[((t * (steps // 4) + s // 4) * 64 + l) * 4 + s % 4] for l in range(64)])
    y1 = []
    for t in range(T1):
        acc = np.zeros((32, 32))
        for s in range(s1p):
            acc = mfma(acc, wl(W1, t, s1p, s), x1[:, s])
        R = regs_of(acc)
        for l in range(64):
            for r in range(16):
                R[l, r] = max(R[l, r] + B1[32 * t + rho(r) + 4 * (l >> 5)], 0.0)
        y1.append(R)
    y2 = []
    for t in range(T2):
        acc = np.zeros((32, 32))
        for ti in range(T1):
            for r in range(16):
                acc = mfma(acc, wl(W2, t, c1 // 2, ti * 16 + r), y1[ti][:, r])
        R = regs_of(acc)
        for l in range(64):
            for r in range(16):
                R[l, r] = max(R[l, r] + B2[32 * t + rho(r) + 4 * (l >> 5)], 0.0)
        y2.append(R)
    out = np.zeros((32, c3))
    for t in range(T3):
        acc = np.zeros((32, 32))
        for ti in range(T2):
            for r in range(16):
                acc = mfma(acc, y2[ti][:, r], wl(W3, t, c2 // 2, ti * 16 + r))
        R = regs_of(acc)
        for l in range(64):
            for r in range(16):
                p = rho(r) + 4 * (l >> 5)
                out[p, 32 * t + (l & 31)] = max(R[l, r] + B3[32 * t + (l & 31)], 0.0)
    return out


@pytest.mark.parametrize("cfg_name,level,branch", [("ssg", 0, 0), ("ssg", 1, 0), ("msg", 0, 2)])
def test_packed_mfma_chain_matches_matrix_form(cfg_name, level, branch):
    cfg = pn.CONFIGS[cfg_name]
    layers = pn.init_weights(cfg, seed=5)[level][branch]
    cf = layers[0][0].shape[0] - 3
    c1, c2, c3 = (w.shape[1] for w, _ in layers)
    packed = pn.pack_branch(layers, cf)
    rng = np.random.default_rng(0)
    rows = rng.standard_normal((32, 3 + cf)).astype(np.float32)
    got = emulate(rows, packed.astype(np.float64), cf, c1, c2, c3)
    h = rows.astype(np.float64)
    for W, b in layers:
        h = np.maximum(h @ W.astype(np.float64) + b, 0)
    np.testing.assert_allclose(got, h, rtol=1e-9, atol=1e-9)
    # and the oracle's fp32 formulation agrees to fp32 precision
    want = tier_n.mlp_maxpool(rows, layers, 32)[0]
    np.testing.assert_allclose(got.max(axis=0), want, rtol=1e-4, atol=1e-5)


# ----------------------------------------------------------------------------- bf16
def bf16_vals(packed_u16):
    return (packed_u16.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def mfma16(acc, a, b):
    """acc (32,32) += A(32x16) B(16x32); lane l holds A[l&31][8h+j], B[8h+j][l&31]."""
    A = np.concatenate([a[:32], a[32:]], axis=1)          # (32, 16): cols 0-7 from h=0
    Bm = np.concatenate([b[:32], b[32:]], axis=1).T      # (16, 32)
    return acc + A @ Bm


def emulate_bf16(x_rows, packed_bytes, cf, c1, c2, c3):
    k1 = (cf + 3 + 15) // 16 * 16
    s1 = k1 // 16
    T1, T2, T3 = c1 // 32, c2 // 32, c3 // 32
    n_w = (T1 * s1 + T2 * T1 * 2 + T3 * T2 * 2) * 64 * 8
    W = bf16_vals(np.frombuffer(packed_bytes[: 2 * n_w], dtype=np.uint16))
    bias = np.frombuffer(packed_bytes[2 * n_w:], dtype=np.float32).astype(np.float64)
    B1, B2, B3 = bias[:c1], bias[c1:c1 + c2], bias[c1 + c2:]
    W1 = W[: T1 * s1 * 512].reshape(T1, s1, 64, 8)
    W2 = W[T1 * s1 * 512: T1 * s1 * 512 + T2 * T1 * 2 * 512].reshape(T2, T1, 2, 64, 8)
    W3 = W[T1 * s1 * 512 + T2 * T1 * 2 * 512:].reshape(T3, T2, 2, 64, 8)
    phys = np.zeros((32, k1))
    phys[:, :cf] = x_rows[:, 3:]
    phys[:, cf:cf + 3] = x_rows[:, :3]
    x1 = np.zeros((s1, 64, 8))
    for s in range(s1):
        for l in range(64):
            x1[s, l] = phys[l & 31, 16 * s + 8 * (l >> 5): 16 * s + 8 * (l >> 5) + 8]

    def frags(D):
        f = np.zeros((2, 64, 8))
        for l in range(64):
            for s in range(2):
                for j in range(8):
                    r = 8 * s + j
                    f[s, l, j] = D[rho(r) + 4 * (l >> 5), l & 31]
        from oracle.tier_n import bf16_round  # the kernel converts fragments with RNE
        return bf16_round(f.astype(np.float32)).astype(np.float64)

    y1 = []
    for t in range(T1):
        acc = np.zeros((32, 32))
        for s in range(s1):
            acc = mfma16(acc, W1[t, s], x1[s])
        acc = np.maximum(acc + B1[32 * t: 32 * t + 32, None], 0)
        y1.append(frags(acc))
    y2 = []
    for t in range(T2):
        acc = np.zeros((32, 32))
        for ti in range(T1):
            for s in range(2):
                acc = mfma16(acc, W2[t, ti, s], y1[ti][s])
        acc = np.maximum(acc + B2[32 * t: 32 * t + 32, None], 0)
        y2.append(frags(acc))
    out = np.zeros((32, c3))
    for t in range(T3):
        acc = np.zeros((32, 32))
        for ti in range(T2):
            for s in range(2):
                acc = mfma16(acc, y2[ti][s], W3[t, ti, s])
        out[:, 32 * t: 32 * t + 32] = np.maximum(acc + B3[None, 32 * t: 32 * t + 32], 0)
    return out


@pytest.mark.parametrize("cfg_name,level,branch", [("msg", 0, 0), ("msg", 1, 1), ("ssg", 1, 0)])
def test_packed_bf16_chain_matches_matrix_form(cfg_name, level, branch):
    from oracle.tier_n import bf16_round
    cfg = pn.CONFIGS[cfg_name]
    layers = pn.init_weights(cfg, seed=6)[level][branch]
    layers = [(bf16_round(W), b) for W, b in layers]  # exact in bf16: a pure layout check
    cf = layers[0][0].shape[0] - 3
    c1, c2, c3 = (w.shape[1] for w, _ in layers)
    packed = pn.pack_branch_bf16(layers, cf)
    rows = bf16_round(np.random.default_rng(2).standard_normal((32, 3 + cf)).astype(np.float32))
    got = emulate_bf16(rows.astype(np.float64), packed.tobytes(), cf, c1, c2, c3)
    h = rows.astype(np.float64)
    for i, (W, b) in enumerate(layers):
        h = np.maximum(h @ W.astype(np.float64) + b, 0)
        if i < 2:  # hidden activations enter the next MFMA as bf16 in both formulations
            h = bf16_round(h.astype(np.float32)).astype(np.float64)
    # same roundings on both sides: equal up to fp64 summation order (a rare bf16 tie flip
    # shows up as one isolated ~2^-8 difference)
    close = np.isclose(got, h, rtol=1e-9, atol=1e-12)
    assert close.mean() > 0.99, f"{(~close).sum()} of {close.size} differ"
    np.testing.assert_allclose(got, h, rtol=2e-2, atol=1e-3)
