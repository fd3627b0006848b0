"""CPU restatement of the north_star operators (Tier N).  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  The product path never imports ``oracle``.

PARITY UNPINNED BY THE REFERENCE: farthest-point sampling, ball query with
``nsample``, grouping, the SetAbstraction MLP and voxel downsampling do not exist
in ``/root/reference``.  This file freezes the
build-defined spec — the canonical PointNet++ semantics — and its
outputs on seeded inputs are committed as ``tests/golden/tier_n.npz``.  The C
loops (``lidar_oracle.c``) are cross-checked against the pure-numpy loops here.

Spec (all fp32, one rounding per operation, never fused multiply-add):
  d(p, q)     = (dx*dx + dy*dy) + dz*dz,  dx = p.x - q.x ...
  fps         idx[0] = 0; dist = +inf; for i >= 1: dist = min(dist, d(., xyz[idx[i-1]]));
              idx[i] = argmax(dist), lowest index on ties.
  ball_query  r2 = r*r (fp32); the first nsample k (ascending) with d(xyz[k], c) < r2;
              unused slots repeat the first hit; no hit -> all 0.
  grouping    [xyz[idx] - centre, features[idx]]  (use_xyz, channels last).
  SA MLP      h = relu(h @ W + b) per layer; max over the nsample axis.
  group_all   input [xyz, features] over all points, max over all points.
  bf16 mode   SA branches: grouped xyz offsets, features, hidden activations and
              weights rounded to bf16 (RNE) before each layer, fp32 accumulation, fp32
              bias/ReLU/pool; group_all stays fp32.
  voxel       per axis the bins of the reference's calculate_grid_density
              (utils/data_processing.py:305-319): edges np.arange(lo - 2v,
              (hi + 2v) + v, v) over the frame's extent (float64), histogram2d's
              rule (searchsorted right, the last edge closed, outside -> none);
              key = (bx * ny + by) * nz + bz; voxels in ascending key order;
              centroid = sequential fp32 sum in point order / count; per-point
              voxel id = rank of its key (-1 outside every bin).  The x/y part is
              PINNED: summed over z the counts equal the reference's own
              calculate_grid_density on the frame's (x, y) (tests/golden/voxel.npz).
"""
import numpy as np

from .tier_r import lib, _ptr


# ----------------------------------------------------------------- sampling
def fps_numpy(xyz, npoint):
    """Pure-numpy FPS (small sizes; cross-checks the C loop)."""
    xyz = np.asarray(xyz, dtype=np.float32)
    n = len(xyz)
    out = np.zeros(npoint, dtype=np.int32)
    dist = np.full(n, np.inf, dtype=np.float32)
    last = 0
    for i in range(1, npoint):
        dd = xyz - xyz[last]
        d = dd[:, 0] * dd[:, 0] + dd[:, 1] * dd[:, 1]
        d = d + dd[:, 2] * dd[:, 2]
        dist = np.minimum(dist, d)
        last = int(np.argmax(dist))
        out[i] = last
    return out


def fps(xyz, npoint):
    """FPS over (N,3) or (B,N,3) float32 -> int32 indices (C loop)."""
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    if xyz.ndim == 3:
        return np.stack([fps(f, npoint) for f in xyz])
    n = len(xyz)
    out = np.zeros(npoint, dtype=np.int32)
    dist = np.empty(max(n, 1), dtype=np.float32)
    lib().orc_fps(_ptr(xyz), n, npoint, _ptr(out), _ptr(dist))
    return out


def ball_query_numpy(xyz, centres, radius, nsample):
    xyz = np.asarray(xyz, dtype=np.float32)
    r2 = np.float32(radius) * np.float32(radius)
    out = np.zeros((len(centres), nsample), dtype=np.int32)
    for c, q in enumerate(np.asarray(centres, dtype=np.float32)):
        dd = xyz - q
        d = dd[:, 0] * dd[:, 0] + dd[:, 1] * dd[:, 1]
        d = d + dd[:, 2] * dd[:, 2]
        hits = np.flatnonzero(d < r2)[:nsample]
        if len(hits):
            out[c, :] = hits[0]
            out[c, :len(hits)] = hits
    return out


def ball_query(xyz, centres, radius, nsample):
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    centres = np.ascontiguousarray(centres, dtype=np.float32)
    if xyz.ndim == 3:
        return np.stack([ball_query(a, b, radius, nsample) for a, b in zip(xyz, centres)])
    out = np.empty((len(centres), nsample), dtype=np.int32)
    lib().orc_ball_query(_ptr(xyz), len(xyz), _ptr(centres), len(centres),
                         float(np.float32(radius)), int(nsample), _ptr(out))
    return out


# ------------------------------------------------------------------ MLP
def bf16_round(x):
    """Round float32 to the nearest bfloat16 (ties to even), returned as float32."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16 << 16
    return u.astype(np.uint32).view(np.float32)


def mlp_maxpool(h, layers, group, bf16=False):
    """h: (R, Cin) rows grouped `group` at a time -> (R/group, Cout) max-pooled.

    fp32: each layer relu(h @ W + b) in float32 (BLAS).  bf16: layer inputs and
    weights rounded to bf16 (RNE), products accumulated in float64 then rounded
    to float32 (an fp32-accumulator stand-in), bias added in fp32.
    """
    h = np.asarray(h, dtype=np.float32)
    for W, b in layers:
        if bf16:
            acc = bf16_round(h).astype(np.float64) @ bf16_round(W).astype(np.float64)
            h = np.maximum(acc.astype(np.float32) + b, np.float32(0))
        else:
            h = np.maximum(h @ W + b, np.float32(0))
    return h.reshape(-1, group, h.shape[-1]).max(axis=1)


def group(xyz, feats, centres, idx):
    """(N,3),(N,C)|None,(M,3),(M,ns) -> (M*ns, 3+C) rows [xyz - centre, feats]."""
    g = xyz[idx] - centres[:, None, :]
    parts = [g.reshape(-1, 3)]
    if feats is not None:
        parts.append(feats[idx].reshape(-1, feats.shape[-1]))
    return np.concatenate(parts, axis=1).astype(np.float32)


def set_abstraction(xyz, feats, npoint, radii, nsamples, branch_layers, bf16=False):
    """One SA level (SSG when len(radii) == 1, MSG otherwise) for one frame."""
    idx = fps(xyz, npoint)
    centres = xyz[idx]
    outs = []
    fin = feats
    if bf16 and fin is not None:
        fin = bf16_round(fin)
    for r, ns, layers in zip(radii, nsamples, branch_layers):
        gi = ball_query(xyz, centres, r, ns)
        outs.append(mlp_maxpool(group(xyz, fin, centres, gi), layers, ns, bf16))
    return centres, np.concatenate(outs, axis=1), idx


def group_all(xyz, feats, layers, bf16=False):
    h = np.concatenate([xyz, bf16_round(feats) if bf16 else feats], axis=1).astype(np.float32)
    return mlp_maxpool(h, layers, len(h), bf16)[0]


def sa_stack(xyz, cfg, weights, bf16=False):
    """Full SSG/MSG backbone on one frame -> (global feature (1024,), per-level info)."""
    feats = None
    levels = []
    for lvl, w in zip(cfg["levels"], weights):
        if lvl.get("group_all"):
            g = group_all(xyz, feats, w[0], False)  # spec: group_all is fp32 in both modes
            levels.append((None, g, None))
            return g, levels
        npoint = lvl["npoint"]
        xyz, feats, idx = set_abstraction(xyz, feats, npoint, lvl["radii"], lvl["nsamples"], w, bf16)
        levels.append((xyz, feats, idx))
    return feats, levels


# ---------------------------------------------------------------- voxels
def voxel_edges(lo, hi, voxel_size):
    """calculate_grid_density's edges for the extent [lo, hi] (utils/data_processing.py:305-313):
    the 2-cell margin, then np.arange(lo - 2v, (hi + 2v) + v, v)."""
    margin = voxel_size * 2
    return np.arange(lo - margin, (hi + margin) + voxel_size, voxel_size)


def voxel_bins(xyz, voxel_size):
    """(N,3) float32 -> per-axis bins (N,3) int64 (-1 outside) and the bin counts (nx, ny, nz):
    histogramdd's rule (numpy/lib/_histograms_impl.py) on voxel_edges of each axis."""
    x = np.asarray(xyz, dtype=np.float32).astype(np.float64)
    v = float(voxel_size)
    bins = np.empty(x.shape, dtype=np.int64)
    dims = []
    for a in range(3):
        e = voxel_edges(float(x[:, a].min()), float(x[:, a].max()), v)
        if len(e) < 2:
            raise ValueError("voxel_downsample: fewer than 2 edges on an axis")
        c = np.searchsorted(e, x[:, a], side="right")
        c[x[:, a] == e[-1]] -= 1
        b = c - 1
        b[(c < 1) | (c > len(e) - 1)] = -1
        bins[:, a] = b
        dims.append(len(e) - 1)
    if dims[0] * dims[1] * dims[2] >= 0xffffffff:
        raise ValueError("voxel_downsample: the voxel grid has 2^32 keys or more")
    return bins, tuple(dims)


def voxel_downsample(xyz, voxel_size):
    """(N,3) float32 -> (centroids (V,3) f32, voxel id per point (N,) int32, counts (V,) int32)."""
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    n = len(xyz)
    if n == 0:
        return np.zeros((0, 3), np.float32), np.zeros(0, np.int32), np.zeros(0, np.int32)
    if not np.isfinite(xyz).all():
        raise ValueError("voxel_downsample: the extent is not finite (np.arange cannot compute a length)")
    bins, (nx, ny, nz) = voxel_bins(xyz, voxel_size)
    inside = (bins >= 0).all(axis=1)
    key = (bins[:, 0] * ny + bins[:, 1]) * nz + bins[:, 2]
    uniq, inv, counts = np.unique(key[inside], return_inverse=True, return_counts=True)
    vid = np.full(n, -1, dtype=np.int64)
    vid[inside] = inv
    sums = np.zeros((len(uniq), 3), dtype=np.float32)
    pts = np.flatnonzero(inside)
    order = pts[np.argsort(vid[pts], kind="stable")]  # point order inside every voxel
    for i in order:  # sequential fp32 sums in point order (small sizes only)
        sums[vid[i]] += xyz[i]
    cent = sums / counts[:, None].astype(np.float32)
    return cent.astype(np.float32), vid.astype(np.int32), counts.astype(np.int32)


def voxel_counts_xy(vid, counts, bins, dims):
    """The (nx, ny) histogram of a frame's voxels summed over z (what calculate_grid_density
    counts on the same x / y edges)."""
    nx, ny, _ = dims
    out = np.zeros((nx, ny), dtype=np.int64)
    inside = vid >= 0
    np.add.at(out, (bins[inside, 0], bins[inside, 1]), 1)
    return out
