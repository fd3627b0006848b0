"""PointNet++ SetAbstraction operators and backbones on liblidar_amd (gfx950 HIP).

These are the north_star operators that the reference does not have (SURVEY.md §0,
§8a N2-N6).  They sit beside the reference's operator set
(``utils/data_processing.py:231`` ``downsample_point_cloud`` and the density model,
``models/crowd_density_model.py:14``), and every one runs on the HIP kernels behind
``include/lidar_amd.h``.  Torch only holds device memory and the stream.

Spec (frozen in DESIGN.md §3, restated by ``oracle/tier_n.py``): fp32 coordinates,
distances ``(dx*dx + dy*dy) + dz*dz`` with one rounding per operation;
FPS starts at index 0 and breaks ties to the lowest index; ball query keeps the first
``nsample`` hits in index order; grouping is ``[xyz - centre, features]`` (use_xyz);
each SA branch is a 3-layer shared MLP (conv1x1 + folded BN + ReLU) max-pooled over
its neighbourhood; the last level is group_all.

Layouts: xyz (B, N, 3) float32; features channels-last (B, N, C) float32.
"""
import ctypes

import numpy as np
import torch

from . import _native as nat
from .streams import side_streams

# ------------------------------------------------------------------ configs
# BASELINE.json configs: C2 = one SA1 layer, C3 = 3-level SSG, C5 = 3-level MSG.
SSG = {
    "name": "ssg",
    "levels": [
        {"npoint_div": 16, "radii": [0.2], "nsamples": [32], "mlps": [[64, 64, 128]]},
        {"npoint_div": 64, "radii": [0.4], "nsamples": [64], "mlps": [[128, 128, 256]]},
        {"group_all": True, "mlps": [[256, 512, 1024]]},
    ],
}
MSG = {
    "name": "msg",
    "levels": [
        {"npoint_div": 16, "radii": [0.1, 0.2, 0.4], "nsamples": [16, 32, 128],
         "mlps": [[32, 32, 64], [64, 64, 128], [64, 96, 128]]},
        {"npoint_div": 64, "radii": [0.2, 0.4, 0.8], "nsamples": [32, 64, 128],
         "mlps": [[64, 64, 128], [128, 128, 256], [128, 128, 256]]},
        {"group_all": True, "mlps": [[256, 512, 1024]]},
    ],
}
SA1_ONLY = {  # C2: 16 384 points -> 1 024 centroids, r = 0.2, nsample 32
    "name": "sa1",
    "levels": [{"npoint_div": 16, "radii": [0.2], "nsamples": [32], "mlps": [[64, 64, 128]]}],
}
CONFIGS = {"ssg": SSG, "msg": MSG, "sa1": SA1_ONLY}


def resolve(cfg, n):
    """Per-level dicts with concrete npoint for an n-point frame (oracle format)."""
    out = []
    for lvl in cfg["levels"]:
        d = dict(lvl)
        if not lvl.get("group_all"):
            d["npoint"] = max(1, n // lvl["npoint_div"])
        out.append(d)
    return out


def init_weights(cfg, seed=0):
    """Deterministic random init (conv1x1 default: U(-1/sqrt(cin), 1/sqrt(cin)), BN folded
    at its fresh-init identity).  Returns [level][branch][layer] = (W (cin, cout), b)."""
    rng = np.random.default_rng(seed)
    weights, cin_feat = [], 0
    for lvl in cfg["levels"]:
        branches, cout_total = [], 0
        for widths in lvl["mlps"]:
            layers, cin = [], 3 + cin_feat
            for cout in widths:
                bound = 1.0 / np.sqrt(cin)
                W = rng.uniform(-bound, bound, (cin, cout)).astype(np.float32)
                b = rng.uniform(-bound, bound, cout).astype(np.float32)
                layers.append((W, b))
                cin = cout
            branches.append(layers)
            cout_total += widths[-1]
        weights.append(branches)
        cin_feat = cout_total
    return weights


def check_weights(cfg, weights):
    """Validate [level][branch][layer] = (W (cin, cout), b (cout,)) against cfg's widths (cin = 3 + the
    previous level's channels); returns them as contiguous float32 arrays.  Raises ValueError naming the
    first mismatch."""
    out, cin_feat = [], 0
    if len(weights) != len(cfg["levels"]):
        raise ValueError(f"weights: {len(weights)} levels, the configuration has {len(cfg['levels'])}")
    for li, (lvl, wl) in enumerate(zip(cfg["levels"], weights)):
        if len(wl) != len(lvl["mlps"]):
            raise ValueError(f"weights level {li}: {len(wl)} branches, the configuration has {len(lvl['mlps'])}")
        branches = []
        for bi, (widths, layers) in enumerate(zip(lvl["mlps"], wl)):
            if len(layers) != len(widths):
                raise ValueError(f"weights level {li} branch {bi}: {len(layers)} layers, expected {len(widths)}")
            cin, conv = 3 + cin_feat, []
            for j, (cout, (W, b)) in enumerate(zip(widths, layers)):
                W = np.ascontiguousarray(W, dtype=np.float32)
                b = np.ascontiguousarray(b, dtype=np.float32).reshape(-1)
                if W.shape != (cin, cout) or b.shape != (cout,):
                    raise ValueError(f"weights level {li} branch {bi} layer {j}: W {W.shape}, b {b.shape}; "
                                     f"expected ({cin}, {cout}) and ({cout},)")
                conv.append((W, b))
                cin = cout
            branches.append(conv)
        out.append(branches)
        cin_feat = sum(w[-1] for w in lvl["mlps"])
    return out


def save_weights(path, weights):
    """Weights to an .npz of plain arrays (keys l<level>_b<branch>_<layer>_{W,b}; no pickled objects)."""
    arrs = {f"l{li}_b{bi}_{j}_{k}": a for li, wl in enumerate(weights) for bi, layers in enumerate(wl)
            for j, wb in enumerate(layers) for k, a in zip("Wb", wb)}
    np.savez(path, **arrs)


def load_weights(path, cfg):
    """The .npz save_weights wrote, in cfg's layout (loaded with allow_pickle=False), validated."""
    with np.load(path, allow_pickle=False) as z:
        w = [[[(z[f"l{li}_b{bi}_{j}_W"], z[f"l{li}_b{bi}_{j}_b"]) for j in range(len(widths))]
              for bi, widths in enumerate(lvl["mlps"])] for li, lvl in enumerate(cfg["levels"])]
    return check_weights(cfg, w)


# --------------------------------------------------------------- functional ops
def _dev_check(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or not t.is_contiguous()):
            raise ValueError("liblidar_amd operators take contiguous CUDA tensors")


def farthest_point_sample(xyz, npoint, return_xyz=False, first_zero=None, prefix_ok=None, slot=0,
                          out_idx=None, out_xyz=None, threads=0):
    """xyz (B, N, 3) float32 CUDA -> idx (B, npoint) int32 [, new_xyz (B, npoint, 3)].

    threads: workgroup size per frame (0 = 1024, 512; frames above 262 144 points always take 512).
    n <= 4 194 304 points per frame.

    first_zero: optional (B,) int32 output — first step whose winning distance was 0.
    prefix_ok: optional (B,) int32 — the parent run's first_zero when xyz is the parent's
    FPS-ordered sample set (nested SA levels): the exact identity result is copied."""
    _dev_check(xyz, first_zero, prefix_ok)
    if xyz.dtype != torch.float32 or xyz.dim() != 3 or xyz.shape[2] != 3:
        raise ValueError("xyz must be (B, N, 3) float32")
    B, N, _ = xyz.shape
    idx = out_idx if out_idx is not None else torch.empty((B, npoint), dtype=torch.int32, device=xyz.device)
    new_xyz = None
    if return_xyz:
        new_xyz = out_xyz if out_xyz is not None else torch.empty((B, npoint, 3), dtype=torch.float32,
                                                                  device=xyz.device)
    nat.call("lidar_fps_ex_f32", nat.handle(xyz.device.index, slot), nat.ptr(xyz), B, N, npoint,
             nat.ptr(idx), nat.ptr(new_xyz), nat.ptr(first_zero), nat.ptr(prefix_ok),
             int(threads), nat.stream_ptr())
    return (idx, new_xyz) if return_xyz else idx


def voxel_downsample_batch(xyz, voxel, slot=0, check=True, out=None):
    """Voxel downsampling of (B, N, 3) float32 CUDA frames on the whole chip
    (lidar_voxel_downsample_batch_f32; per frame equal to data_processing.voxel_downsample).
    Returns device tensors (centroids (B, N, 3), voxel_id (B, N) int32, counts (B, N) int32,
    nvox (B,) int32): the first nvox[f] centroid / count rows of frame f are valid; nvox -1 marks
    a frame whose extent is not finite or whose voxel grid has 2^32 keys or more.  Voxels are
    calculate_grid_density's grid extended to z (data_processing.voxel_downsample).

    nvox <= -2 is a library failure, never expected: -2 one of the launch's bounded in-launch waits
    timed out, -3 a bucket table that is not a partition of the frame.  check=True (default) reads
    nvox back (a host synchronisation on the stream) and raises LidarError on either; check=False
    leaves nvox on the device (throughput loops: check_voxel_counts(nvox) later).  out: the four output
    tensors of an earlier call of the same shape, written again (a stream of batches allocates once)."""
    _dev_check(xyz)
    if xyz.dtype != torch.float32 or xyz.dim() != 3 or xyz.shape[2] != 3:
        raise ValueError("xyz must be (B, N, 3) float32")
    B, N, _ = xyz.shape
    dev = xyz.device
    if out is not None:
        cent, vid, cnt, nvox = out
        if (tuple(cent.shape) != (B, N, 3) or tuple(vid.shape) != (B, N) or tuple(cnt.shape) != (B, N)
                or tuple(nvox.shape) != (B,) or cent.dtype != torch.float32
                or any(t.dtype != torch.int32 for t in (vid, cnt, nvox))):
            raise ValueError("voxel_downsample_batch: out must be (B, N, 3) float32, (B, N) int32 x 2, (B,) int32")
        _dev_check(cent, vid, cnt, nvox)
    else:
        cent = torch.empty((B, N, 3), dtype=torch.float32, device=dev)
        vid = torch.empty((B, N), dtype=torch.int32, device=dev)
        cnt = torch.empty((B, N), dtype=torch.int32, device=dev)
        nvox = torch.empty(B, dtype=torch.int32, device=dev)
    if B and N:
        nat.call("lidar_voxel_downsample_batch_f32", nat.handle(dev.index, slot), nat.ptr(xyz), B, N,
                 float(voxel), nat.ptr(vid), nat.ptr(cent), nat.ptr(cnt), nat.ptr(nvox), nat.stream_ptr())
        if check:
            check_voxel_counts(nvox)
    return cent, vid, cnt, nvox


VOXEL_FAILURES = {-2: "an in-launch hand-off of the voxel launches timed out",
                  -3: "a voxel bucket table is not a partition of its frame"}


def check_voxel_counts(nvox):
    """Raise LidarError if any frame's nvox reports a library failure (<= -2; reads nvox back)."""
    bad = nvox[nvox <= -2]
    if bad.numel():
        code = int(bad.min().item())
        raise nat.LidarError(f"voxel_downsample_batch: {VOXEL_FAILURES.get(code, 'unknown failure')} "
                             f"(nvox {code} in {bad.numel()} frame(s); a library bug, please report)")


BQ_MODES = {"auto": 0, "scan": 1, "grid": 2}
BQ_GRID_MIN_N = 1024  # csrc/bq_grid.hpp kGridMinN: "auto" bins frames of at least this many points


def ball_query(radius, nsample, xyz, new_xyz, out=None, slot=0, mode="auto", grid=None):
    """-> idx (B, M, nsample) int32 (pointnet2 argument order).

    mode: "auto" (the (index window, cell) grid for N >= 1024, else the index-order scan),
    "scan" or "grid" — identical results.  grid: a buffer filled by ball_query_bin for
    these xyz (the binning then does not run here)."""
    _dev_check(xyz, new_xyz, out)
    B, N, _ = xyz.shape
    M = new_xyz.shape[1]
    idx = out if out is not None else torch.empty((B, M, nsample), dtype=torch.int32, device=xyz.device)
    h = nat.handle(xyz.device.index, slot)
    if grid is not None:
        nat.call("lidar_ball_query_binned_f32", h, nat.ptr(xyz), nat.ptr(grid), nat.ptr(new_xyz),
                 B, N, M, float(radius), int(nsample), nat.ptr(idx), nat.stream_ptr())
    else:
        nat.call("lidar_ball_query_mode_f32", h, nat.ptr(xyz), nat.ptr(new_xyz),
                 B, N, M, float(radius), int(nsample), BQ_MODES[mode], nat.ptr(idx), nat.stream_ptr())
    return idx


def ball_query_grid_buffer(B, N, device):
    """Device buffer for ball_query_bin over (B, N, 3) frames."""
    nbytes = nat.load_library().lidar_ball_query_grid_bytes(B, N)
    return torch.empty((max(1, nbytes),), dtype=torch.uint8, device=device)


def ball_query_bin(radius, nsample, xyz, grid, slot=0):
    """Bin (B, N, 3) frames for later ball_query(..., grid=grid) calls (any stream order
    that puts this launch first).  Depends only on xyz."""
    _dev_check(xyz, grid)
    B, N, _ = xyz.shape
    nat.call("lidar_ball_query_bin_f32", nat.handle(xyz.device.index, slot), nat.ptr(xyz), B, N,
             float(radius), int(nsample), nat.ptr(grid), nat.stream_ptr())
    return grid


# (xyz_level, c1, c2, c3, nsample) combinations lidar_sa_group_mlp16_f32 instantiates
MLP16_SHAPES = {(True, 64, 64, 128, 32), (True, 32, 32, 64, 16), (True, 64, 96, 128, 128), (False, 128, 128, 256, 64),
                (False, 128, 128, 256, 128), (False, 64, 64, 128, 32)}


def pack_branch16(layers, xyz_level):
    """Host-side packed image for lidar_sa_group_mlp16_f32 (16x16x4 MFMA fragments)."""
    (w1, b1), (w2, b2), (w3, b3) = layers
    c1, c2, c3 = w1.shape[1], w2.shape[1], w3.shape[1]
    lib = nat.load_library()
    out = np.zeros(lib.lidar_mlp_packed_size16(int(xyz_level), c1, c2, c3), dtype=np.float32)
    arrs = [np.ascontiguousarray(a, dtype=np.float32) for a in (w1, b1, w2, b2, w3, b3)]
    nat.check(lib.lidar_mlp_pack16_f32(int(xyz_level), c1, c2, c3, *[a.ctypes.data_as(ctypes.c_void_p) for a in arrs],
                                       out.ctypes.data_as(ctypes.c_void_p)), "lidar_mlp_pack16_f32")
    return out


def group_mlp16(p, q, idx, n, packed, widths, out, out_offset=0, xyz_level=False):
    """16-row fused branch.  xyz_level: p = xyz (B, N, 3), q = centres (B, M, 3); else
    p / q are group_mlp_pre's per-point / per-centre layer-1 rows.  -> out[..., off:off+c3]."""
    B, M, ns = idx.shape
    c1, c2, c3 = widths
    if xyz_level:
        if p.numel() < B * n * 3 or q.numel() < B * M * 3 or not (p.is_contiguous() and q.is_contiguous()):
            raise ValueError("group_mlp16: xyz / centres must be contiguous (B, N, 3) / (B, M, 3)")
        stride = 3
    else:
        if p.shape[0] < B * n or q.shape[0] < B * M or p.shape[1] < c1 or q.shape[1] != p.shape[1]:
            raise ValueError("group_mlp16: p/q shapes do not match the batch")
        stride = p.shape[1]
    _dev_check(p, q, idx, packed, out)
    nat.call("lidar_sa_group_mlp16_f32", nat.handle(p.device.index), int(xyz_level), nat.ptr(p), stride,
             nat.ptr(q), nat.ptr(idx), B, n, M, ns, c1, c2, c3, nat.ptr(packed), nat.ptr(out), out.shape[-1],
             out_offset, nat.stream_ptr())
    return out


def pack_branch_x3(layers, xyz_level):
    """Host-side packed image (uint8) for lidar_sa_group_mlp_x3_f32 (fp16 hi/lo fragments of each layer's
    W 2^s, h3 arithmetic; csrc/h3.hpp)."""
    (w1, b1), (w2, b2), (w3, b3) = layers
    c1, c2, c3 = w1.shape[1], w2.shape[1], w3.shape[1]
    lib = nat.load_library()
    out = np.zeros(lib.lidar_mlp_packed_size_x3(int(xyz_level), c1, c2, c3), dtype=np.uint8)
    arrs = [np.ascontiguousarray(a, dtype=np.float32) for a in (w1, b1, w2, b2, w3, b3)]
    nat.check(lib.lidar_mlp_pack_x3_f32(int(xyz_level), c1, c2, c3, *[a.ctypes.data_as(ctypes.c_void_p) for a in arrs],
                                        out.ctypes.data_as(ctypes.c_void_p)), "lidar_mlp_pack_x3_f32")
    return out


def pack_branch_x1(layers):
    """Host-side packed image (uint8) for lidar_sa_group_mlp_x1_f32 (bf16 spec: bf16-rounded
    W1 xyz rows, hi fragments of W2 / W3, fp32 biases)."""
    (w1, b1), (w2, b2), (w3, b3) = layers
    c1, c2, c3 = w1.shape[1], w2.shape[1], w3.shape[1]
    lib = nat.load_library()
    out = np.zeros(lib.lidar_mlp_packed_size_x1(c1, c2, c3), dtype=np.uint8)
    arrs = [np.ascontiguousarray(a, dtype=np.float32) for a in (w1, b1, w2, b2, w3, b3)]
    nat.check(lib.lidar_mlp_pack_x1_f32(c1, c2, c3, *[a.ctypes.data_as(ctypes.c_void_p) for a in arrs],
                                        out.ctypes.data_as(ctypes.c_void_p)), "lidar_mlp_pack_x1_f32")
    return out


def group_mlp_x1(p, idx, n, packed, widths, out, out_offset=0, xyz=None, centres=None):
    """One SA branch in the bf16 spec (lidar_sa_group_mlp_x1_f32).  xyz level: p = the level's
    points (B, n, 3), centres (B, M, 3).  Feature level: p (B*n, >= c1) = bf16(f) bf16(W1_f) + b1
    per point (layer1_points_x1): rows of one stride, possibly a column slice of the level's fused
    layer-1 output; xyz = the level's points, centres."""
    B, M, ns = idx.shape
    c1, c2, c3 = widths
    mode = 2 if xyz is not None else 0
    if mode == 0:
        _dev_check(p, centres, idx, packed, out)
        stride = 3
    else:
        _dev_check(xyz, centres, idx, packed, out)
        if not p.is_cuda or p.dim() != 2 or p.stride(1) != 1:
            raise ValueError("group_mlp_x1: per-point rows must be a CUDA (rows, cols) tensor with unit column stride")
        stride = p.stride(0)
        if p.shape[0] < B * n or p.shape[1] < c1:
            raise ValueError("group_mlp_x1: per-point rows do not match the batch")
    nat.call("lidar_sa_group_mlp_x1_f32", nat.handle(p.device.index), mode, nat.ptr(p), stride,
             nat.ptr(centres) if mode == 0 else None, nat.ptr(xyz), nat.ptr(centres), nat.ptr(idx), B, n, M, ns,
             c1, c2, c3, nat.ptr(packed), nat.ptr(out), out.shape[-1], out_offset, nat.stream_ptr())
    return out


def layer1_points_x1(x_rows, xyz, cfeat, branches, cat=None):
    """Per-point layer-1 feature part of a bf16-spec level: P = bf16(f) bf16(W1_f) + b1 for every
    branch (x_rows: the level's padded rows [f, x, y, z, 0-pad]; the xyz rows of W1_f are zero,
    the offsets' part runs per grouped row in lidar_sa_group_mlp_x1_f32).  cat: the branches' W1_f
    side by side (fused_layer1_x1): one GEMM reads the rows once for every branch, and each branch's
    P is its column slice — the same products in the same order per column (the bf16 spec's image has
    no per-matrix scale), so bit-identical to one GEMM per branch."""
    B, N, _ = xyz.shape
    nat.call("lidar_concat_xyz_pad_f32", nat.handle(xyz.device.index), nat.ptr(xyz), B * N, nat.ptr(x_rows),
             x_rows.shape[1], cfeat, nat.stream_ptr())
    if cat is not None:
        full = dense_x3s(x_rows, cat["w1f_x1"], cat["b1"], cat["w1f"].shape[1], relu=False, x1=True)
        return [full[:, o:o + w] for o, w in cat["cols"]]
    return [dense_x3s(x_rows, br["pre_x1"]["w1f_x1"], br["pre_x1"]["b1"], br["pre_x1"]["w1f"].shape[1],
                      relu=False, x1=True) for br in branches]


FUSE_LAYER1 = True  # backbones built while True fuse a bf16 level's per-point layer-1 GEMMs (A/B switch)


def fused_layer1_x1(branches):
    """The bf16-spec branches' per-point layer-1 weights side by side: {"w1f" (k, sum cp), "b1", "w1f_x1"
    (the packed image), "cols": [(column offset, cp) per branch]} — None for fewer than two branches."""
    if len(branches) < 2 or any("pre_x1" not in br for br in branches):
        return None
    ws = [br["pre_x1"]["w1f"] for br in branches]
    cols, o = [], 0
    for w in ws:
        cols.append((o, w.shape[1]))
        o += w.shape[1]
    w1f = torch.cat(ws, dim=1).contiguous()
    b1 = torch.cat([br["pre_x1"]["b1"] for br in branches]).contiguous()
    return {"w1f": w1f, "b1": b1, "w1f_x1": pack_dense_x3(w1f, x1=True), "cols": cols}


def group_mlp_x3(p, q, idx, n, packed, widths, out, out_offset=0, xyz_level=False):
    """group_mlp16 with layers 2-3 in h3 arithmetic (scaled fp16 hi/lo pieces on the fp16 MFMAs,
    fp32-class products, see sa_mlp_x3.hip)."""
    B, M, ns = idx.shape
    c1, c2, c3 = widths
    stride = 3 if xyz_level else p.shape[1]
    if xyz_level and not (p.is_contiguous() and q.is_contiguous()):
        raise ValueError("group_mlp_x3: xyz / centres must be contiguous")
    if not xyz_level and (p.shape[0] < B * n or q.shape[0] < B * M or p.shape[1] < c1 or q.shape[1] != p.shape[1]):
        raise ValueError("group_mlp_x3: p/q shapes do not match the batch")
    _dev_check(p, q, idx, packed, out)
    nat.call("lidar_sa_group_mlp_x3_f32", nat.handle(p.device.index), int(xyz_level), nat.ptr(p), stride,
             nat.ptr(q), nat.ptr(idx), B, n, M, ns, c1, c2, c3, nat.ptr(packed), nat.ptr(out), out.shape[-1],
             out_offset, nat.stream_ptr())
    return out


def group_mlp_bq(xyz, centres, grid, radius, nsample, packed, widths, out, out_offset=0, x1=False, out_idx=None):
    """One xyz-level SA branch with its ball queries answered inside the MLP kernel
    (lidar_sa_group_mlp_bq_f32): grid = ball_query_bin(radius, nsample, xyz, ...) of these
    frames; packed = the branch's x3 image (x1=False) or bf16-spec image (x1=True).  Equal bit
    for bit to ball_query(..., grid=grid) then group_mlp_x3 / group_mlp_x1; out_idx (B, M, ns)
    int32, optional, receives the ball-query indices."""
    B, n, _ = xyz.shape
    M = centres.shape[1]
    c1, c2, c3 = widths
    if not (xyz.is_contiguous() and centres.is_contiguous()):
        raise ValueError("group_mlp_bq: xyz / centres must be contiguous")
    if out_idx is not None and (tuple(out_idx.shape) != (B, M, nsample) or out_idx.dtype != torch.int32):
        raise ValueError("group_mlp_bq: out_idx must be (B, M, nsample) int32")
    _dev_check(xyz, centres, grid, packed, out, *([out_idx] if out_idx is not None else []))
    nat.call("lidar_sa_group_mlp_bq_f32", nat.handle(xyz.device.index), int(bool(x1)), nat.ptr(xyz), nat.ptr(grid),
             nat.ptr(centres), B, n, M, float(radius), int(nsample), c1, c2, c3, nat.ptr(packed), nat.ptr(out),
             out.shape[-1], out_offset, nat.ptr(out_idx) if out_idx is not None else None, nat.stream_ptr())
    return out


def generic_branch_weights(layers, cfeat, to_dev, arith):
    """Dense-GEMM operands of an SA branch of any shape (sa_branch_generic): layer 1's rows reordered
    from the canonical [x, y, z, f...] to the grouped rows' [f..., x, y, z, 0-pad] (k padded to 16),
    every layer's columns (and the next layer's rows) zero-padded to a multiple of 128.  arith: "x3"
    (h3 images), "x1" (bf16-spec images) or "f32" (the native fp32 GEMM's plain weights)."""
    kp = (cfeat + 3 + 15) // 16 * 16
    out = {"k": kp, "layers": [], "c3": layers[-1][0].shape[1], "arith": arith}
    kin = kp
    for li, (w, b) in enumerate(layers):
        w = np.asarray(w, np.float32)
        cin, c = w.shape
        cp = (c + 127) // 128 * 128
        wp = np.zeros((kin, cp), np.float32)
        if li == 0:
            wp[:cfeat, :c] = w[3:]
            wp[cfeat:cfeat + 3, :c] = w[:3]
        else:
            wp[:cin, :c] = w
        bp = np.zeros(cp, np.float32)
        bp[:c] = b
        wd = to_dev(wp)
        lay = {"w": wd, "b": to_dev(bp), "cout": cp}
        if arith != "f32":
            lay["packed"] = pack_dense_x3(wd, x1=arith == "x1")
        out["layers"].append(lay)
        kin = cp
    return out


def sa_branch_generic(feat, cfeat, xyz, centres, idx, gw, out, out_offset=0, max_bytes=1 << 30, slot=0):
    """One SA branch of any (widths, nsample) on the byte-moving kernels of csrc/sa_generic.hip and the
    dense GEMMs: grouped rows [f[idx], xyz[idx] - centre, 0-pad] -> per layer x W + b, ReLU (h3 / bf16
    spec / fp32 as gw["arith"]) -> max over each centre's nsample rows -> out[..., off:off + c3].
    feat: (B, n, >= cfeat) fp32 with unit column stride (None when cfeat = 0); idx (B, M, ns) int32
    (ball_query); gw = generic_branch_weights(...).  Frames run in chunks whose activations stay
    under max_bytes."""
    B, M, ns = idx.shape
    n = xyz.shape[1]
    if out.dim() != 3 or out.shape[0] != B or out.shape[1] != M or out.stride(2) != 1 or out.stride(1) != out.shape[2]:
        raise ValueError("sa_branch_generic: out must be a contiguous (B, M, stride) tensor")
    if out_offset < 0 or out_offset + gw["c3"] > out.shape[2]:
        raise ValueError("sa_branch_generic: out columns out of range")
    if cfeat and (feat is None or feat.shape[0] != B or feat.shape[1] != n or feat.shape[2] < cfeat
                  or feat.stride(2) != 1 or feat.stride(0) != n * feat.stride(1)):
        raise ValueError("sa_branch_generic: feat must be (B, n, >= cfeat) with rows of one stride")
    if not (xyz.is_contiguous() and centres.is_contiguous() and idx.is_contiguous()):
        raise ValueError("sa_branch_generic: xyz / centres / idx must be contiguous")
    _dev_check(xyz, centres, idx, out)
    if cfeat and not feat.is_cuda:  # strided rows (checked above), not necessarily contiguous
        raise ValueError("sa_branch_generic: feat must be a CUDA tensor")
    dev = xyz.device
    h = nat.handle(dev.index, slot)
    kp = gw["k"]
    cmax = max([kp] + [lay["cout"] for lay in gw["layers"]])
    fc = max(1, min(B, max_bytes // max(1, 2 * M * ns * cmax * 4)))
    ldf = feat.stride(1) if cfeat else 0
    for b0 in range(0, B, fc):
        nb = min(B, b0 + fc) - b0
        grouped = nb * M * ns
        R = (grouped + 127) // 128 * 128
        rows = torch.empty((R, kp), dtype=torch.float32, device=dev)
        nat.call("lidar_sa_group_rows_f32", h, nat.ptr(feat[b0:b0 + nb]) if cfeat else None, ldf, cfeat,
                 nat.ptr(xyz[b0:b0 + nb]), nat.ptr(centres[b0:b0 + nb]), nat.ptr(idx[b0:b0 + nb]), nb, n, M, ns,
                 nat.ptr(rows), R, kp, nat.stream_ptr())
        a = rows
        for lay in gw["layers"]:
            if gw["arith"] == "f32":
                a = dense(a, lay["w"], lay["b"], relu=True)
            else:
                a = dense_x3s(a, lay["packed"], lay["b"], lay["cout"], relu=True, x1=gw["arith"] == "x1", slot=slot)
        dst = out[b0:b0 + nb]
        nat.call("lidar_group_max_f32", h, nat.ptr(a), a.shape[1], nb * M, ns, gw["c3"], nat.ptr(dst),
                 out.shape[2], out_offset, nat.stream_ptr())
    return out


def layer1_weights(layer, cfeat, to_dev):
    """(W1 (3 + cfeat, c1), b1) -> the per-point GEMM operands of layer1_per_point:
    w1 rows [f..., x, y, z, 0-pad] (k padded to 16), wq rows [x, y, z, 0-pad] (16), columns
    zero-padded to a multiple of 128 (the dense kernel's tile)."""
    w1, b1 = layer
    c1 = w1.shape[1]
    kp = (cfeat + 3 + 15) // 16 * 16
    cp = (c1 + 127) // 128 * 128
    w1p = np.zeros((kp, cp), np.float32)
    w1p[:cfeat, :c1] = w1[3:]
    w1p[cfeat:cfeat + 3, :c1] = w1[:3]
    wq = np.zeros((16, cp), np.float32)
    wq[:3, :c1] = w1[:3]
    bp = np.zeros(cp, np.float32)
    bp[:c1] = b1
    return {"w1": to_dev(w1p), "b1": to_dev(bp), "wq": to_dev(wq), "zero": to_dev(np.zeros(cp, np.float32))}


def centre_layer1(new_xyz, branches, out=None, slot=0):
    """Q = [c, 0-pad] W1_xyz' per centre of a feature level, every branch (the per-centre half of
    layer1_per_point, h3 GEMM; rows B*M rounded up to 128) -> [Q per branch].  out: [(cpad (R, 16) zeroed
    past the centres' rows, Q (R, cp))] per branch, preallocated."""
    B, M, _ = new_xyz.shape
    dev = new_xyz.device
    h = nat.handle(dev.index, slot)
    rq = (B * M + 127) // 128 * 128
    res = []
    for i, br in enumerate(branches):
        pre = br["pre"]
        cp = pre["w1"].shape[1]
        cpad, q = out[i] if out is not None else (torch.zeros((rq, 16), dtype=torch.float32, device=dev), None)
        cpad, q = cpad[:rq], (q[:rq] if q is not None else None)
        nat.call("lidar_concat_xyz_pad_f32", h, nat.ptr(new_xyz), B * M, nat.ptr(cpad), 16, 0, nat.stream_ptr())
        res.append(dense_x3s(cpad, pre["wq_x3"], pre["zero"], cp, relu=False, out=q, slot=slot))
    return res


def layer1_per_point(x_rows, xyz, cfeat, new_xyz, branches, x3=True):
    """Layer 1 of every branch of a level, per point instead of per grouped row.

    x_rows: (R, kp) padded rows [f (cfeat), x, y, z, 0...] of the level's B*N points
    (R = B*N rounded up to 128; the previous level wrote f in place), xyz (B, N, 3);
    new_xyz (B, M, 3).  Returns per branch (P, Q): P = x_rows W1' + b1 (R, c1),
    Q = [c, 0] W1_xyz' (B*M rounded to 128, c1), both without ReLU (columns padded to a
    multiple of 128 with zero weights).  x3: on the h3 GEMM (fp32 rows in, scaled and split in the
    tile loop); else the native fp32 MFMA GEMM."""
    B, N, _ = xyz.shape
    M = new_xyz.shape[1]
    R, kp = x_rows.shape
    dev = xyz.device
    h = nat.handle(dev.index)
    nat.call("lidar_concat_xyz_pad_f32", h, nat.ptr(xyz), B * N, nat.ptr(x_rows), kp, cfeat, nat.stream_ptr())
    if x3:
        qs = centre_layer1(new_xyz, branches)
        return [(dense_x3s(x_rows, br["pre"]["w1_x3"], br["pre"]["b1"], br["pre"]["w1"].shape[1], relu=False), q)
                for br, q in zip(branches, qs)]
    rq = (B * M + 127) // 128 * 128
    cpad = torch.zeros((rq, 16), dtype=torch.float32, device=dev)
    nat.call("lidar_concat_xyz_pad_f32", h, nat.ptr(new_xyz), B * M, nat.ptr(cpad), 16, 0, nat.stream_ptr())
    return [(dense(x_rows, br["pre"]["w1"], br["pre"]["b1"], relu=False),
             dense(cpad, br["pre"]["wq"], br["pre"]["zero"], relu=False)) for br in branches]


def pack_dense_x3(w, x1=False):
    """(k, cout) fp32 CUDA weights -> the dense GEMM's packed image (device): the h3 image (fp16 hi /
    lo of W 2^s, lidar_dense_x3_pack_f32) or, x1, the bf16 spec's image (lidar_dense_x1_pack_f32)."""
    _dev_check(w)
    k, cout = w.shape
    nbytes = nat.load_library().lidar_dense_x3_packed_size(k, cout)
    out = torch.empty((nbytes,), dtype=torch.uint8, device=w.device)
    nat.call("lidar_dense_x1_pack_f32" if x1 else "lidar_dense_x3_pack_f32", nat.handle(w.device.index), nat.ptr(w),
             k, cout, nat.ptr(out), nat.stream_ptr())
    return out


def dense(x, w, b, relu=True, pool_rows=0, out=None):
    """x (rows, k) @ w (k, cout) + b [-> ReLU] [-> max over runs of pool_rows rows] on the native
    fp32 matrix cores (lidar_dense_f32)."""
    rows, k = x.shape
    cout = w.shape[1]
    if out is None:
        shape = (rows // pool_rows, cout) if pool_rows else (rows, cout)
        out = (torch.zeros if pool_rows else torch.empty)(shape, dtype=torch.float32, device=x.device)
    _dev_check(x, w, b, out)
    nat.call("lidar_dense_f32", nat.handle(x.device.index), nat.ptr(x), rows, k, nat.ptr(w), nat.ptr(b), cout,
             1 if relu else 0, pool_rows, nat.ptr(out), nat.stream_ptr())
    return out


def dense_relu(x, w, b, pool_rows=0, out=None):
    return dense(x, w, b, True, pool_rows, out)


def dense_x3s(a, wpack, b, cout, relu=True, pool_rows=0, out=None, x1=False, slot=0):
    """a (rows, k) fp32 @ W + b on the dense GEMM of csrc/dense_x3s.hip (lidar_dense_x3f_f32; wpack =
    pack_dense_x3(W), h3 arithmetic; x1: pack_dense_x3(W, x1=True), the bf16 spec).  Returns fp32
    rows (rows, cout) or, with pool_rows, the fp32 max over runs of pool_rows rows (ReLU)."""
    rows, lda = a.shape
    dev = a.device
    if pool_rows:
        mode = 2
        if out is None:
            out = torch.zeros((rows // pool_rows, cout), dtype=torch.float32, device=dev)
    else:
        mode = 0
        if out is None:
            out = torch.empty((rows, cout), dtype=torch.float32, device=dev)
    _dev_check(a, wpack, b, out)
    nat.call("lidar_dense_x3f_f32", nat.handle(dev.index, slot), nat.ptr(a), lda, rows, lda, nat.ptr(wpack), nat.ptr(b),
             cout, mode | (4 if x1 else 0), 1 if relu else 0, pool_rows, nat.ptr(out), 0, out.shape[1],
             nat.stream_ptr())
    return out


def h3_bounds(w, b):
    """(w_colsum, b_max) of a dense layer for lidar_dense_h3p_f32's mode-1 exponent bound: the largest
    column sum of |W| and the largest |b|, each rounded up to the next float32."""
    cs = np.abs(np.asarray(w, np.float64)).sum(axis=0).max() if np.size(w) else 0.0
    bm = np.abs(np.asarray(b, np.float64)).max() if np.size(b) else 0.0
    up = lambda v: float(np.nextafter(np.float32(v), np.float32(np.inf)))
    return up(cs), up(bm)


def dense_h3p(a, a_exp, wpack, b, cout, mode, bounds=(0.0, 0.0), relu=True, pool_rows=0, out=None):
    """One layer of group_all's h3 chain (lidar_dense_h3p_f32).  A: fp32 rows (rows, k) with a_exp None,
    or h3 planes (2, rows, k) float16 (hi, lo) with a_exp (rows,) int32 — mode 1's output.  mode 0 ->
    fp32 rows (rows, cout); 1 -> (planes (2, rows, cout) float16, exponents (rows,) int32), the next
    layer's A; 2 -> ReLU + max over runs of pool_rows rows (rows / pool_rows, cout) fp32.  bounds: the
    layer's h3_bounds(W, b) (mode 1)."""
    dev = a.device
    # the two operand forms are told apart only by a_exp: check that the tensors match the form, so a
    # mismatch raises instead of being reinterpreted by the kernel
    if a_exp is None:
        if a.dtype != torch.float32 or a.dim() != 2:
            raise ValueError(f"dense_h3p: fp32 rows (rows, k) expected without a_exp, got {a.dtype} {tuple(a.shape)}")
        rows, k = a.shape
    else:
        if a.dtype != torch.float16 or a.dim() != 3 or a.shape[0] != 2:
            raise ValueError(f"dense_h3p: h3 planes (2, rows, k) float16 expected with a_exp, got {a.dtype} "
                             f"{tuple(a.shape)}")
        _, rows, k = a.shape
        if a_exp.dtype != torch.int32 or tuple(a_exp.shape) != (rows,):
            raise ValueError(f"dense_h3p: a_exp must be int32 of shape ({rows},), got {a_exp.dtype} "
                             f"{tuple(a_exp.shape)}")
    lda = k
    if mode not in (0, 1, 2):
        raise ValueError(f"dense_h3p: mode must be 0, 1 or 2, got {mode}")
    if mode == 2 and (pool_rows <= 0 or rows % pool_rows):
        raise ValueError(f"dense_h3p: pool_rows ({pool_rows}) must divide rows ({rows})")
    if mode == 2:
        out = torch.zeros((rows // pool_rows, cout), dtype=torch.float32, device=dev) if out is None else out
        oexp = None
    elif mode == 1:
        out = torch.empty((2, rows, cout), dtype=torch.float16, device=dev) if out is None else out
        oexp = torch.empty(rows, dtype=torch.int32, device=dev)
    else:
        out = torch.empty((rows, cout), dtype=torch.float32, device=dev) if out is None else out
        oexp = None
    _dev_check(a, a_exp, wpack, b, out, oexp)
    nat.call("lidar_dense_h3p_f32", nat.handle(dev.index), nat.ptr(a), lda, rows, k, nat.ptr(a_exp), nat.ptr(wpack),
             nat.ptr(b), cout, mode, 1 if relu else 0, pool_rows, nat.ptr(out), nat.ptr(oexp), cout, float(bounds[0]),
             float(bounds[1]), nat.stream_ptr())
    return (out, oexp) if mode == 1 else out


# ----------------------------------------------------------------------- backbone
class _Timers:
    """Optional per-launch HIP-event timing on the launching stream (bench.py): per kernel name
    the launches made, each with the number of frames it processed."""

    def __init__(self):
        self.ev = {}

    def __call__(self, name, frames, fn, *a, **k):
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        out = fn(*a, **k)
        e1.record(s)
        self.ev.setdefault(name, []).append((e0, e1, int(frames)))
        return out

    def totals(self):
        """{name: (launches, frames over all launches, total ms)} (waits for the events)."""
        return {k: (len(v), sum(f for _, _, f in v), sum(a.elapsed_time(b) for a, b, _ in v))
                for k, v in self.ev.items()}

    def mean_ms(self):
        return {k: t / n for k, (n, _, t) in self.totals().items()}


def _call(timers, name, frames, fn, *a, **k):
    return timers(name, frames, fn, *a, **k) if timers is not None else fn(*a, **k)


class PointNet2Backbone:
    """SSG / MSG PointNet++ encoder on liblidar_amd.  ``forward(xyz)`` -> global feature
    (B, C_last) plus, with keep_levels, per level (new_xyz, features, fps_idx, [ball-query
    idx per branch])."""

    def __init__(self, cfg=SSG, weights=None, device="cuda", seed=0, dtype="f32", x3=True):
        """dtype "f32" (the fp32 contract: features within 1e-4 of the fp32 oracle): x3=True (default)
        runs the MLPs on the fp16 matrix cores in h3 arithmetic (lidar_sa_group_mlp_x3_f32,
        lidar_dense_x3f_f32), x3=False on the native fp32 matrix cores (lidar_sa_group_mlp16_f32,
        lidar_dense_f32) — the strict-fp32 path.
        dtype "bf16" (BASELINE configs[4]): the SA branches in the bf16 spec on the X1 kernels
        (inputs, activations and weights rounded to bf16, fp32 accumulation); group_all stays in
        fp32 arithmetic on the x3 GEMM.
        Levels with point features run layer 1 per point (layer1_per_point / layer1_points_x1) and
        the fused kernel from layer 2 on.

        cfg: any SSG / MSG configuration (levels of radii / nsamples / mlps with three layers per
        branch, then optionally group_all).  The fused branch kernels are instantiated for the six
        (xyz level, c1, c2, c3, nsample) shapes of MLP16_SHAPES (the SSG / MSG configurations of
        SURVEY §8a); a branch of any other shape runs sa_branch_generic — its grouped rows
        materialised in HBM, the same dense GEMMs (same arithmetic: h3, bf16 spec or fp32), then the
        max over nsample — with the same results contract and HBM-bound speed."""
        if dtype not in ("f32", "bf16"):
            raise ValueError("dtype must be 'f32' or 'bf16'")
        self.bf16 = dtype == "bf16"
        self.x3 = bool(x3) or self.bf16  # the dense GEMMs (per-point layer 1, group_all)
        self.cfg = cfg
        self.device = torch.device(device)
        self.weights = weights if weights is not None else init_weights(cfg, seed)
        self.levels = []
        cfeat = 0
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(self.device)
        for lvl, wl in zip(cfg["levels"], self.weights):
            kp = (cfeat + 3 + 15) // 16 * 16
            if lvl.get("group_all"):
                (w1, b1), (w2, b2), (w3, b3) = wl[0]
                # canonical rows [x, y, z, f...] -> physical input [f..., x, y, z, 0-pad]; every
                # width zero-padded to the GEMM's 128 columns (and the next layer's rows)
                cp = [(w.shape[1] + 127) // 128 * 128 for w in (w1, w2, w3)]
                w1p = np.zeros((kp, cp[0]), np.float32)
                w1p[:cfeat, :w1.shape[1]] = w1[3:]
                w1p[cfeat:cfeat + 3, :w1.shape[1]] = w1[:3]
                w2p = np.zeros((cp[0], cp[1]), np.float32)
                w2p[:w2.shape[0], :w2.shape[1]] = w2
                w3p = np.zeros((cp[1], cp[2]), np.float32)
                w3p[:w3.shape[0], :w3.shape[1]] = w3
                bp = [np.pad(np.asarray(bb_, np.float32), (0, c - len(bb_))) for bb_, c in zip((b1, b2, b3), cp)]
                entry = {"group_all": True, "k": kp, "cfeat": cfeat, "cout": w3.shape[1],
                         "w": [t(w1p), t(w2p), t(w3p)], "b": [t(v) for v in bp]}
                if self.x3:  # packed once into x3 B fragments
                    entry["w_x3"] = [pack_dense_x3(w) for w in entry["w"]]
                    entry["h3_bounds"] = [h3_bounds(w1p, bp[0]), h3_bounds(w2p, bp[1]), h3_bounds(w3p, bp[2])]
                self.levels.append(entry)
                cfeat = w3.shape[1]
                continue
            xyz_level = cfeat == 0
            branches = []
            for (r, ns, widths, layers) in zip(lvl["radii"], lvl["nsamples"], lvl["mlps"], wl):
                br = {"r": r, "ns": ns, "widths": widths}
                if (xyz_level, *widths, ns) not in MLP16_SHAPES:
                    # no fused kernel for this shape: grouped rows in HBM + the dense GEMMs (sa_branch_generic)
                    arith = "x1" if self.bf16 else ("x3" if x3 else "f32")
                    br["generic"] = generic_branch_weights(layers, cfeat, t, arith)
                elif self.bf16:
                    br["packed_x1"] = torch.from_numpy(pack_branch_x1(layers)).to(self.device)
                    if not xyz_level:  # W1_f: rows [f..., (x, y, z) = 0, 0-pad], columns to 128
                        w1, b1 = layers[0]
                        cp = (w1.shape[1] + 127) // 128 * 128
                        w1f = np.zeros((kp, cp), np.float32)
                        w1f[:cfeat, :w1.shape[1]] = w1[3:]
                        b1p = np.zeros(cp, np.float32)
                        b1p[:w1.shape[1]] = b1
                        br["pre_x1"] = {"w1f": t(w1f), "b1": t(b1p)}
                        br["pre_x1"]["w1f_x1"] = pack_dense_x3(br["pre_x1"]["w1f"], x1=True)
                else:
                    if x3:
                        br["packed_x3"] = torch.from_numpy(pack_branch_x3(layers, xyz_level)).to(self.device)
                    else:
                        br["packed16"] = torch.from_numpy(pack_branch16(layers, xyz_level)).to(self.device)
                    if not xyz_level:
                        br["pre"] = layer1_weights(layers[0], cfeat, t)
                        if x3:
                            br["pre"]["w1_x3"] = pack_dense_x3(br["pre"]["w1"])
                            br["pre"]["wq_x3"] = pack_dense_x3(br["pre"]["wq"])
                branches.append(br)
            entry = {"div": lvl["npoint_div"], "branches": branches, "cfeat": cfeat}
            if not xyz_level:  # the previous level writes this level's padded rows [f, x, y, z, 0]
                entry.update(pre=True, k=kp)
                if self.bf16 and FUSE_LAYER1 and all("pre_x1" in br for br in branches):
                    entry["pre_x1_cat"] = fused_layer1_x1(branches)  # one layer-1 GEMM for every branch
            self.levels.append(entry)
            cfeat = sum(w[-1] for w in lvl["mlps"])
        self.out_channels = cfeat
        self.timers = None  # set to a _Timers() to time every launch

    def _grid_buffer(self, B, N, device):
        """The ball-query grid buffer forward() bins xyz levels into (grown on demand, reused by
        every branch and call on this backbone's stream)."""
        need = nat.load_library().lidar_ball_query_grid_bytes(B, N)
        if getattr(self, "_grid", None) is None or self._grid.numel() < need:
            self._grid = torch.empty((max(1, need),), dtype=torch.uint8, device=device)
        return self._grid

    def forward_from_sa1_fps(self, xyz, idx1, new_xyz1, fz1, gidx1=None, keep_levels=False, grids1=None, pre2=None):
        """forward() with level 0's FPS (and its ball queries: gidx1, or their binning: grids1)
        already computed (StreamingSSG); pre2: level 1's {"fps": ..., "bq": ...} likewise."""
        pre = {0: {"fps": (idx1, new_xyz1, fz1), "bq": gidx1, "grid": grids1}}
        if pre2 is not None:
            pre[1] = pre2
        return self.forward(xyz, keep_levels, pre=pre)

    def forward(self, xyz, keep_levels=False, pre=None):
        """pre: {level: {"fps": (idx, new_xyz, first_zero), "bq": [gidx per branch] | "grid": [ball_query_bin
        buffer per branch]}} — work already done for those levels (StreamingSSG's side streams);
        every other step runs here."""
        pre = pre or {}
        B, N, _ = xyz.shape
        N0 = N  # npoint_div is relative to the input frame (N/16, N/64)
        feats = None
        rows = None  # flat padded (R, k) rows behind `feats` when the next level reads them
        out_levels = []
        fz = None  # previous level's FPS first_zero (nested-FPS shortcut)
        t = self.timers
        for li, lvl in enumerate(self.levels):
            if lvl.get("group_all"):
                g = self._group_all(xyz, feats, lvl, rows)
                return (g if g.shape[1] == lvl["cout"] else g[:, :lvl["cout"]].contiguous()), out_levels
            M = max(1, N0 // lvl["div"])
            pl = pre.get(li, {})
            if pl.get("fps") is not None:
                idx, new_xyz, nfz = pl["fps"]
            else:
                nfz = torch.empty(B, dtype=torch.int32, device=xyz.device)
                idx, new_xyz = _call(t, f"sa{li + 1}_fps", B, farthest_point_sample, xyz, M, return_xyz=True,
                                     first_zero=nfz, prefix_ok=fz)
            fz = nfz
            ctot = sum(br["widths"][-1] for br in lvl["branches"])
            nxt = self.levels[li + 1] if li + 1 < len(self.levels) else None
            # a level feeding group_all or a per-point layer 1 writes straight into the
            # next level's padded input rows [f, x, y, z, 0-pad] (R = B*M rounded to 128)
            padded = nxt is not None and (nxt.get("group_all") or nxt.get("pre"))
            stride = nxt["k"] if padded else ctot
            R = (B * M + 127) // 128 * 128 if padded else B * M
            out_rows = torch.empty((R, stride), dtype=torch.float32, device=xyz.device)
            out = out_rows[:B * M].view(B, M, stride)
            pq = None  # per-point layer 1 of the fused branches: {branch index: rows}
            fb = [i for i, br in enumerate(lvl["branches"]) if "generic" not in br]
            if lvl.get("pre") and fb:
                fbr = [lvl["branches"][i] for i in fb]
                if self.bf16:
                    cat = lvl.get("pre_x1_cat") if len(fbr) == len(lvl["branches"]) else None
                    res = _call(t, f"sa{li + 1}_layer1_points", B, layer1_points_x1, rows, xyz, lvl["cfeat"], fbr,
                                cat=cat)
                else:
                    res = _call(t, f"sa{li + 1}_layer1_points", B, layer1_per_point, rows, xyz, lvl["cfeat"],
                                new_xyz, fbr, x3=self.x3)
                pq = dict(zip(fb, res))
            off = 0
            gidxs = []
            for bi_, br in enumerate(lvl["branches"]):
                tag = f"sa{li + 1}" + (f"_b{bi_}" if len(lvl["branches"]) > 1 else "")
                # work done elsewhere for this branch (StreamingSSG's side streams): its ball-query
                # indices, or the binning of its frames (None per branch: not done)
                pb = pl["bq"][bi_] if pl.get("bq") is not None else None
                pg = pl["grid"][bi_] if pl.get("grid") is not None else None
                if "generic" in br:
                    if pb is not None:
                        gidx = pb
                    else:
                        gidx = _call(t, f"{tag}_ball_query", B, ball_query, br["r"], br["ns"], xyz, new_xyz,
                                     grid=pg)
                    gidxs.append(gidx)
                    _call(t, f"{tag}_group_mlp", B, sa_branch_generic, feats, lvl["cfeat"], xyz, new_xyz, gidx,
                          br["generic"], out, off)
                    off += br["widths"][-1]
                    continue
                fused = pq is None and pb is None and (self.bf16 or "packed_x3" in br) and (
                    pg is not None or N >= BQ_GRID_MIN_N)
                if fused:
                    # xyz level: the MLP kernel answers the ball queries from the frame's grid
                    if pg is not None:
                        grid = pg
                    else:
                        grid = _call(t, f"{tag}_bq_bin", B, ball_query_bin, br["r"], br["ns"], xyz,
                                     self._grid_buffer(B, N, xyz.device))
                    gidx = (torch.empty((B, M, br["ns"]), dtype=torch.int32, device=xyz.device)
                            if keep_levels else None)
                    _call(t, f"{tag}_group_mlp", B, group_mlp_bq, xyz, new_xyz, grid, br["r"], br["ns"],
                          br["packed_x1"] if self.bf16 else br["packed_x3"], br["widths"], out=out, out_offset=off,
                          x1=self.bf16, out_idx=gidx)
                    gidxs.append(gidx)
                    off += br["widths"][-1]
                    continue
                if pb is not None:
                    gidx = pb
                else:
                    gidx = _call(t, f"{tag}_ball_query", B, ball_query, br["r"], br["ns"], xyz, new_xyz, grid=pg)
                gidxs.append(gidx)
                if self.bf16:
                    if pq is not None:
                        _call(t, f"{tag}_group_mlp", B, group_mlp_x1, pq[bi_], gidx, N, br["packed_x1"],
                              br["widths"], out=out, out_offset=off, xyz=xyz, centres=new_xyz)
                    else:
                        _call(t, f"{tag}_group_mlp", B, group_mlp_x1, xyz, gidx, N, br["packed_x1"],
                              br["widths"], out=out, out_offset=off, centres=new_xyz)
                else:
                    p16, q16 = (pq[bi_] if pq is not None else (xyz, new_xyz))
                    kern = group_mlp_x3 if "packed_x3" in br else group_mlp16
                    _call(t, f"{tag}_group_mlp", B, kern, p16, q16, gidx, N,
                          br["packed_x3"] if "packed_x3" in br else br["packed16"], br["widths"], out=out,
                          out_offset=off, xyz_level=pq is None)
                off += br["widths"][-1]
            if keep_levels:
                out_levels.append((new_xyz, out[..., :ctot], idx, gidxs))
            xyz, feats, rows = new_xyz, (out[..., :ctot] if padded else out), out_rows
            N = M
        return feats, out_levels

    def _group_all(self, xyz, feats, lvl, rows=None):
        B, M, _ = xyz.shape
        kp, cfeat = lvl["k"], lvl["cfeat"]
        # the previous level wrote its features into padded rows [f, x, y, z, 0-pad]
        x = rows[:B * M].view(B, M, kp) if rows is not None and rows.shape[1] == kp else None
        if x is None:  # previous level did not pre-pad (only when group_all is level 0)
            x = torch.empty((B, M, kp), dtype=torch.float32, device=xyz.device)
            if feats is not None:
                x[..., :cfeat] = feats
        nat.call("lidar_concat_xyz_pad_f32", nat.handle(xyz.device.index), nat.ptr(xyz), B * M,
                 nat.ptr(x), kp, cfeat, nat.stream_ptr())
        rows = B * M
        x2 = x.view(rows, kp)
        if M % 128:
            # the MFMA tiles want 128-row runs: pad each frame with copies of its first row
            # (the max-pool is invariant to duplicated rows)
            mp = (M + 127) // 128 * 128
            sel = torch.cat([torch.arange(M, device=x.device),
                             torch.zeros(mp - M, dtype=torch.long, device=x.device)])
            x2 = x.view(B, M, kp)[:, sel].reshape(B * mp, kp).contiguous()
            M, rows = mp, B * mp
        t = self.timers
        ws, bs = lvl["w"], lvl["b"]
        if self.x3 and not hasattr(nat.load_library(), "lidar_dense_h3p_f32"):
            # an earlier round's library (A/B through LIDAR_AMD_LIB): fp32 rows between the layers
            wp = lvl["w_x3"]
            h1 = _call(t, "sa3_dense1", B, dense_x3s, x2, wp[0], bs[0], ws[0].shape[1])
            h2 = _call(t, "sa3_dense2", B, dense_x3s, h1, wp[1], bs[1], ws[1].shape[1])
            return _call(t, "sa3_dense3_pool", B, dense_x3s, h2, wp[2], bs[2], ws[2].shape[1], pool_rows=M)
        if self.x3:  # h3 planes between the layers (split once, by the producer); dense3 fuses the max-pool
            wp, bd = lvl["w_x3"], lvl["h3_bounds"]
            h1, e1 = _call(t, "sa3_dense1", B, dense_h3p, x2, None, wp[0], bs[0], ws[0].shape[1], 1, bd[0])
            h2, e2 = _call(t, "sa3_dense2", B, dense_h3p, h1, e1, wp[1], bs[1], ws[1].shape[1], 1, bd[1])
            return _call(t, "sa3_dense3_pool", B, dense_h3p, h2, e2, wp[2], bs[2], ws[2].shape[1], 2, pool_rows=M)
        h1 = _call(t, "sa3_dense1", B, dense_relu, x2, ws[0], bs[0])
        h2 = _call(t, "sa3_dense2", B, dense_relu, h1, ws[1], bs[1])
        out = torch.zeros((rows // M, ws[2].shape[1]), dtype=torch.float32, device=x.device)
        return _call(t, "sa3_dense3_pool", B, dense_relu, h2, ws[2], bs[2], pool_rows=M, out=out)

    __call__ = forward


# ------------------------------------------------------------------ streaming executor
class StreamingSSG:
    """Frame-batch pipeline for a continuous feed (SSG/MSG backbone).

    SA1's farthest-point sampling is a serial chain of N/16 argmax steps per frame
    (latency-bound, one workgroup per frame), while everything after it (fused MFMA MLPs,
    SA2's nested FPS and ball queries, group_all) fills the whole GPU.  Later batches' SA1 FPS
    and level-0 ball queries therefore run on `depth` side streams (own library handles /
    workspaces) while earlier batches' remaining levels run on the main stream; events order
    the hand-off and a ring of `slots` (default depth + 3) staging slots bounds memory.

    fps_group = G > 1: G consecutive batches are staged into one (G*B, N, 3) buffer; one
    side-stream launch runs their SA1 FPS (G*B workgroups share the serial chain of steps
    without needing more streams than the device's hardware queues) and one main-stream
    pass runs their MFMA levels (larger launches fill the chip better).  Every operator is
    per frame, so results are identical to ``PointNet2Backbone.forward`` per batch.

    ``run(batches)`` processes a finite list (pipeline fill and drain included); ``feed()``
    returns a persistent feed whose ``push(batch)`` keeps `depth` groups in flight (the steady
    state of a LiDAR stream) and ``flush()`` drains it.
    """

    def __init__(self, backbone, batch, n, depth=1, fps_group=1, fps_threads=0, side_priority=0,
                 ramp=True,
                 reserve=True, keep_levels=False, slots=None, bq="bin", l2_side=False):
        """fps_threads: SA1 FPS workgroup size (0 = 1024; 512: half the CU footprint beside the
        MLPs).  ramp: in run(), the first groups hold 1, 2, ... batches (a shorter pipeline fill).
        slots: staging slots (>= depth + 1; default depth + 3).  Group k's FPS reuses the slot of
        group k - slots, so it waits for that group's main-stream pass: with depth + 1 slots the
        side chain could only start a group once the main stream was `depth` groups behind it,
        which left the main stream idle whenever FPS took about `depth` main passes.
        keep_levels: every output is (global feature, per-level (new_xyz, features, fps idx,
        [ball-query idx per branch])) instead of the global feature alone.  l2_side: level 1's FPS
        (nested: the prefix shortcut over SA1's centroids) and ball queries depend only on SA1's
        FPS output, so they run on the side stream too (the main stream then runs only MLP work
        and level 1's per-point layer 1).

        Host frames: feed().push_host(frames) takes a batch of host NumPy frames, stages it in
        pinned memory (parallel host threads) and copies it to the device on the group's side
        stream ahead of its FPS (the PCIe-inclusive feed; results equal push() of the same data)."""
        self.bb = backbone
        self.B, self.N, self.depth, self.G = batch, n, depth, max(1, int(fps_group))
        self.ramp = bool(ramp)
        self.fps_threads = int(fps_threads)
        self.keep = bool(keep_levels)
        if bq not in ("side", "bin", "main"):
            raise ValueError("StreamingSSG: bq must be 'side', 'bin' or 'main'")
        self.bq = bq
        dev = backbone.device
        lvl0 = backbone.levels[0]
        self.M1 = max(1, n // lvl0["div"])
        # side_priority < 0 puts the latency-bound FPS chains ahead of the MLP waves in the
        # dispatcher (HIP stream priority); results do not depend on it
        # the process's shared side streams: a pipeline created after another keeps its queues
        # (streams.py: fresh streams can land on the main stream's hardware queue)
        self.fps_streams = side_streams(dev, depth, priority=side_priority)
        nslot = depth + 3 if slots is None else int(slots)
        if nslot < depth + 1:
            raise ValueError("StreamingSSG: slots must be >= depth + 1")
        self.nslot = nslot
        GB = self.G * batch
        self.stage = [torch.empty((GB, n, 3), dtype=torch.float32, device=dev) if self.G > 1 else None
                      for _ in range(nslot)]
        self.staged = [self.G > 1] * nslot  # the slot's group lives in stage[slot] (else in the caller's batch)
        self.idx = [torch.empty((GB, self.M1), dtype=torch.int32, device=dev) for _ in range(nslot)]
        self.cxyz = [torch.empty((GB, self.M1, 3), dtype=torch.float32, device=dev) for _ in range(nslot)]
        self.fz = [torch.empty(GB, dtype=torch.int32, device=dev) for _ in range(nslot)]
        # level-0 ball-query indices computed on the side streams (bq="side"; with "bin" the MLP kernel
        # answers them from the side streams' grids)
        self.side_q = [bq == "side" for br in lvl0["branches"]]
        self.gidx = [[torch.empty((GB, self.M1, br["ns"]), dtype=torch.int32, device=dev) if sq else None
                      for br, sq in zip(lvl0["branches"], self.side_q)]
                     for _ in range(nslot)] if any(self.side_q) else None
        self.grid = [[ball_query_grid_buffer(GB, n, dev) for br in lvl0["branches"]]
                     for _ in range(nslot)] if bq == "bin" else None
        lvl1 = backbone.levels[1] if len(backbone.levels) > 1 else None
        self.l2 = bool(l2_side) and lvl1 is not None and not lvl1.get("group_all")
        if self.l2:
            self.M2 = max(1, n // lvl1["div"])
            self.idx2 = [torch.empty((GB, self.M2), dtype=torch.int32, device=dev) for _ in range(nslot)]
            self.cxyz2 = [torch.empty((GB, self.M2, 3), dtype=torch.float32, device=dev) for _ in range(nslot)]
            self.fz2 = [torch.empty(GB, dtype=torch.int32, device=dev) for _ in range(nslot)]
            self.gidx2 = [[torch.empty((GB, self.M2, br["ns"]), dtype=torch.int32, device=dev)
                           for br in lvl1["branches"]] for _ in range(nslot)]
        # setup-time workspace sizing of the side handles (FPS + ball queries), so no stage's
        # first call grows a workspace (lidar_reserve; growth retires the old block, no device sync)
        if reserve:
            lib = nat.load_library()
            need = max(lib.lidar_fps_workspace_bytes(GB, n), lib.lidar_ball_query_grid_bytes(GB, n))
            for sl in range(1, depth + 1):
                nat.call("lidar_reserve", nat.handle(dev.index, sl), need)
        self.fps_done = [torch.cuda.Event() for _ in range(nslot)]
        self.slot_free = [torch.cuda.Event() for _ in range(nslot)]
        for e in self.slot_free:
            e.record(torch.cuda.current_stream(dev))

    def _stage(self, slot, fs, main):
        """The slot's staging buffer (allocated on first use when G = 1) — from the pool of the side stream
        that writes it: a block the caching allocator took from the main stream's pool could be one a
        main-stream pass still queued on the device has just freed, and the side stream does not wait
        for the main stream.  Main-stream passes read it too (record_stream: its block outlives them)."""
        if self.stage[slot] is None:
            with torch.cuda.stream(fs):
                st = torch.empty((self.G * self.B, self.N, 3), dtype=torch.float32, device=self.bb.device)
            st.record_stream(main)
            self.stage[slot] = st
        return self.stage[slot]

    def _fps(self, k, xs, ready, main=None):
        """SA1 FPS + level-0 ball queries of group k (the batches in xs, readable after the
        events in `ready`) on a side stream; `main` the stream the group's MFMA levels will run on."""
        slot = k % self.nslot
        fs = self.fps_streams[k % self.depth]
        hs = 1 + k % self.depth  # the side stream's own library handle
        fs.wait_event(self.slot_free[slot])
        for ev in ready:
            fs.wait_event(ev)
        g = len(xs) * self.B
        t = self.bb.timers
        host = any(isinstance(xj, _HostBatch) for xj in xs)
        self.staged[slot] = self.G > 1 or host
        if self.staged[slot]:
            self._stage(slot, fs, main if main is not None else torch.cuda.current_stream(self.bb.device))
        with torch.cuda.stream(fs):
            if self.staged[slot]:
                x = self.stage[slot][:g]
                B, j = self.B, 0
                grp = None
                while j < len(xs):
                    if isinstance(xs[j], _HostBatch):
                        # a run of host batches (consecutive rows of one pinned group buffer): one DMA copy
                        e = j
                        while e + 1 < len(xs) and isinstance(xs[e + 1], _HostBatch):
                            e += 1
                        grp = xs[j].grp
                        x[j * B:(e + 1) * B].copy_(grp.pinned[j * B:(e + 1) * B], non_blocking=True)
                        j = e + 1
                    else:
                        x[j * B:(j + 1) * B].copy_(xs[j], non_blocking=True)
                        j += 1
                if grp is not None:  # the group buffer may be refilled once its copies have completed
                    grp.copied.record(fs)
            else:
                x = xs[0]
            for xj in xs:  # read on this stream: keep the caller's buffers alive until then
                if not isinstance(xj, _HostBatch):
                    xj.record_stream(fs)
            _call(t, "sa1_fps", g, farthest_point_sample, x, self.M1, return_xyz=True, first_zero=self.fz[slot][:g],
                  slot=hs, out_idx=self.idx[slot][:g], out_xyz=self.cxyz[slot][:g], threads=self.fps_threads)
            lvl0 = self.bb.levels[0]
            for bi_, br in enumerate(lvl0["branches"]):
                tag = "sa1" + (f"_b{bi_}" if len(lvl0["branches"]) > 1 else "")
                if self.bq == "side":
                    _call(t, f"{tag}_ball_query", g, ball_query, br["r"], br["ns"], x, self.cxyz[slot][:g],
                          out=self.gidx[slot][bi_][:g], slot=hs)
                elif self.bq == "bin":  # depends only on the points: the queries run on the main stream
                    _call(t, f"{tag}_bq_bin", g, ball_query_bin, br["r"], br["ns"], x, self.grid[slot][bi_], slot=hs)
            if self.l2:
                c1 = self.cxyz[slot][:g]
                _call(t, "sa2_fps", g, farthest_point_sample, c1, self.M2, return_xyz=True,
                      first_zero=self.fz2[slot][:g], prefix_ok=self.fz[slot][:g], slot=hs,
                      out_idx=self.idx2[slot][:g], out_xyz=self.cxyz2[slot][:g])
                lvl1 = self.bb.levels[1]
                for bi_, br in enumerate(lvl1["branches"]):
                    tag = "sa2" + (f"_b{bi_}" if len(lvl1["branches"]) > 1 else "")
                    _call(t, f"{tag}_ball_query", g, ball_query, br["r"], br["ns"], c1, self.cxyz2[slot][:g],
                          out=self.gidx2[slot][bi_][:g], slot=hs)

            self.fps_done[slot].record(fs)
        return slot

    def _rest(self, slot, xs, main):
        """The MFMA levels of a group: one pass over its staged frames (every operator is per
        frame, so the per-batch outputs are views of the group's), split back per batch."""
        main.wait_event(self.fps_done[slot])
        B, g = self.B, len(xs) * self.B
        x = self.stage[slot][:g] if self.staged[slot] else xs[0]
        lvl0 = [self.idx[slot][:g], self.cxyz[slot][:g], self.fz[slot][:g],
                [gi[:g] if gi is not None else None for gi in self.gidx[slot]] if self.gidx is not None else None]
        pre2 = None
        if self.l2:
            pre2 = {"fps": (self.idx2[slot][:g], self.cxyz2[slot][:g], self.fz2[slot][:g]),
                    "bq": [gi[:g] for gi in self.gidx2[slot]]}

        if self.keep:  # the slot's buffers are reused by a later group
            lvl0 = [a.clone() for a in lvl0[:3]] + [[gi.clone() if gi is not None else None for gi in lvl0[3]]
                                                    if lvl0[3] is not None else None]
            if pre2 is not None:
                pre2 = {"fps": tuple(a.clone() for a in pre2["fps"]), "bq": [gi.clone() for gi in pre2["bq"]]}
        out, levels = self.bb.forward_from_sa1_fps(x, *lvl0, keep_levels=self.keep,
                                                   grids1=self.grid[slot] if self.grid is not None else None,
                                                   pre2=pre2)
        self.slot_free[slot].record(main)
        outs = list(out.split(B))
        if not self.keep:
            return outs
        per = []
        for j in range(len(xs)):
            sl = slice(j * B, (j + 1) * B)
            per.append((outs[j], [(nx[sl], nf[sl], ni[sl], [gi[sl] for gi in ng]) for nx, nf, ni, ng in levels]))
        return per

    def feed(self):
        return _Feed(self)

    def run(self, inputs):
        """inputs: list of (B, N, 3) CUDA tensors -> list of global features (B, C), in order."""
        f = _Feed(self)
        outs, i, k = [], 0, 0
        while i < len(inputs):
            # ramp: groups of 1, 2, ... G batches — the first group's FPS (the pipeline fill,
            # during which the main stream waits) is a third as long as a full group's
            sz = min(self.G, k + 1) if self.ramp else self.G
            outs += f._issue(list(inputs[i:i + sz]))
            i, k = i + sz, k + 1
        return outs + f.flush()


_HOST_READY = object()  # push_host's "ready" marker: the batch sits in pinned host memory already


class _HostGroup:
    """A group's pinned host buffer (G batches of rows); `copied` is recorded on the side stream after its
    host-to-device copy (the buffer may be refilled once it has completed)."""

    def __init__(self, pinned):
        self.pinned = pinned
        self.copied = torch.cuda.Event()
        self.copied.record()  # (a fresh buffer is free)


class _HostBatch:
    """One batch of host frames: rows j*B .. (j+1)*B of a pinned group buffer."""

    def __init__(self, grp, j):
        self.grp, self.j = grp, j


class _Feed:
    """StreamingSSG's persistent feed: push(batch) stages batches; every full group of G issues
    its SA1 FPS on a side stream and, once `depth` groups are in flight, the oldest group's
    remaining levels on the main stream (the caller's current stream).  push returns the
    outputs of the batches that call completed (in input order); flush() issues a partial last
    group and drains the pipeline.  push_host(frames) is push() for host NumPy frames."""

    def __init__(self, pipe):
        self.p = pipe
        self.main = torch.cuda.current_stream(pipe.bb.device)
        self.buf, self.pending, self.k = [], [], 0
        self.readies = []  # push()'s ready event per buffered batch
        # push_host's ring of pinned group buffers, the current group's, and the fill threads
        self._ring, self._ri, self._grp, self._pool = [], 0, None, None

    def push_host(self, frames, threads=4):
        """frames: one batch of host frames, a (B, N, 3) array or B arrays of shape (N, 3), of any real
        dtype (converted to float32 as numpy's astype does).  They are copied into the group's pinned
        buffer (G batches of rows) by `threads` host threads (frames split between them; numpy releases
        the GIL in the copy), and the group's side stream copies the buffer to the device ahead of its FPS
        in one DMA copy (a copy per batch, queued behind the side stream's kernels, held the calling
        thread for milliseconds now and then).  The pinned ring holds depth + 2 groups; a buffer is
        refilled only after its device copy has completed (a host wait on that event, the feed's
        back-pressure).  The batch that opens a group issues the oldest
        in-flight group's main-stream pass (push() issues it when the new group completes), so the main
        stream works while the host fills.  Returns the outputs of the batches that call completed, in
        input order; every output equals forward() of the same frames on the device."""
        import numpy as _np
        p = self.p
        B, N = p.B, p.N
        if isinstance(frames, _np.ndarray):
            if frames.shape != (B, N, 3):
                raise ValueError(f"push_host: frames must be ({B}, {N}, 3), got {frames.shape}")
            parts = list(frames)
        else:
            parts = [_np.asarray(f) for f in frames]
            if len(parts) != B or any(f.shape != (N, 3) for f in parts):
                raise ValueError(f"push_host: {B} frames of shape ({N}, 3) expected")
        out = []
        if not self.buf and len(self.pending) >= p.depth:
            # the batch opens a group whose completion would issue the oldest group's main-stream pass:
            # issue it now, so the main stream runs it while the host fills this group's batches
            slot, pxs = self.pending.pop(0)
            out = p._rest(slot, pxs, self.main)
        if not self._ring:
            import concurrent.futures
            self._ring = [_HostGroup(torch.empty((p.G * B, N, 3), dtype=torch.float32, pin_memory=True))
                          for _ in range(p.depth + 2)]
            self._nthreads = max(1, int(threads))
            self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=self._nthreads)
        if self._grp is None:  # the group's first host batch takes the next pinned group buffer
            self._grp = self._ring[self._ri]
            self._ri = (self._ri + 1) % len(self._ring)
            self._grp.copied.synchronize()  # its previous group has reached the device
        hb = _HostBatch(self._grp, len(self.buf))
        dst = self._grp.pinned[hb.j * B:(hb.j + 1) * B].numpy()
        step = -(-B // self._nthreads)

        def fill(lo):
            for j in range(lo, min(B, lo + step)):
                _np.copyto(dst[j], parts[j], casting="unsafe")

        for f in [self._pool.submit(fill, lo) for lo in range(0, B, step)]:
            f.result()
        self.buf.append(hb)
        self.readies.append(_HOST_READY)  # filled by the host: no device event to wait for
        if len(self.buf) < p.G:
            return out
        xs, evs = self.buf, self.readies
        self.buf, self.readies = [], []
        return out + self._issue(xs, evs)

    def _issue(self, xs, readies=None):
        self._grp = None  # the next group's host batches take a fresh pinned group buffer
        evs = [e for e in (readies or [None]) if e is not None and e is not _HOST_READY]
        if readies is None or any(e is None for e in readies):
            ev = torch.cuda.Event()
            ev.record(self.main)  # the inputs exist on the caller's stream
            evs.append(ev)
        self.pending.append((self.p._fps(self.k, xs, evs, self.main), xs))
        self.k += 1
        if len(self.pending) > self.p.depth:
            slot, pxs = self.pending.pop(0)
            return self.p._rest(slot, pxs, self.main)
        return []

    def push(self, x, ready=None):
        """ready: a CUDA event after which x is readable; None records one on the caller's stream
        when the group issues — which also orders the group's FPS after every main-stream pass
        issued so far, so a feed whose inputs were produced earlier passes the producer's event."""
        self.buf.append(x)
        self.readies.append(ready)
        if len(self.buf) < self.p.G:
            return []
        xs, evs = self.buf, self.readies
        self.buf, self.readies = [], []
        return self._issue(xs, evs)

    def close(self):
        """Stop push_host's copy threads and free the pinned ring (once its copies have completed)."""
        if self._pool is not None:
            self._pool.shutdown(wait=False)
            self._pool = None
            for grp in self._ring:
                grp.copied.synchronize()
            self._ring, self._grp = [], None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def flush(self, trim=True):
        """Issue a partial last group and drain the pipeline.  trim: then wait for the side streams
        and free the workspaces the library's handles retired while growing (lidar_trim)."""
        out = []
        if self.buf:
            xs, evs = self.buf, self.readies
            self.buf, self.readies = [], []
            out += self._issue(xs, evs)
        while self.pending:
            slot, pxs = self.pending.pop(0)
            out += self.p._rest(slot, pxs, self.main)
        if trim:
            for fs in self.p.fps_streams:
                fs.synchronize()
            self.main.synchronize()
            nat.trim(self.p.bb.device.index)
        return out
