"""Tier R parity on the GPU: the drop-in operators vs what the REFERENCE returned.

Every case of ``tests/golden/tier_r.json`` (captured by running the reference's
``preprocess_lidar_data`` -> ``extract_people_positions`` -> ``CrowdDensityModel.analyze``)
is rebuilt from its seed and run through the HIP path; arrays must be byte-identical
(ground plane: golden_cases.check_plane, gelsd's rank rule and eps*kappa), scalars
identical in value and type, hotspots identical in order.  Plus the reference's
error behaviour, the standalone DBSCAN kernel against the oracle on adversarial
frames, and voxel downsampling against the oracle and (its x / y binning) the reference's own
calculate_grid_density outputs (tests/golden/voxel.npz).
"""
import os

import numpy as np
import pytest

from golden.voxel_cases import VOXEL_CASES
from golden_cases import ARRAYS, ERROR_FRAMES, FRAMES, META, check_plane, check_tier_r
from lidar_ai_recommendation_software_amd import data_processing as dp
from lidar_ai_recommendation_software_amd.crowd_density_model import CrowdDensityModel
from lidar_ai_recommendation_software_amd.synthetic import STRESS_KINDS, lattice_frame, stress_frame, uniform_frame
from oracle import tier_n, tier_r

HERE = os.path.dirname(os.path.abspath(__file__))


pytestmark = pytest.mark.gpu


def unit_frames_np(b, n, seed):
    from lidar_ai_recommendation_software_amd.synthetic import unit_frames
    return unit_frames(b, n, seed)


@pytest.mark.parametrize("name", sorted(META["cases"]))
def test_reference_golden(cuda, name):
    pts = FRAMES[name]()
    pd = dp.preprocess_lidar_data(pts)
    people = dp.extract_people_positions(pd)
    check_tier_r(name, pd, people, lambda: CrowdDensityModel().analyze(pd))


@pytest.mark.parametrize("name", sorted(ERROR_FRAMES))
def test_reference_errors(cuda, name):
    want = META["errors"][name]
    with pytest.raises(Exception) as ei:
        dp.preprocess_lidar_data(ERROR_FRAMES[name]())
    assert type(ei.value).__name__ == want


@pytest.mark.parametrize("seed,eps", [(0, 0.5), (1, 0.3), (2, 0.8), (3, 0.05)])
def test_dbscan_kernel_vs_oracle(cuda, seed, eps):
    import torch
    from lidar_ai_recommendation_software_amd import _native as nat
    x = lattice_frame(4, 200, 300, seed, 3.0, 0.3)
    x[: len(x) // 10] = x[len(x) // 10: 2 * (len(x) // 10)]  # duplicates: zero distances
    want, wcnt = tier_r.dbscan_labels(x, eps, 5, return_counts=True)
    xt = torch.from_numpy(x).cuda()
    lab = torch.empty(len(x), dtype=torch.int64, device="cuda")
    cnt = torch.empty(len(x), dtype=torch.int32, device="cuda")
    nat.call("lidar_dbscan_f64", nat.handle(0), nat.ptr(xt), len(x), float(eps), 5, nat.ptr(lab),
             nat.ptr(cnt), nat.stream_ptr())
    assert np.array_equal(cnt.cpu().numpy(), wcnt)
    assert np.array_equal(lab.cpu().numpy(), want)


def test_people_and_density_on_foreign_input(cuda):
    # processed_data not produced by our preprocess (no device cache): upload path
    pd = tier_r.preprocess_lidar_data(lattice_frame(4, 60, 150, 0))
    pd = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in pd.items()}
    want_p = tier_r.extract_people_positions(pd)
    got_p = dp.extract_people_positions(pd)
    assert np.array_equal(got_p, want_p)
    for g in (1.0, 0.5, 2, 3.7):
        a = dp.calculate_grid_density(got_p, pd["dimensions"]["x_range"], pd["dimensions"]["y_range"], g)
        b = tier_r.calculate_grid_density(want_p, pd["dimensions"]["x_range"], pd["dimensions"]["y_range"], g)
        for u, v in zip(a, b):
            assert np.array_equal(u, v)
        ra = CrowdDensityModel(g).analyze(pd)
        rb = tier_r.analyze(pd, g)
        assert ra["hotspots"] == rb["hotspots"] and ra["avg_density"] == rb["avg_density"]


def test_downsample_point_cloud_matches_reference(cuda):
    base = np.arange(3000, dtype=np.float64).reshape(1000, 3)
    for key in META["downsample"]:
        seed, factor = key.split("_")
        np.random.seed(int(seed[1:]))
        out = dp.downsample_point_cloud(base, float(factor[1:]))
        assert np.array_equal((out[:, 0] // 3).astype(np.int64), ARRAYS[f"downsample/{key}"])


@pytest.mark.parametrize("n,v", [(4096, 0.1), (65536, 0.05), (20000, 0.5), (3000, 10.0), (1, 0.1)])
def test_voxel_downsample_vs_oracle(cuda, n, v):
    x = uniform_frame(n, 3, -1, 1).astype(np.float32)
    if n > 10:
        x[n // 2:] = x[: n - n // 2]  # duplicated points share voxels
    c, vid, cnt = dp.voxel_downsample(x, v)
    wc, wvid, wcnt = tier_n.voxel_downsample(x, v)
    assert np.array_equal(vid, wvid)
    assert np.array_equal(cnt, wcnt)
    assert np.array_equal(c, wc)


def _edge_frame(n, v, seed):
    """A [-1, 1] frame plus points on (and one float either side of) every grid edge inside the extent,
    on every axis: the keys launch's float threshold tables must bin them as the float64 edges do."""
    x = uniform_frame(n, seed, -1, 1).astype(np.float32)
    lo, hi = x.min(axis=0).astype(np.float64), x.max(axis=0).astype(np.float64)
    extra = []
    for a in range(3):
        e = np.arange(lo[a] - 2 * v, (hi[a] + 2 * v) + v, v)
        e = e[(e >= lo[a]) & (e <= hi[a])]
        for c in (np.float32(e), np.nextafter(np.float32(e), np.float32(np.inf)),
                  np.nextafter(np.float32(e), np.float32(-np.inf))):
            c = c[(c >= lo[a]) & (c <= hi[a])]
            pts = x[: len(c)].copy()
            pts[:, a] = c
            extra.append(pts)
    return np.concatenate([x] + extra).astype(np.float32)


@pytest.mark.parametrize("case", ["edges", "edges_coarse", "long_axis", "near_table_limit", "far_offset", "lidar_400m"])
def test_voxel_keys_table_and_float64_paths(cuda, case):
    """The keys launch bins in float against per-axis tables of the float64 edges' float thresholds
    (<= 8 192 edges per axis) and in float64 otherwise: both bit-exact against the oracle, points on
    the edges included, guesses off by more than a bin (large offsets) included."""
    rng = np.random.default_rng(11)
    if case == "edges":
        x, v = _edge_frame(20000, 0.05, 5), 0.05
    elif case == "edges_coarse":
        x, v = _edge_frame(5000, 0.3, 6), 0.3
    else:
        n = 50000
        x = rng.random((n, 3)).astype(np.float32)
        x[:, 1:] *= np.float32(0.002)
        if case == "long_axis":  # x: ~10 000 edges, past the table
            v = 1e-4
        elif case == "near_table_limit":  # x: ~8 005 edges, in the table
            x[:, 0] *= np.float32(0.8)
            v = 1e-4
        elif case == "lidar_400m":  # ±200 m (±1 m in z) at 5 cm: ~8 000 edges on x and y, in the tables
            x = (rng.uniform(-1, 1, (n, 3)) * [200, 200, 1]).astype(np.float32)
            v = 0.05
        else:  # coordinates near 1 000: float spacing 6e-5 against a 1e-3 voxel
            x[:, 0] = x[:, 0] + np.float32(1000.0)
            v = 1e-3
    c, vid, cnt = dp.voxel_downsample(x, v)
    wc, wvid, wcnt = tier_n.voxel_downsample(x, v)
    assert np.array_equal(vid, wvid), case
    assert np.array_equal(cnt, wcnt), case
    assert np.array_equal(c, wc), case


class DiagVoxel:
    """The diagnostic build (liblidar_amd_diag.so, `make diag`): the product library plus its testing aids
    (lidar_debug_fill_workspace / _set_epoch / _voxel_inject), which the product ABI does not export.  It is
    loaded beside the product library and keeps handles of its own, so the voxel calls below run the diag
    build's copy of csrc/voxel_batch.hip (the same source)."""

    _lib = None

    def __init__(self, device=0):
        import ctypes
        from lidar_ai_recommendation_software_amd import _native as nat
        if DiagVoxel._lib is None:
            path = os.path.join(os.path.dirname(nat.__file__), "liblidar_amd_diag.so")
            assert os.path.exists(path), "liblidar_amd_diag.so not built (__graft_entry__.build(): make diag)"
            lib = ctypes.CDLL(path)
            for name, at in nat.SIGNATURES.items():
                fn = getattr(lib, name)
                fn.argtypes = at
                fn.restype = nat._RESTYPES.get(name, ctypes.c_int)
            lib.lidar_debug_fill_workspace.argtypes = [nat.P, ctypes.c_uint64, ctypes.c_uint64, nat.P]
            lib.lidar_debug_set_epoch.argtypes = [nat.P, ctypes.c_uint32]
            lib.lidar_debug_voxel_inject.argtypes = [ctypes.c_int64]
            lib.lidar_last_error.restype = ctypes.c_char_p
            DiagVoxel._lib = lib
        self.lib, self.nat = DiagVoxel._lib, nat
        hp = nat.P()
        self.call("lidar_create", int(device), ctypes.byref(hp))
        self.h = hp

    def call(self, name, *args):
        rc = getattr(self.lib, name)(*args)
        assert rc == 0, (name, rc, self.lib.lidar_last_error())

    def voxel(self, xt, voxel):
        import torch
        B, N, _ = xt.shape
        cent = torch.empty((B, N, 3), dtype=torch.float32, device=xt.device)
        vid = torch.empty((B, N), dtype=torch.int32, device=xt.device)
        cnt = torch.empty((B, N), dtype=torch.int32, device=xt.device)
        nvox = torch.empty(B, dtype=torch.int32, device=xt.device)
        p = self.nat.ptr
        self.call("lidar_voxel_downsample_batch_f32", self.h, p(xt), B, N, float(voxel), p(vid), p(cent), p(cnt),
                  p(nvox), self.nat.stream_ptr())
        return cent, vid, cnt, nvox


def test_product_abi_has_no_testing_aids(cuda):
    from lidar_ai_recommendation_software_amd import _native as nat
    lib = nat.load_library()
    for name in ("lidar_debug_fill_workspace", "lidar_debug_set_epoch", "lidar_debug_voxel_inject"):
        assert getattr(DiagVoxel().lib, name, None) is not None
        assert not hasattr(lib, name), name


@pytest.mark.parametrize("B,n", [(32, 65536), (3, 20000), (1, 150001)])
def test_voxel_ignores_workspace_leftovers(cuda, B, n):
    """The batched voxel path's in-launch hand-offs read only granules of the handle's tag block, which
    holds earlier calls' tags at other layouts: a workspace full of tag-like garbage (high halves 1..64,
    the next calls' tags) and the other layout's leftovers change nothing (the diagnostic build)."""
    import torch
    from lidar_ai_recommendation_software_amd.synthetic import unit_frames
    dv = DiagVoxel()
    x = unit_frames(B, n, 8)
    xt = torch.from_numpy(x).to(cuda)
    need = dv.lib.lidar_voxel_batch_workspace_bytes(B, n) + (1 << 20)
    other = torch.from_numpy(unit_frames(5, 7001, 9)).to(cuda)
    for seed in (1, 2, 3):
        # the tag block: tags of earlier calls at another layout (never this call's epoch)
        dv.voxel(other, 0.02 * seed)
        dv.call("lidar_debug_fill_workspace", dv.h, need, seed, dv.nat.stream_ptr())
        c, vid, cnt, nv = dv.voxel(xt, 0.05)
        torch.cuda.synchronize()
        nv = nv.cpu().numpy()
        for f in (0, B - 1):
            wc, wvid, wcnt = tier_n.voxel_downsample(x[f], 0.05)
            assert nv[f] == len(wc), (seed, f)
            assert np.array_equal(vid[f].cpu().numpy(), wvid)
            assert np.array_equal(cnt[f, :nv[f]].cpu().numpy(), wcnt)
            assert np.array_equal(c[f, :nv[f]].cpu().numpy(), wc)


@pytest.mark.parametrize("B,n,bucket", [(32, 65536, 3), (2, 65536, 31), (3, 300000, 0), (4, 20000, 9)])
def test_voxel_failure_is_sticky(cuda, B, n, bucket):
    """A bucket that fails (here: the diagnostic build's injected inconsistent bucket table at `bucket` of
    every frame, nvox -3) wins over the voxel count the frame's last bucket writes — in the middle, at the
    last bucket, at the first one (the look-back's start), on a frame of the three-launch keys path; the
    Python layer raises LidarError on it, and the next call is clean again."""
    import torch
    from lidar_ai_recommendation_software_amd import _native as nat
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    from lidar_ai_recommendation_software_amd.synthetic import unit_frames
    dv = DiagVoxel()
    x = torch.from_numpy(unit_frames(B, n, 31)).to(cuda)
    nb = (n + 2047) // 2048
    assert bucket < nb
    dv.call("lidar_debug_voxel_inject", bucket)
    try:
        _, _, _, nv = dv.voxel(x, 0.05)
        torch.cuda.synchronize()
    finally:
        dv.call("lidar_debug_voxel_inject", -1)
    assert (nv.cpu().numpy() == -3).all(), nv
    with pytest.raises(nat.LidarError, match="bucket table"):
        pn.check_voxel_counts(nv)
    c, vid, cnt, nv = dv.voxel(x, 0.05)
    torch.cuda.synchronize()
    wc, wvid, wcnt = tier_n.voxel_downsample(x[B - 1].cpu().numpy(), 0.05)
    assert nv[B - 1].item() == len(wc) and np.array_equal(vid[B - 1].cpu().numpy(), wvid)


def test_voxel_beside_ssg_feed(cuda):
    """The fused keys launch's in-launch hand-offs assume a frame's <= 16 tiles become co-resident (one
    XCD, dispatched together).  Here 32 x 65 536-point batched voxel calls run on their own stream and
    handle slot while the SSG feed (512-thread SA1 FPS on three side streams, the MFMA levels on the main
    stream) occupies the chip: every call bit-exact against the oracle (frames 0 and 31), no nvox < 0."""
    import torch
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    from lidar_ai_recommendation_software_amd.synthetic import unit_frames
    from lidar_ai_recommendation_software_amd.streams import side_streams
    B, N = 32, 65536
    xv = torch.from_numpy(unit_frames(B, N, 41)).to(cuda)
    want = {f: tier_n.voxel_downsample(xv[f].cpu().numpy(), 0.05) for f in (0, B - 1)}
    bb = pn.PointNet2Backbone(pn.SSG, device=cuda, seed=0)
    xs = [torch.from_numpy(unit_frames(B, N, 60 + i)).to(cuda) for i in range(2)]
    feed = pn.StreamingSSG(bb, B, N, depth=3, fps_group=2, fps_threads=512, ramp=False, bq="bin",
                           l2_side=True).feed()
    vs = side_streams(cuda, 1, start=3)[0]  # beyond the feed's three side streams
    outs = []
    for i in range(16):
        outs += feed.push(xs[i % 2])
        if i >= 6:  # the pipeline is full: FPS workgroups resident, MFMA levels queued
            with torch.cuda.stream(vs):
                c, vid, cnt, nv = pn.voxel_downsample_batch(xv, 0.05, slot=12, check=False)
                outs_v = (c, vid, cnt, nv)
            vs.synchronize()
            nvh = nv.cpu().numpy()
            assert (nvh >= 0).all(), (i, nvh)
            for f, (wc, wvid, wcnt) in want.items():
                assert nvh[f] == len(wc), (i, f)
                assert np.array_equal(vid[f].cpu().numpy(), wvid), (i, f)
                assert np.array_equal(c[f, :nvh[f]].cpu().numpy(), wc), (i, f)
    outs += feed.flush()
    torch.cuda.synchronize()
    assert len(outs) == 16
    del outs_v


def test_voxel_batch_output_reuse(cuda):
    """out=: a stream of batches writes the same four output tensors call after call (check=False leaves
    nvox on the device); every call equals a fresh call, and a mismatched out is refused."""
    import torch
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    from lidar_ai_recommendation_software_amd.synthetic import unit_frames
    xs = [torch.from_numpy(unit_frames(4, 30000, 50 + i)).to(cuda) for i in range(3)]
    res = pn.voxel_downsample_batch(xs[0], 0.05)
    for x in xs[1:] + xs[:1]:
        pn.voxel_downsample_batch(x, 0.05, check=False, out=res)
        want = pn.voxel_downsample_batch(x, 0.05)
        pn.check_voxel_counts(res[3])
        assert torch.equal(res[3], want[3]) and torch.equal(res[1], want[1])
        for f in range(4):
            v = int(want[3][f])
            assert torch.equal(res[0][f, :v], want[0][f, :v]) and torch.equal(res[2][f, :v], want[2][f, :v])
    with pytest.raises(ValueError, match="out must be"):
        pn.voxel_downsample_batch(xs[0][:2].contiguous(), 0.05, out=res)


@pytest.mark.parametrize("case", ["wide_keys", "lidar_sparse", "runs_128", "runs_129", "runs_600"])
def test_voxel_bucket_sort_paths(cuda, case):
    """The bucket launch's sorts: the LDS counting sort (runs of up to SEGMAX = 128 equal keys ordered by
    index in place), its shifted form for sparse grids (a key range past 4 096: counters over the keys'
    high bits, each run ordered by (key, index) words), the LDS bitonic sort (a longer run, in buckets of
    up to 2 048 pairs) and the global radix sort (the same in larger buckets) — each bit-exact against the oracle,
    through the batched path (two frames) and the drop-in."""
    import torch
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    rng = np.random.default_rng(21)
    if case == "wide_keys":  # ~100^3 keys over 65 536 points: every bucket past the counting range
        x, v = rng.random((65536, 3)).astype(np.float32), 0.01
    elif case == "lidar_sparse":  # 200 x 200 x 10 m at 5 cm: ~3.3e9 keys, a bucket's keys far apart
        x, v = (rng.uniform(-1, 1, (65536, 3)) * [100, 100, 5]).astype(np.float32), 0.05
    else:  # clusters of exactly r points inside one voxel each, plus uniform points
        r = int(case.split("_")[1])
        k = 40000 // r
        c = (rng.integers(0, 20, (k, 3)) * 0.05 + 0.025).astype(np.float32)
        pts = np.repeat(c, r, axis=0) + rng.uniform(-0.01, 0.01, (k * r, 3)).astype(np.float32)
        x = np.concatenate([pts, rng.random((8000, 3)).astype(np.float32)])[rng.permutation(k * r + 8000)]
        v = 0.05
    xb = np.stack([x, x[::-1].copy()])
    c, vid, cnt, nv = (t.cpu().numpy() for t in pn.voxel_downsample_batch(torch.from_numpy(xb).to(cuda), v))
    for f in range(2):
        wc, wvid, wcnt = tier_n.voxel_downsample(xb[f], v)
        assert nv[f] == len(wcnt), (case, f)
        assert np.array_equal(vid[f], wvid) and np.array_equal(cnt[f, :nv[f]], wcnt), (case, f)
        assert np.array_equal(c[f, :nv[f]].view(np.uint32), wc.view(np.uint32)), (case, f)
    c1, vid1, cnt1 = dp.voxel_downsample(x, v)
    assert np.array_equal(vid1, vid[0]) and np.array_equal(c1.view(np.uint32), c[0, :nv[0]].view(np.uint32))


@pytest.mark.parametrize("seed", range(12))
def test_voxel_random_frames_vs_oracle(cuda, seed):
    """Randomised frames through the batched path (three frames per call): sizes from 1 to 40 000 points,
    extents from centimetres to hundreds of metres, voxel sizes over four decades, duplicated points and
    tight clusters — every sort path (dense / shifted counting, bitonic, radix) in some bucket; ids, counts
    and centroids bit-exact against the oracle, nvox -1 exactly where the oracle refuses the grid."""
    import torch
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.choice([1, 7, 300, 5000, 20000, 40000]))
    frames = []
    for _ in range(3):
        ext = 10.0 ** rng.uniform(-2, 2.5, 3)
        x = (rng.uniform(-1, 1, (n, 3)) * ext + rng.uniform(-50, 50, 3)).astype(np.float32)
        if n > 10 and rng.random() < 0.5:  # duplicates
            k = int(n * rng.uniform(0.1, 0.5))
            x[rng.integers(0, n, k)] = x[rng.integers(0, n, k)]
        if n > 100 and rng.random() < 0.5:  # a tight cluster
            k = int(n * rng.uniform(0.05, 0.3))
            x[:k] = x[0] + rng.normal(0, 1e-3, (k, 3)).astype(np.float32)
        frames.append(x)
    xb = np.stack(frames)
    span = float(np.median((xb.max(axis=1) - xb.min(axis=1)).max(axis=1)))
    v = float(span / 10.0 ** rng.uniform(0.5, 3.3)) or 1.0
    c, vid, cnt, nv = (t.cpu().numpy() for t in pn.voxel_downsample_batch(torch.from_numpy(xb).to(cuda), v))
    for f in range(3):
        try:
            wc, wvid, wcnt = tier_n.voxel_downsample(xb[f], v)
        except ValueError:
            assert nv[f] == -1, (seed, f)
            continue
        assert nv[f] == len(wcnt), (seed, f, n, v)
        assert np.array_equal(vid[f], wvid) and np.array_equal(cnt[f, :nv[f]], wcnt), (seed, f, n, v)
        assert np.array_equal(c[f, :nv[f]].view(np.uint32), wc.view(np.uint32)), (seed, f, n, v)


@pytest.mark.parametrize("seed", range(3))
def test_voxel_random_large_sparse_frames_vs_oracle(cuda, seed):
    """Real LiDAR sizes (150 000 - 300 000 points: the extent / keys / scatter launches) over sparse grids
    (tens to hundreds of metres at 2-20 cm: the shifted counting sort, and its bitonic / radix fallbacks
    where (key bits + index bits) pass 32), two frames per call, bit-exact against the oracle."""
    import torch
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    rng = np.random.default_rng(2000 + seed)
    n = int(rng.choice([150001, 220000, 300000]))
    ext = np.array([rng.uniform(20, 150), rng.uniform(20, 150), rng.uniform(0.5, 4)])
    xb = (rng.uniform(-1, 1, (2, n, 3)) * ext).astype(np.float32)
    xb[1, : n // 4] = xb[1, 0] + rng.normal(0, 0.05, (n // 4, 3)).astype(np.float32)  # a dense clump
    v = float(rng.choice([0.02, 0.05, 0.2]))
    c, vid, cnt, nv = (t.cpu().numpy() for t in pn.voxel_downsample_batch(torch.from_numpy(xb).to(cuda), v))
    for f in range(2):
        try:
            wc, wvid, wcnt = tier_n.voxel_downsample(xb[f], v)
        except ValueError:
            assert nv[f] == -1, (seed, f)
            continue
        assert nv[f] == len(wcnt), (seed, f, n, v)
        assert np.array_equal(vid[f], wvid) and np.array_equal(cnt[f, :nv[f]], wcnt), (seed, f, n, v)
        assert np.array_equal(c[f, :nv[f]].view(np.uint32), wc.view(np.uint32)), (seed, f, n, v)


def test_voxel_epoch_wrap(cuda):
    """The voxel calls' tags across the 32-bit epoch wrap (the tag block zeroed again there): the calls
    before, at and after the wrap all equal the oracle (the diagnostic build's epoch setter)."""
    import torch
    from lidar_ai_recommendation_software_amd.synthetic import unit_frames
    x = unit_frames(3, 20000, 12)
    xt = torch.from_numpy(x).to(cuda)
    want = [tier_n.voxel_downsample(x[f], 0.05) for f in range(3)]
    dv = DiagVoxel()
    dv.call("lidar_debug_set_epoch", dv.h, 0xfffffffd)
    for _ in range(4):  # epochs 0xfffffffe, 0xffffffff, then 1 (wrapped), 2
        c, vid, cnt, nv = dv.voxel(xt, 0.05)
        torch.cuda.synchronize()
        nv = nv.cpu().numpy()
        for f in range(3):
            wc, wvid, wcnt = want[f]
            assert nv[f] == len(wc)
            assert np.array_equal(vid[f].cpu().numpy(), wvid)
            assert np.array_equal(cnt[f, :nv[f]].cpu().numpy(), wcnt)
            assert np.array_equal(c[f, :nv[f]].cpu().numpy(), wc)


def test_fps_extension(cuda):
    x = uniform_frame(5000, 1, -1, 1).astype(np.float32)
    assert np.array_equal(dp.farthest_point_sample(x, 256), tier_n.fps(x, 256))


@pytest.mark.parametrize("name", ["lattice_62978_s2", "crowd_65536_s3", "lattice_8163_s4"])
def test_dbscan_labels_deterministic(cuda, name):
    """Union-find runs with racing atomics across workgroups (and XCDs); the labels must
    not depend on the schedule.  A path-halving store racing the roots pass once left a
    non-root in parent[] in ~1 run of 3 — repeated runs pin that down."""
    from golden_cases import FRAMES, META, digest
    if name not in FRAMES:
        pytest.skip(f"{name} not in the golden set")
    pts = FRAMES[name]()
    want = META["cases"][name]["clusters"]["sha256"]
    for r in range(8):
        got = digest(dp.preprocess_lidar_data(pts)["clusters"])["sha256"]
        assert got == want, f"run {r}: labels differ from the reference"


def test_density_stream_matches_drop_in(cuda):
    """The device-resident multi-stream executor returns, frame for frame, what the
    drop-in preprocess_lidar_data + CrowdDensityModel.analyze return."""
    import torch
    from lidar_ai_recommendation_software_amd.density_stream import DensityStream
    names = ["uniform_16384_s0", "crowd_16384_s7", "lattice_8163_s4", "small_20", "small_12", "int_4096"]
    names = [k for k in names if k in FRAMES]
    frames = [FRAMES[k]() for k in names]
    ds = DensityStream(cuda, workers=3)
    got = ds.run([torch.from_numpy(np.ascontiguousarray(f, dtype=np.float64)).to(cuda) for f in frames])
    model = CrowdDensityModel(1.0)
    for name, f, g in zip(names, frames, got):
        want = model.analyze(dp.preprocess_lidar_data(np.asarray(f, dtype=np.float64)))
        assert g["total_people"] == want["total_people"], name
        assert float(g["avg_density"]).hex() == float(want["avg_density"]).hex(), name
        assert float(g["max_density"]).hex() == float(want["max_density"]).hex(), name
        assert np.array_equal(g["density_map"], want["density_map"]), name
        assert [(h["x"], h["y"], h["density"]) for h in g["hotspots"]] == \
               [(h["x"], h["y"], h["density"]) for h in want["hotspots"]], name


def _same_analyze(name, g, want):
    assert g["total_people"] == want["total_people"], name
    assert float(g["avg_density"]).hex() == float(want["avg_density"]).hex(), name
    assert float(g["max_density"]).hex() == float(want["max_density"]).hex(), name
    assert type(g["avg_density"]) is type(want["avg_density"]), name
    assert np.array_equal(g["density_map"], want["density_map"]), name
    assert np.array_equal(g["grid_coordinates"][0], want["grid_coordinates"][0]), name
    assert np.array_equal(g["density_values"], want["density_values"]), name
    assert [(h["x"], h["y"], h["density"]) for h in g["hotspots"]] == \
           [(h["x"], h["y"], h["density"]) for h in want["hotspots"]], name


def test_density_batch_matches_drop_in(cuda):
    """lidar_preprocess_batch_f64 / lidar_people_batch_f64 / lidar_density_batch_f64: one
    launch per phase over a CSR batch of frames of different sizes (incl. a 12-point frame,
    a frame with no cluster and int input) equals the per-frame drop-in, frame for frame."""
    import torch
    from lidar_ai_recommendation_software_amd.density_stream import DensityStream
    names = ["uniform_16384_s0", "small_12", "crowd_16384_s7", "lattice_8163_s4", "small_20", "int_4096",
             "uniform_65536_s0", "blobs_4293_s0", "dup_4096", "tight_2048"]
    names = [k for k in names if k in FRAMES]
    frames = [np.asarray(FRAMES[k](), dtype=np.float64) for k in names]
    ds = DensityStream(cuda, workers=1)
    got = ds.run_batch([torch.from_numpy(np.ascontiguousarray(f)).to(cuda) for f in frames])
    model = CrowdDensityModel(1.0)
    for name, f, g in zip(names, frames, got):
        _same_analyze(name, g, model.analyze(dp.preprocess_lidar_data(f)))
    # the same batch twice in a row (workspace reuse) gives the same
    again = ds.run_batch([torch.from_numpy(np.ascontiguousarray(f)).to(cuda) for f in frames])
    for name, a, b in zip(names, got, again):
        _same_analyze(name, a, b)


def test_density_run_batches_pipelined(cuda):
    """DensityStream.run_batches: batches in flight on two lanes (host thread + HIP stream +
    handle each) give run_batch's results batch by batch, in order; a failing batch raises the
    reference's exception."""
    import torch
    from lidar_ai_recommendation_software_amd.density_stream import DensityStream
    names = [k for k in ["uniform_16384_s0", "small_12", "crowd_16384_s7", "lattice_8163_s4", "small_20",
                         "int_4096", "blobs_4293_s0", "dup_4096", "tight_2048"] if k in FRAMES]
    T = lambda k: torch.from_numpy(np.ascontiguousarray(np.asarray(FRAMES[k](), dtype=np.float64))).to(cuda)
    batches = [[T(k) for k in names[i:i + 3]] for i in range(0, len(names), 3)] * 2
    ds = DensityStream(cuda, workers=1)
    want = [ds.run_batch(b) for b in batches]
    people_last = ds.people_of_last_batch().clone()
    got = ds.run_batches(batches, lanes=2)
    assert len(got) == len(want)
    for wb, gb in zip(want, got):
        for name, a, b in zip(names * 2, wb, gb):
            _same_analyze(name, a, b)
    # the people of the last batch in batch order, whichever lane finished last
    assert torch.equal(ds.people_of_last_batch(), people_last)
    # an empty last batch keeps them (as run_batch does)
    ds.run_batches(batches[:2] + [[]], lanes=2)
    assert torch.equal(ds.people_of_last_batch(), people_last)
    # the lanes are persistent threads: a second call reuses their handles
    lanes = list(ds._lanes)
    ds.run_batches(batches, lanes=2)
    assert ds._lanes == lanes
    bad = batches[:2] + [[T(names[0]), torch.zeros((0, 3), dtype=torch.float64, device=cuda)]]
    with pytest.raises(ValueError):
        ds.run_batches(bad, lanes=2)
    # the default (three lanes) and more lanes than hardware queues give the same results
    for ln in (None, 5):
        got = ds.run_batches(batches) if ln is None else ds.run_batches(batches, lanes=ln)
        for wb, gb in zip(want, got):
            for name, a, b in zip(names * 2, wb, gb):
                _same_analyze(name, a, b)
    ds.close()


def test_workspace_growth_retires_then_trims(cuda):
    """A handle's workspace grows while its earlier kernels are still queued: the old block is
    retired (no device-wide sync), the queued work still reads valid memory and its results are
    right, and lidar_trim frees the retired block once the stream has drained."""
    import ctypes
    import torch
    from lidar_ai_recommendation_software_amd import _native as nat
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    small = torch.from_numpy(unit_frames_np(2, 4096, 1)).to(cuda)
    big = torch.from_numpy(unit_frames_np(8, 65536, 2)).to(cuda)
    h = nat.handle(cuda.index, slot=5)
    nat.trim(cuda.index)
    a = pn.farthest_point_sample(small, 512, slot=5)         # sizes the workspace
    b = pn.farthest_point_sample(big, 2048, slot=5)          # grows it while `a` may be queued
    c = pn.farthest_point_sample(small, 512, slot=5)
    torch.cuda.synchronize()
    assert torch.equal(a, c)
    assert np.array_equal(b.cpu().numpy()[3], tier_n.fps(big[3].cpu().numpy(), 2048))
    freed = ctypes.c_uint64(0)
    nat.call("lidar_trim", h, ctypes.byref(freed))
    assert freed.value > 0, "the growth retired the first workspace"
    nat.call("lidar_trim", h, ctypes.byref(freed))
    assert freed.value == 0


@pytest.mark.parametrize("bad,exc", [("empty", ValueError), ("const_col", IndexError), ("nan", IndexError)])
def test_density_batch_errors(cuda, bad, exc):
    import torch
    from lidar_ai_recommendation_software_amd.density_stream import DensityStream
    frames = [FRAMES["uniform_4096_s0"](), ERROR_FRAMES[bad](), FRAMES["uniform_4096_s1"]()]
    with pytest.raises(exc):
        DensityStream(cuda).run_batch([torch.from_numpy(np.ascontiguousarray(f, dtype=np.float64)).to(cuda)
                                       for f in frames])


@pytest.mark.parametrize("kind,n,r,dim", [("uniform", 20000, 0.5, 3), ("crowd", 16384, 0.5, 3), ("uniform", 20000, 0.5, 2),
                                          ("dups", 4096, 0.5, 3), ("uniform", 3000, 2.0, 3), ("uniform", 1, 0.5, 3)])
def test_radius_count_matches_sklearn_kdtree(cuda, kind, n, r, dim):
    """The reference's density colouring: KDTree(points).query_radius(points, r, count_only=True)
    (sklearn is in this image; the call and its arguments are the reference's)."""
    from sklearn.neighbors import KDTree
    from lidar_ai_recommendation_software_amd.synthetic import crowd_frame
    if kind == "crowd":
        pts = crowd_frame(n, 3)
    elif kind == "dups":
        pts = np.repeat(uniform_frame(n // 4, 4), 4, axis=0)
    else:
        pts = uniform_frame(n, 6)
    pts = np.ascontiguousarray(pts[:, :dim], dtype=np.float64)
    want = KDTree(pts).query_radius(pts, r=r, count_only=True)
    got = dp.radius_count(pts, r)
    assert got.dtype == want.dtype and np.array_equal(got, want)


@pytest.mark.parametrize("n,bins,rng", [(20000, 50, [(-15, 15), (-15, 15)]), (5000, 17, [(-3.2, 11.7), (-15, 0)]),
                                        (1000, 50, None), (0, 5, [(0, 1), (0, 1)])])
def test_histogram2d_matches_numpy(cuda, n, bins, rng):
    """The reference's projection heatmap: np.histogram2d(d1, d2, bins=resolution, range=[...])."""
    pts = uniform_frame(max(n, 1), 8)[:n]
    pts[: n // 10, 0] = 11.7  # values on an edge
    want = np.histogram2d(pts[:, 0], pts[:, 1], bins=bins, range=rng)
    got = dp.histogram2d(pts[:, 0], pts[:, 1], bins=bins, range=rng)
    for g, w in zip(got, want):
        assert g.dtype == w.dtype and np.array_equal(g, w)


# ------------------------------------------------- variant pipeline
from golden_cases import VERROR_FRAMES, VFRAMES, VMETA, check_variant  # noqa: E402
from lidar_ai_recommendation_software_amd import variant_pipeline as vp  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import blob_frame, crowd_frame  # noqa: E402


@pytest.mark.parametrize("name", sorted(VFRAMES))
def test_variant_golden(cuda, name):
    """app_simplified.py's preprocess_point_cloud -> analyze_crowd_density on the GPU vs
    scikit-learn's DBSCAN / KDTree results (tests/golden/gen_variant.py), byte for byte."""
    pd = vp.preprocess_point_cloud(VFRAMES[name]())
    check_variant(name, pd, vp.analyze_crowd_density(pd))


@pytest.mark.parametrize("name", sorted(VERROR_FRAMES))
def test_variant_errors(cuda, name):
    with pytest.raises(Exception) as ei:
        vp.analyze_crowd_density(vp.preprocess_point_cloud(VERROR_FRAMES[name]()))
    assert type(ei.value).__name__ == VMETA["errors"][name]


@pytest.mark.parametrize("seed", range(6))
def test_variant_vs_oracle_random(cuda, seed):
    """more frames than the fixtures hold: crowd / blob frames of varied size vs the
    oracle's restatement (pinned to scikit-learn by tests/test_oracle.py)."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2000, 40000))
    pts = crowd_frame(n, 100 + seed) if seed % 2 else blob_frame(int(rng.integers(20, 200)), 50, 300, seed, 12, 0.35)
    got_pd = vp.preprocess_point_cloud(pts)
    want_pd = tier_r.variant_preprocess_point_cloud(pts)
    assert np.array_equal(got_pd["clusters"], want_pd["clusters"])
    assert np.array_equal(got_pd["points"], want_pd["points"])
    got, want = vp.analyze_crowd_density(got_pd), tier_r.variant_analyze_crowd_density(want_pd)
    assert got["total_people"] == want["total_people"]
    assert np.array_equal(got["density_grid"], want["density_grid"])
    assert float(got["avg_density"]).hex() == float(want["avg_density"]).hex()
    assert [(float(h["x"]).hex(), float(h["y"]).hex(), h["density"]) for h in got["hotspots"]] == \
        [(float(h["x"]).hex(), float(h["y"]).hex(), h["density"]) for h in want["hotspots"]]


def test_cell_radius_density_boundary(cuda):
    """people exactly at distance r (counted: <=) and just beyond; grid edges from np.arange."""
    import torch
    from lidar_ai_recommendation_software_amd import _native as nat
    people = np.array([[0.5, 0.5], [2.5, 0.5], [0.5, 2.5 + 1e-12], [-1.5, 0.5]], dtype=np.float64)
    xg, yg = np.arange(0.0, 4.0, 1.0), np.arange(0.0, 3.0, 1.0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    out = torch.empty((len(yg) - 1, len(xg) - 1), dtype=torch.float64, device="cuda")
    pd_, xd, yd = T(people), T(xg), T(yg)  # kept alive until the kernel has run
    nat.call("lidar_cell_radius_density_f64", nat.handle(0), nat.ptr(pd_), len(people), nat.ptr(xd),
             len(xg), nat.ptr(yd), len(yg), 2.0, 4.0, nat.ptr(out), nat.stream_ptr())
    cx, cy = (xg[:-1] + xg[1:]) / 2, (yg[:-1] + yg[1:]) / 2
    d = (cx[None, :, None] - people[None, None, :, 0]) ** 2 + (cy[:, None, None] - people[None, None, :, 1]) ** 2
    assert np.array_equal(out.cpu().numpy(), np.sum(d <= 4.0, axis=2) / 4.0)


def _outside_frame(n):
    """Points near 2^30 with a voxel of 3.3 float64 ulps there: numpy's arange spacing
    (e[1] - e[0]) rounds below the step, so the edges stop short of the extent and the top
    third of the points lies outside every bin (histogram2d drops them; voxel id -1)."""
    lo = np.float32(2.0 ** 30 + 1024)
    x = np.zeros((n, 3), np.float32)
    x[:, 0] = np.where(np.arange(n) % 3 == 1, lo + np.float32(128), lo)
    x[:, 1] = np.float32(0.5)
    x[:, 2] = np.float32(-0.25)
    return x, 3.3 * 2.0 ** -22


def test_voxel_downsample_batch_vs_oracle(cuda):
    """The chip-wide batched voxel path vs the oracle frame by frame: different extents and
    voxel sizes per key range (0 to 4 radix passes), duplicated points, a one-voxel frame, a flat
    frame, a frame with points outside every bin (32-bit keys), and grids of 2^32 keys or more or
    with a NaN extent (nvox -1)."""
    import torch
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    rng = np.random.default_rng(11)
    B, N = 6, 5001
    x = rng.uniform(-1, 1, (B, N, 3)).astype(np.float32)
    x[1] *= 7.5
    x[2, N // 2:] = x[2, : N - N // 2]  # duplicates share voxels
    x[3] = x[3, 0]  # one voxel (no radix pass)
    x[4, :, 2] = 0.25  # a flat frame
    for voxel in (0.5, 0.07, 0.013):
        c, vid, cnt, nv = pn.voxel_downsample_batch(torch.from_numpy(x).to(cuda), voxel)
        c, vid, cnt, nv = c.cpu().numpy(), vid.cpu().numpy(), cnt.cpu().numpy(), nv.cpu().numpy()
        for f in range(B):
            wc, wvid, wcnt = tier_n.voxel_downsample(x[f], voxel)
            assert nv[f] == len(wcnt), (voxel, f)
            assert np.array_equal(vid[f], wvid) and np.array_equal(cnt[f, :nv[f]], wcnt)
            assert np.array_equal(c[f, :nv[f]].view(np.uint32), wc.view(np.uint32)), (voxel, f)
    xo, vo = _outside_frame(N)
    xb = np.stack([xo, xo])
    xb[1, 7, 1] = np.nan  # NaN extent: np.arange cannot compute a length
    c, vid, cnt, nv = (t.cpu().numpy() for t in pn.voxel_downsample_batch(torch.from_numpy(xb).to(cuda), vo))
    wc, wvid, wcnt = tier_n.voxel_downsample(xo, vo)
    assert (wvid < 0).sum() == N // 3 + (N % 3 > 1) and nv.tolist() == [len(wcnt), -1]
    assert np.array_equal(vid[0], wvid) and np.array_equal(cnt[0, :nv[0]], wcnt)
    assert np.array_equal(c[0, :nv[0]].view(np.uint32), wc.view(np.uint32))
    _, _, _, nv = pn.voxel_downsample_batch(torch.from_numpy(x[:2]).to(cuda), 1e-6)
    assert nv.cpu().numpy().tolist() == [-1, -1]


@pytest.mark.parametrize("n", [150001, 300000])
def test_voxel_downsample_large_frames_vs_oracle(cuda, n):
    """Real LiDAR frame sizes (100k-300k points): many tiles and buckets per frame, through
    the batched path (a uniform frame, a clumped frame whose dense core overflows a bucket's LDS sort,
    and a frame with points outside every bin) and the drop-in dp.voxel_downsample."""
    import torch
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    rng = np.random.default_rng(n)
    x = rng.uniform(-20, 20, (2, n, 3)).astype(np.float32)
    x[1, : n // 2] *= np.float32(0.002)  # half the frame inside ~0.1 m: a few coarse bins hold it
    xo, vo = _outside_frame(n)
    for xb, voxel in ((x, 0.25), (x, 0.07), (xo[None], vo)):
        c, vid, cnt, nv = (t.cpu().numpy() for t in pn.voxel_downsample_batch(torch.from_numpy(xb).to(cuda), voxel))
        for f in range(len(xb)):
            wc, wvid, wcnt = tier_n.voxel_downsample(xb[f], voxel)
            assert nv[f] == len(wcnt), (voxel, f)
            assert np.array_equal(vid[f], wvid) and np.array_equal(cnt[f, :nv[f]], wcnt), (voxel, f)
            assert np.array_equal(c[f, :nv[f]].view(np.uint32), wc.view(np.uint32)), (voxel, f)
    c, vid, cnt = dp.voxel_downsample(x[0], 0.25)
    wc, wvid, wcnt = tier_n.voxel_downsample(x[0], 0.25)
    assert np.array_equal(vid, wvid) and np.array_equal(cnt, wcnt) and np.array_equal(c, wc)


def test_voxel_downsample_one_huge_voxel(cuda):
    """Every point in one voxel (a voxel larger than the frame): one bucket holds the whole frame and
    sorts it in global memory; the centroid is the index-order fp32 sum."""
    x = uniform_frame(70000, 2, -1, 1).astype(np.float32)
    for v in (100.0, 0.9):
        c, vid, cnt = dp.voxel_downsample(x, v)
        wc, wvid, wcnt = tier_n.voxel_downsample(x, v)
        assert np.array_equal(vid, wvid) and np.array_equal(cnt, wcnt)
        assert np.array_equal(c.view(np.uint32), wc.view(np.uint32))


@pytest.mark.parametrize("name", list(VOXEL_CASES))
def test_voxel_downsample_pinned_to_reference(cuda, name):
    """SURVEY §8a N1's voxel key is calculate_grid_density's grid hash extended to z: the GPU's voxel
    ids, summed over z, divided by v^2, equal the density grid the REFERENCE returned for the frame's
    (x, y) (tests/golden/voxel.npz, captured by gen_voxel.py) bit for bit; ids, counts and centroids
    equal the oracle's."""
    g = np.load(os.path.join(HERE, "golden", "voxel.npz"), allow_pickle=False)
    make, v = VOXEL_CASES[name]
    x = make()
    c, vid, cnt = dp.voxel_downsample(x, v)
    wc, wvid, wcnt = tier_n.voxel_downsample(x, v)
    assert np.array_equal(vid, wvid) and np.array_equal(cnt, wcnt)
    assert np.array_equal(c.view(np.uint32), wc.view(np.uint32))
    bins, dims = tier_n.voxel_bins(x, v)
    hist = tier_n.voxel_counts_xy(vid, cnt, bins, dims)
    want = g[f"{name}__density"]
    assert np.array_equal((hist / (v * v)).view(np.uint64), want.view(np.uint64))


def test_voxel_downsample_errors_like_arange(cuda):
    x = uniform_frame(2000, 4, -1, 1).astype(np.float32)
    x[5, 2] = np.inf
    with pytest.raises(ValueError):
        dp.voxel_downsample(x, 0.1)
    with pytest.raises(ValueError):
        dp.voxel_downsample(uniform_frame(2000, 4, -1, 1).astype(np.float32), 1e-4)  # >= 2^32 keys
    with pytest.raises(ValueError):
        dp.voxel_downsample(uniform_frame(20, 4, -1, 1).astype(np.float32), 0.0)


def test_voxel_single_workgroup_entry_matches_batched(cuda):
    """lidar_voxel_downsample_f32 (one frame, one workgroup; the C-ABI single-frame entry)
    equals the batched chip-wide path, incl. points outside every bin."""
    import torch
    for xn, vv in ((uniform_frame(30000, 5, -1, 1).astype(np.float32), 0.06), _outside_frame(3001)):
        _single_vs_batched(cuda, torch.from_numpy(xn).to(cuda), vv)


def _single_vs_batched(cuda, x, voxel):
    import ctypes
    import torch
    from lidar_ai_recommendation_software_amd import _native as nat
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    n = len(x)
    vid = torch.empty(n, dtype=torch.int32, device=cuda)
    cent = torch.empty((n, 3), dtype=torch.float32, device=cuda)
    cnt = torch.empty(n, dtype=torch.int32, device=cuda)
    v = nat.I64(0)
    nat.call("lidar_voxel_downsample_f32", nat.handle(0), nat.ptr(x), n, voxel, nat.ptr(vid), nat.ptr(cent),
             nat.ptr(cnt), ctypes.byref(v), nat.stream_ptr())
    c2, vid2, cnt2, nv = pn.voxel_downsample_batch(x[None].contiguous(), voxel)
    v = v.value
    assert int(nv[0]) == v
    assert torch.equal(vid, vid2[0]) and torch.equal(cnt[:v], cnt2[0, :v])
    assert torch.equal(cent[:v].view(torch.int32), c2[0, :v].view(torch.int32))


# ------------------------------------------------- boundary (round 2)
def test_wide_and_narrow_frames_raise_like_reference(cuda):
    """(N, k > 3): the reference raises ValueError unpacking np.min(inliers, axis=0) into three
    names (utils/data_processing.py:207) — IndexError first when the k-column 3-sigma filter keeps
    nothing; (N, 2): IndexError at points[:, 2]; the variant pipeline raises the same."""
    pts4 = np.column_stack([uniform_frame(3000, 3), np.arange(3000.0)])
    for fn in (dp.preprocess_lidar_data, vp.preprocess_point_cloud):
        with pytest.raises(ValueError, match="too many values to unpack"):
            fn(pts4)
        with pytest.raises(IndexError):
            fn(uniform_frame(100, 1)[:, :2])
        bad = pts4.copy()
        bad[7, 3] = np.nan  # NaN std: nothing strictly inside 3 sigma
        with pytest.raises(IndexError):
            fn(bad)


def test_in_place_edits_are_seen(cuda):
    """The device cache never serves stale data: editing pd["points"], pd["clusters"] or the
    returned people array in place changes the results exactly as it changes the reference's."""
    pd = dp.preprocess_lidar_data(FRAMES["lattice_8163_s4"]())
    before = dp.extract_people_positions(pd)
    pd["points"][:, :2] += 100.0
    got = dp.extract_people_positions(pd)
    assert not np.array_equal(got, before)
    assert np.array_equal(got, tier_r.extract_people_positions(pd))
    pd["clusters"][pd["clusters"] > 3] = 0
    assert np.array_equal(dp.extract_people_positions(pd), tier_r.extract_people_positions(pd))
    people = dp.extract_people_positions(pd)
    dims = pd["dimensions"]
    people[0] = (dims["x_range"][1] + 50.0, dims["y_range"][1] + 50.0)  # moved out of the grid
    a = dp.calculate_grid_density(people, (dims["x_range"][0] + 100, dims["x_range"][1] + 100),
                                  (dims["y_range"][0] + 100, dims["y_range"][1] + 100))
    b = tier_r.calculate_grid_density(people, (dims["x_range"][0] + 100, dims["x_range"][1] + 100),
                                      (dims["y_range"][0] + 100, dims["y_range"][1] + 100))
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


@pytest.mark.parametrize("name", ["small_12", "uniform_16384_s0", "uniform_65536_s0"])
def test_density_model_backbone_option(cuda, name):
    """CrowdDensityModel(backbone="ssg"): the reference's keys and values are
    unchanged, and backbone_feature is the SSG stack over ALL the frame's inlier points
    (normalised to its bounding box) — vs the oracle at 1e-4."""
    import torch  # noqa: F401
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    pd = dp.preprocess_lidar_data(FRAMES[name]())
    base = CrowdDensityModel().analyze(pd)
    m = CrowdDensityModel(backbone="ssg")
    res = m.analyze(pd)
    assert set(res) == set(base) | {"backbone_feature", "backbone_weights"}
    assert res["backbone_weights"] == "random-init"
    assert res["total_people"] == base["total_people"] and res["hotspots"] == base["hotspots"]
    assert np.array_equal(res["density_map"], base["density_map"])
    unit = CrowdDensityModel.normalise(pd["points"])
    want, _ = tier_n.sa_stack(unit, {"levels": pn.resolve(pn.SSG, len(unit))}, m._net.weights)
    got = res["backbone_feature"]
    scale = np.sqrt(np.mean(want.astype(np.float64) ** 2)) + 1e-30
    assert got.shape == (1024,) and np.all(np.abs(got - want) <= 1e-4 * np.abs(want) + 1e-4 * scale)


def test_density_model_backbone_large_frame(cuda):
    """The backbone over a frame of more than 262 144 inlier points: the SSG
    stack runs over all of them (FPS on 64 x PPL-point buckets) and matches the oracle at 1e-4."""
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    pts = uniform_frame(300000, 5, -15, 15)
    pd = dp.preprocess_lidar_data(pts)
    assert len(pd["points"]) > 262144
    m = CrowdDensityModel(backbone="ssg")
    res = m.analyze(pd)
    unit = CrowdDensityModel.normalise(pd["points"])
    want, _ = tier_n.sa_stack(unit, {"levels": pn.resolve(pn.SSG, len(unit))}, m._net.weights)
    got = res["backbone_feature"]
    scale = np.sqrt(np.mean(want.astype(np.float64) ** 2)) + 1e-30
    assert got.shape == (1024,) and np.all(np.abs(got - want) <= 1e-4 * np.abs(want) + 1e-4 * scale)


@pytest.mark.parametrize("via", ["arrays", "npz"])
def test_density_model_backbone_supplied_weights(cuda, tmp_path, via):
    """CrowdDensityModel(backbone="ssg", backbone_weights=...): supplied weights (other
    than the seed-0 init) change the feature, which matches the oracle's sa_stack with those weights at
    1e-4, and the result says so; backbone=None stays the reference's dict, key for key and byte for byte;
    a weight set of the wrong shape fails at construction."""
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    pd = dp.preprocess_lidar_data(FRAMES["uniform_16384_s0"]())
    w = pn.init_weights(pn.SSG, 77)
    arg = w
    if via == "npz":
        arg = str(tmp_path / "ssg.npz")
        pn.save_weights(arg, w)
    m = CrowdDensityModel(backbone="ssg", backbone_weights=arg)
    res = m.analyze(pd)
    assert res["backbone_weights"] == "supplied"
    rnd = CrowdDensityModel(backbone="ssg").analyze(pd)["backbone_feature"]
    unit = CrowdDensityModel.normalise(pd["points"])
    want, _ = tier_n.sa_stack(unit, {"levels": pn.resolve(pn.SSG, len(unit))}, w)
    got = res["backbone_feature"]
    scale = np.sqrt(np.mean(want.astype(np.float64) ** 2)) + 1e-30
    assert np.all(np.abs(got - want) <= 1e-4 * np.abs(want) + 1e-4 * scale)
    assert not np.allclose(got, rnd, rtol=1e-2, atol=1e-3 * scale)
    base = CrowdDensityModel().analyze(pd)
    ref = tier_r.analyze(pd) if hasattr(tier_r, "analyze") else None
    assert "backbone_feature" not in base and "backbone_weights" not in base
    if ref is not None:
        assert set(base) == set(ref) and np.array_equal(base["density_map"], ref["density_map"])
    bad = pn.init_weights(pn.MSG, 0)
    with pytest.raises(ValueError, match="weights"):
        CrowdDensityModel(backbone="ssg", backbone_weights=bad)


def test_downsample_point_cloud_device_gather(cuda):
    """A13: the draw is the global legacy RNG's (same indices and RNG state as the reference),
    the gather runs on the GPU — numpy in / numpy out of any dtype, CUDA tensor in / out."""
    import torch
    base = uniform_frame(5000, 2)
    for arr in (base, base.astype(np.float32), np.floor(base * 10).astype(np.int64), base[:, 0].copy()):
        np.random.seed(7)
        got = dp.downsample_point_cloud(arr, 0.13)
        after = np.random.random()
        np.random.seed(7)
        want = arr[np.random.choice(len(arr), max(1, int(len(arr) * 0.13)), replace=False)]
        assert np.random.random() == after
        assert got.dtype == want.dtype and got.shape == want.shape and np.array_equal(got, want)
    np.random.seed(3)
    got = dp.downsample_point_cloud(torch.from_numpy(base).cuda(), 0.5)
    np.random.seed(3)
    want = base[np.random.choice(5000, 2500, replace=False)]
    assert got.is_cuda and np.array_equal(got.cpu().numpy(), want)
    assert dp.downsample_point_cloud(base, 1.0) is base


@pytest.mark.parametrize("case", ["spread", "line", "two_far"])
def test_dbscan_coarse_grid_path_vs_oracle(cuda, case):
    """DBSCAN's two grids: frames whose eps/sqrt(3) cells would exceed the cell cap take the coarse
    grid (cells > eps, no same-cell shortcut, per-point union) — exact like the fine one."""
    import torch
    from lidar_ai_recommendation_software_amd import _native as nat
    x = lattice_frame(3, 60, 100, 5, 3.0, 0.3)
    if case == "spread":
        x = x * np.array([400.0, 400.0, 1.0])
    elif case == "line":
        x[:, 0] *= 1e4
    else:
        x[::2] += 1e6
    for eps in (0.3, 0.5):
        want, wcnt = tier_r.dbscan_labels(x, eps, 5, return_counts=True)
        xt = torch.from_numpy(np.ascontiguousarray(x)).cuda()
        lab = torch.empty(len(x), dtype=torch.int64, device="cuda")
        cnt = torch.empty(len(x), dtype=torch.int32, device="cuda")
        nat.call("lidar_dbscan_f64", nat.handle(0), nat.ptr(xt), len(x), float(eps), 5, nat.ptr(lab), nat.ptr(cnt),
                 nat.stream_ptr())
        assert np.array_equal(cnt.cpu().numpy(), wcnt)
        assert np.array_equal(lab.cpu().numpy(), want), case
        nat.call("lidar_dbscan_f64", nat.handle(0), nat.ptr(xt), len(x), float(eps), 5, nat.ptr(lab), None,
                 nat.stream_ptr())  # counts stop at min_samples without the counts output
        assert np.array_equal(lab.cpu().numpy(), want), case


@pytest.mark.parametrize("seed,eps,ms", [(0, 0.5, 5), (1, 0.2, 5), (2, 0.45, 1), (3, 0.5, 12), (4, 0.31, 3)])
def test_dbscan_fine_grid_vs_oracle(cuda, seed, eps, ms):
    """The fine grid (cells of eps/sqrt(3): same-cell shortcut, cell-pair links) on standardized
    crowd and blob frames, several min_samples: labels and exact counts equal the oracle's."""
    import torch
    from lidar_ai_recommendation_software_amd import _native as nat
    from oracle.tier_r import standard_scale
    pts = crowd_frame(20000, 40 + seed) if seed % 2 else blob_frame(120, 80, 2000, seed, 12, 0.5)
    x = standard_scale(pts)[0]
    want, wcnt = tier_r.dbscan_labels(x, eps, ms, return_counts=True)
    xt = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    lab = torch.empty(len(x), dtype=torch.int64, device="cuda")
    cnt = torch.empty(len(x), dtype=torch.int32, device="cuda")
    nat.call("lidar_dbscan_f64", nat.handle(0), nat.ptr(xt), len(x), float(eps), ms, nat.ptr(lab), nat.ptr(cnt),
             nat.stream_ptr())
    assert np.array_equal(cnt.cpu().numpy(), wcnt)
    assert np.array_equal(lab.cpu().numpy(), want)
    nat.call("lidar_dbscan_f64", nat.handle(0), nat.ptr(xt), len(x), float(eps), ms, nat.ptr(lab), None,
             nat.stream_ptr())
    assert np.array_equal(lab.cpu().numpy(), want)


def test_venue_grid_equals_grid_density_of_all_people(cuda):
    """people of many frames binned into one fixed venue grid equal
    calculate_grid_density of all those people over the venue extent, bit for bit."""
    from lidar_ai_recommendation_software_amd.global_density import VenueGrid
    frames = [FRAMES[k]() for k in ("crowd_16384_s7", "lattice_8163_s4", "blobs_4293_s0", "uniform_4096_s1")]
    people = [dp.extract_people_positions(dp.preprocess_lidar_data(f)) for f in frames]
    people = [p for p in people if len(p)]
    xr, yr = (-16.0, 16.5), (-15.5, 16.0)
    vg = VenueGrid(xr, yr, 1.0)
    for p in people:
        vg.add(p)
    gx, gy, dens = tier_r.calculate_grid_density(np.concatenate(people), xr, yr, 1.0)
    assert np.array_equal(vg.density(), dens)
    cx, cy = vg.centres()
    assert np.array_equal(cx, gx) and np.array_equal(cy, gy)
    edge = np.array([[xr[0] - 2.0, yr[0] - 2.0], [xr[1] + 2.0, yr[1] + 2.0], [xr[1] + 3.0, 0.0], [0.0, np.nan]])
    vg2 = VenueGrid(xr, yr, 1.0).add(edge)  # on the first edge, on the last edge (closed), outside, NaN
    assert np.array_equal(vg2.density(), tier_r.calculate_grid_density(edge, xr, yr, 1.0)[2])


def test_host_frame_feed_matches_drop_in(cuda, tmp_path):
    """frame_feed.HostFrameFeed (pinned staging + H2D on a copy stream + batched kernels) gives the
    drop-in API's analyze dict for every frame, from arrays and from files; errors as the reference."""
    from lidar_ai_recommendation_software_amd.frame_feed import HostFrameFeed
    names = ["uniform_16384_s0", "small_12", "crowd_16384_s7", "int_4096", "lattice_8163_s4", "small_20", "dup_4096"]
    frames = [FRAMES[k]() for k in names]
    for lanes in (1, 2, 3):  # one batch at a time (run_batch), and batches in flight (run_batches)
        got = HostFrameFeed(batch=2 if lanes == 2 else 3, lanes=lanes).run(frames)
        assert len(got) == len(frames)
        for name, f, g in zip(names, frames, got):
            _same_analyze(name, g, CrowdDensityModel().analyze(dp.preprocess_lidar_data(f)))
    feed = HostFrameFeed(batch=3)
    paths = []
    for i, f in enumerate(frames[:3]):
        p = tmp_path / f"f{i}.pcd"
        with open(p, "w") as fh:
            fh.write(f"VERSION .7\nFIELDS x y z\nPOINTS {len(f)}\nDATA ascii\n")
            fh.writelines(f"{a!r} {b!r} {c!r}\n" for a, b, c in np.asarray(f, dtype=np.float64).tolist())
        paths.append(str(p))
    for name, g in zip(names, feed.run_files(paths)):
        _same_analyze(name, g, CrowdDensityModel().analyze(dp.preprocess_lidar_data(dp.load_lidar_data(
            paths[names.index(name)]))))
    with pytest.raises(IndexError):
        feed.run([frames[0], ERROR_FRAMES["const_col"]()])
    # the first bad frame's exception, in frame order, whichever stage finds it: a kernel-side IndexError in
    # batch 0 beats a staging-side ValueError (an empty frame) in batch 1 of the same window
    with pytest.raises(IndexError):
        HostFrameFeed(batch=2, lanes=3).run([frames[0], ERROR_FRAMES["const_col"](), np.zeros((0, 3))])
    with pytest.raises(ValueError):
        HostFrameFeed(batch=2, lanes=3).run([frames[0], frames[1], np.zeros((0, 3))])


@pytest.mark.parametrize("kind", STRESS_KINDS)
def test_preprocess_chain_stress_vs_oracle(cuda, kind):
    """preprocess_lidar_data on frames built against the chain emulation and the ground-plane fit
    == the oracle's numpy / scikit-learn restatement of the reference: byte for byte, the plane by
    check_plane (gelsd's rank decision and truncated minimum-norm solution; `cancel`, `tiny`,
    `offset_ties`, `far_1e8` and `collinear` are rank-deficient for rcond = eps * M)."""
    pts = stress_frame(kind)
    try:
        want = tier_r.preprocess_lidar_data(pts.copy())
    except Exception as e:  # noqa: BLE001 — the reference's exception is the expected result
        with pytest.raises(type(e)):
            dp.preprocess_lidar_data(pts)
        return
    got = dp.preprocess_lidar_data(pts)
    for k in ("points", "colors", "normals", "clusters"):
        a, b = np.asarray(got[k]), np.asarray(want[k])
        assert a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes(), f"{kind}.{k}"
    for k in ("x_range", "y_range", "z_range"):
        assert [float(v).hex() for v in got["dimensions"][k]] == [float(v).hex() for v in want["dimensions"][k]]
    check_plane(kind, got["ground_plane"], want["ground_plane"], want["points"])
