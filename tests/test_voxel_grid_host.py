"""The voxel binning the kernels run (csrc/voxel_grid.hpp: make_grid, bin, key, and the keys launch's
float-threshold tables: ru_float, faxis, bin_tab_c / bin_tab_search / bin_of_c), compiled for the host
(tests/host/voxel_grid_host.cpp, hipcc, -ffp-contract=off as the library) and compared with
oracle/tier_n.voxel_bins — numpy's searchsorted on np.arange edges, itself pinned to the reference's
calculate_grid_density (test_oracle.py::test_voxel_bins_pinned_to_reference) — on the golden frames and
on frames built to miss the spacing guess (far offsets, voxel sizes that are not binary fractions, points
one ulp either side of an edge, the last edge)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from golden.voxel_cases import VOXEL_CASES
from oracle import tier_n

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "lidar_ai_recommendation_software_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    exe = str(tmp_path_factory.mktemp("vgh") / "voxel_grid_host")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC,
                    os.path.join(HERE, "host", "voxel_grid_host.cpp"), "-o", exe], check=True)
    return exe


def run(exe, x, v):
    x = np.ascontiguousarray(x, dtype=np.float32)
    inp = np.array([len(x)], np.int64).tobytes() + np.array([v], np.float64).tobytes() + x.tobytes()
    out = subprocess.run([exe], input=inp, capture_output=True, check=True).stdout
    head = np.frombuffer(out[:32], np.int64)
    if not head[0]:
        return None, None, None
    n = len(x)
    bins = np.frombuffer(out[32:32 + 24 * n], np.int64).reshape(n, 3)
    o = 32 + 24 * n
    keys = np.frombuffer(out[o:o + 4 * n], np.uint32)
    run.tab = int(np.frombuffer(out[o + 4 * n:o + 4 * n + 8], np.int64)[0])
    run.fbins = np.frombuffer(out[o + 4 * n + 8:], np.int64).reshape(n, 3)
    return bins, tuple(int(d) for d in head[1:]), keys


def near_edges(seed, v, lo, n=3000, bins=40, yz_bins=None):
    """Points at, one ulp below and one ulp above the float32 values nearest to interior edges."""
    rng = np.random.default_rng(seed)
    span = np.array([bins, yz_bins or bins, yz_bins or bins]) * v
    x = (rng.random((n, 3)) * span + lo).astype(np.float32)
    e = tier_n.voxel_edges(float(x[:, 0].min()), float(x[:, 0].max()), v)
    pick = e[rng.integers(2, len(e) - 2, n // 3)].astype(np.float32)
    x[: n // 3, 0] = pick
    x[n // 3: 2 * n // 3, 0] = np.nextafter(pick, np.float32(-np.inf))
    x[2 * n // 3: 3 * (n // 3), 0] = np.nextafter(pick, np.float32(np.inf))
    return x


ADVERSARIAL = {
    "far_1e6_v0.1": (lambda: (np.random.default_rng(1).random((4000, 3)) * 3 + 1.0e6).astype(np.float32), 0.1),
    "far_2p30_fine": (lambda: (np.float64(2 ** 30 + 1024) + np.random.default_rng(2).integers(0, 64, (2000, 3)) * 128.0)
                      .astype(np.float32), 3.3 * 2 ** -22 * 1e4),
    "v_0.3_near_edges": (lambda: near_edges(3, 0.3, -5.0), 0.3),
    "v_0.07_near_edges": (lambda: near_edges(4, 0.07, 123.0), 0.07),
    "v_1e-3_near_edges": (lambda: near_edges(5, 1e-3, 0.5), 1e-3),
    # about 8000 bins on x: the widest tables; 9000: past them (float64 key())
    "tab_8000_bins": (lambda: near_edges(7, 0.05, -77.7, n=6000, bins=8000, yz_bins=30), 0.05),
    "tab_9000_bins": (lambda: near_edges(8, 0.05, 31.3, n=6000, bins=9000, yz_bins=30), 0.05),
    "negative_far": (lambda: (np.random.default_rng(6).random((3000, 3)) * -50 - 2.5e4).astype(np.float32), 0.37),
}


def outside_frame(n=999):
    """Points near 2^30 with a voxel of 3.3 float64 ulps there (tests/test_gpu_tier_r.py::_outside_frame):
    the edges stop short of the extent, a third of the points lies outside every bin."""
    lo = np.float32(2.0 ** 30 + 1024)
    x = np.zeros((n, 3), np.float32)
    x[:, 0] = np.where(np.arange(n) % 3 == 1, lo + np.float32(128), lo)
    x[:, 1] = np.float32(0.5)
    x[:, 2] = np.float32(-0.25)
    return x


ADVERSARIAL["outside_2p30"] = (outside_frame, 3.3 * 2.0 ** -22)


K_TAB_EDGES = 8192  # csrc/voxel_grid.hpp kTabEdges: a finer axis runs lidar_vox::key in float64


@pytest.mark.parametrize("name", sorted(VOXEL_CASES) + sorted(ADVERSARIAL))
def test_kernel_binning_equals_oracle(harness, name):
    make, v = (VOXEL_CASES.get(name) or ADVERSARIAL[name])
    x = make()
    bins, dims, keys = run(harness, x, v)
    try:
        want, wdims = tier_n.voxel_bins(x, v)
    except ValueError:  # a grid of 2^32 keys or more: the kernels refuse it too (nvox -1)
        assert bins is None
        return
    assert dims == wdims
    bad = np.flatnonzero((bins != want).any(axis=1))
    assert bad.size == 0, f"{bad.size} points binned differently, first {x[bad[:3]]}: {bins[bad[:3]]} vs {want[bad[:3]]}"
    # the keys launch's float tables (csrc/voxel_grid.hpp kTabEdges edges per axis at most): the same bins
    assert run.tab == int(all(d + 1 <= K_TAB_EDGES for d in dims))
    bad = np.flatnonzero((run.fbins != want).any(axis=1))
    assert bad.size == 0, (f"float tables: {bad.size} points binned differently, first {x[bad[:3]]}: "
                           f"{run.fbins[bad[:3]]} vs {want[bad[:3]]}")
    inside = (want >= 0).all(axis=1)
    wkey = (want[:, 0] * wdims[1] + want[:, 1]) * wdims[2] + want[:, 2]
    assert np.array_equal(keys[inside], wkey[inside].astype(np.uint32))
    assert (keys[~inside] == 0xffffffff).all()
    if name.startswith("tab_"):
        assert run.tab == int(name == "tab_8000_bins")
    if name == "outside_2p30":
        assert 0 < (~inside).sum() < len(x)


def test_grid_limits_match_oracle(harness):
    # >= 2^32 - 1 keys: both refuse
    x = np.array([[0, 0, 0], [1000, 1000, 10]], np.float32)
    assert run(harness, x, 0.05)[0] is None
    with pytest.raises(ValueError):
        tier_n.voxel_bins(x, 0.05)
