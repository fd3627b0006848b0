"""CPU tests of the drop-in boundary's host logic (no GPU): the reference's error conventions
that are decided before any kernel runs, and calculate_risk_level
(``models/crowd_density_model.py:100-117``)."""
import numpy as np
import pytest

from lidar_ai_recommendation_software_amd import data_processing as dp
from lidar_ai_recommendation_software_amd.crowd_density_model import CrowdDensityModel


@pytest.mark.parametrize("density,want", [(0.0, "Low"), (0.999, "Low"), (1.0, "Moderate"), (2.49, "Moderate"),
                                          (2.5, "High"), (3.99, "High"), (4.0, "Critical"), (1e9, "Critical"),
                                          (-1.0, "Low"), (np.float64(2.5), "High")])
def test_calculate_risk_level(density, want):
    # models/crowd_density_model.py:100-117: < 1 Low, < 2.5 Moderate, < 4 High, else Critical
    assert CrowdDensityModel().calculate_risk_level(density) == want


def test_risk_level_nan_is_critical():
    # every comparison with NaN is False: the reference falls through to "Critical"
    assert CrowdDensityModel().calculate_risk_level(float("nan")) == "Critical"


@pytest.mark.parametrize("shape", [(0, 2), (5, 2), (5, 1), (7,), (0,)])
def test_preprocess_narrow_input_raises_index_error(shape):
    # the reference indexes points[:, 2] first (utils/data_processing.py:143)
    with pytest.raises(IndexError):
        dp.preprocess_lidar_data(np.zeros(shape))


def test_preprocess_empty_frame_raises_value_error():
    # np.min of an empty column (utils/data_processing.py:143)
    with pytest.raises(ValueError):
        dp.preprocess_lidar_data(np.zeros((0, 3)))
    with pytest.raises(ValueError):
        dp.preprocess_lidar_data(np.zeros((0, 5)))


def test_preprocess_wide_input_raises_like_reference():
    # (N, k > 3): the reference's 3-sigma mask and DBSCAN use all k columns, then unpacking
    # np.min(inlier_points, axis=0) into three names raises ValueError (:207); a frame whose
    # k-column 3-sigma filter keeps nothing raises IndexError from np.percentile first (:164)
    rng = np.random.default_rng(0)
    with pytest.raises(ValueError, match="too many values to unpack"):
        dp.preprocess_lidar_data(rng.uniform(-15, 15, (500, 4)))
    const4 = rng.uniform(-15, 15, (500, 4))
    const4[:, 3] = 1.0  # a constant column: std 0, nothing is strictly inside 3 sigma
    with pytest.raises(IndexError):
        dp.preprocess_lidar_data(const4)


def test_downsample_host_input_is_reference_indexing():
    """downsample_point_cloud (utils/data_processing.py:231-249) on host input is the reference's
    own ``points[np.random.choice(...)]`` on the host: same rows, same global RNG state after, same
    exception for a Python list (no GPU, no PCIe round trip)."""
    from lidar_ai_recommendation_software_amd.synthetic import uniform_frame
    base = uniform_frame(3000, 4)
    for arr in (base, base.astype(np.float32), np.floor(base * 10).astype(np.int64), base[:, 0].copy()):
        np.random.seed(11)
        got = dp.downsample_point_cloud(arr, 0.21)
        after = np.random.random()
        np.random.seed(11)
        want = arr[np.random.choice(len(arr), max(1, int(len(arr) * 0.21)), replace=False)]
        assert np.random.random() == after
        assert got.dtype == want.dtype and np.array_equal(got, want)
    assert dp.downsample_point_cloud(base, 1.0) is base
    with pytest.raises(TypeError):
        dp.downsample_point_cloud(base.tolist(), 0.5)


def test_device_cache_digest_without_xxhash():
    """xxhash is optional: with it hidden, the device-cache digest falls back to the
    standard library's blake2b and still tells edited arrays apart."""
    import subprocess
    import sys
    code = ("import sys; sys.modules['xxhash'] = None\n"
            "import numpy as np\n"
            "from lidar_ai_recommendation_software_amd import data_processing as dp\n"
            "assert dp._xxhash is None\n"
            "a = np.arange(30.0).reshape(10, 3); d0 = dp._digest(a); a[3, 1] += 1e-9\n"
            "assert dp._digest(a) != d0 and dp._digest(a) == dp._digest(a.copy())\n"
            "print('ok')\n")
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=repo, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


@pytest.mark.parametrize("x_max,err", [(1e13, MemoryError), (1e12, MemoryError), (float("inf"), ValueError),
                                       (1e300, ValueError), (float("nan"), ValueError), (2e18, ValueError)])
def test_grid_dims_errors_match_numpy(x_max, err):
    """calculate_grid_density's grid (utils/data_processing.py:305-319) for extreme extents: the
    error type numpy's np.arange raises for the same edges (a length it cannot hold or compute:
    ValueError; a representable but unallocatable grid: MemoryError)."""
    from lidar_ai_recommendation_software_amd import _native as nat
    with pytest.raises(err):
        np.arange(0.0 - 2.0, (x_max + 2.0) + 1.0, 1.0) if err is ValueError else nat.grid_dims(0.0, x_max, 0.0, 1.0, 1.0)
    with pytest.raises(err):
        nat.grid_dims(0.0, x_max, 0.0, 1.0, 1.0)
    assert nat.grid_dims(0.0, 30.0, -15.0, 15.0, 1.0) == (34, 34)


def test_backbone_weights_roundtrip_and_validation(tmp_path):
    """pointnet2.save_weights / load_weights (plain .npz, no pickles) round-trip bit for bit; check_weights
    names the first mismatch; CrowdDensityModel refuses weights without a backbone (no GPU needed)."""
    import numpy as np
    import pytest
    from lidar_ai_recommendation_software_amd import pointnet2 as pn
    from lidar_ai_recommendation_software_amd.crowd_density_model import CrowdDensityModel
    for cfg in (pn.SSG, pn.MSG):
        w = pn.init_weights(cfg, 5)
        p = tmp_path / f"{cfg['name']}.npz"
        pn.save_weights(str(p), w)
        got = pn.load_weights(str(p), cfg)
        for la, lb in zip(w, got):
            for ba, bb in zip(la, lb):
                for (wa, ca), (wb, cb) in zip(ba, bb):
                    assert np.array_equal(wa, wb) and np.array_equal(ca, cb)
    w = pn.init_weights(pn.SSG, 0)
    w[1][0][2] = (w[1][0][2][0][:, :100], w[1][0][2][1][:100])
    with pytest.raises(ValueError, match="level 1 branch 0 layer 2"):
        pn.check_weights(pn.SSG, w)
    with pytest.raises(ValueError, match="without a backbone"):
        CrowdDensityModel(backbone_weights=pn.init_weights(pn.SSG, 0))
    m = CrowdDensityModel(backbone="ssg", backbone_weights=str(tmp_path / "ssg.npz"))
    assert m._weights is not None
