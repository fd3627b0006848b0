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
