"""Drop-in for the reference's ``models/crowd_flow_model.py``.

``CrowdFlowModel().analyze(processed_data)`` returns the reference's dict — flow vectors on
the 1 m grid of the frame's extent, average speed, dominant direction and up to five
bottlenecks — bit for bit (``tests/test_flow.py``, ``tests/golden/flow.json`` captured from
the reference itself).  People positions come from the GPU path
(``data_processing.extract_people_positions``); the flow field and the bottleneck search run
in the library's native host code (``csrc/flow.hip``): every deciding operation there is a
glibc ``sin`` / ``cos`` / ``pow`` call or an sklearn KD-tree traversal that only the host C
library reproduces exactly, on a few thousand grid nodes.
"""
import ctypes

import numpy as np

from . import _native as nat
from .data_processing import extract_people_positions


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class CrowdFlowModel:
    """``models/crowd_flow_model.py:6-279``: same attributes, methods and outputs."""

    def __init__(self):
        self.prev_positions = None
        self.flow_vectors = None
        self.simulation_params = {
            "flow_field_complexity": 2,
            "bottleneck_count": 3,
            "flow_speed_range": (0.2, 1.5),
            "random_seed": 42,
        }

    def analyze(self, processed_data):
        """``crowd_flow_model.py:28-86``."""
        people_positions = extract_people_positions(processed_data)
        if len(people_positions) == 0:
            return {"flow_vectors": {"positions": np.zeros((0, 2)), "vectors": np.zeros((0, 2)),
                                     "magnitudes": np.zeros(0)},
                    "avg_speed": 0.0, "dominant_direction": "N/A", "bottlenecks": []}
        flow_vectors = self._generate_simulated_flow(people_positions, processed_data)
        magnitudes = flow_vectors["magnitudes"]
        vectors = flow_vectors["vectors"]
        avg_speed = np.mean(magnitudes)
        if len(vectors) > 0:  # the reference's scalar epilogue, same numpy calls
            avg_vector = np.mean(vectors, axis=0)
            angle = np.arctan2(avg_vector[1], avg_vector[0]) * 180 / np.pi
            directions = ["E", "NE", "N", "NW", "W", "SW", "S", "SE", "E"]
            dominant_direction = directions[int((angle + 22.5) % 360 / 45)]
        else:
            dominant_direction = "N/A"
        bottlenecks = self._identify_bottlenecks(flow_vectors, processed_data)
        return {"flow_vectors": flow_vectors, "avg_speed": avg_speed,
                "dominant_direction": dominant_direction, "bottlenecks": bottlenecks}

    def _generate_simulated_flow(self, people_positions, processed_data):
        """``crowd_flow_model.py:88-184``.  Seeds and draws the GLOBAL legacy NumPy RNG
        exactly as the reference does (seed 42, then two uniforms per bottleneck)."""
        np.random.seed(self.simulation_params["random_seed"])
        x_range = processed_data["dimensions"]["x_range"]
        y_range = processed_data["dimensions"]["y_range"]
        grid_size = 1.0
        x_grid = np.ascontiguousarray(np.arange(x_range[0], x_range[1] + grid_size, grid_size), dtype=np.float64)
        y_grid = np.ascontiguousarray(np.arange(y_range[0], y_range[1] + grid_size, grid_size), dtype=np.float64)
        exit_x = x_range[1]
        exit_y = (y_range[0] + y_range[1]) / 2
        nb = self.simulation_params["bottleneck_count"]
        bn = np.empty((nb, 2), dtype=np.float64)
        for k in range(nb):
            bn[k, 0] = np.random.uniform(x_range[0] + 1, x_range[1] - 1)
            bn[k, 1] = np.random.uniform(y_range[0] + 1, y_range[1] - 1)
        m = len(x_grid) * len(y_grid)
        positions = np.empty((m, 2), dtype=np.float64)
        vectors = np.empty((m, 2), dtype=np.float64)
        magnitudes = np.empty(m, dtype=np.float64)
        lo, hi = self.simulation_params["flow_speed_range"]
        nat.check(nat.load_library().lidar_flow_field_f64(
            _p(x_grid), len(x_grid), _p(y_grid), len(y_grid), float(exit_x), float(exit_y),
            int(self.simulation_params["flow_field_complexity"]), _p(bn), nb, float(lo), float(hi),
            _p(positions), _p(vectors), _p(magnitudes)), "lidar_flow_field_f64")
        return {"positions": positions, "vectors": vectors, "magnitudes": magnitudes}

    def _identify_bottlenecks(self, flow_vectors, processed_data):
        """``crowd_flow_model.py:186-279``: nodes slower than 0.5 m/s with >= 5 neighbours
        within 3 m and >= 3 more within 5 m; severity from the speed gradient and the flow
        convergence; top 5 by severity (stable)."""
        positions = np.ascontiguousarray(flow_vectors["positions"], dtype=np.float64)
        vectors = np.ascontiguousarray(flow_vectors["vectors"], dtype=np.float64)
        magnitudes = np.ascontiguousarray(flow_vectors["magnitudes"], dtype=np.float64)
        m = len(positions)
        if m == 0:
            return []
        cap = m
        ox, oy = np.empty(cap), np.empty(cap)
        osev = np.empty(cap, dtype=np.int64)
        n = nat.I64(0)
        nat.check(nat.load_library().lidar_flow_bottlenecks_f64(
            _p(positions), _p(vectors), _p(magnitudes), m, 0.5, 3.0, 5.0, 5, 3, _p(ox), _p(oy), _p(osev), None,
            cap, ctypes.byref(n)), "lidar_flow_bottlenecks_f64")
        n = n.value
        cand = [{"x": positions[0, 0].dtype.type(ox[i]), "y": positions[0, 0].dtype.type(oy[i]),
                 "severity": int(osev[i])} for i in range(n)]
        return sorted(cand, key=lambda b: b["severity"], reverse=True)[:5]
