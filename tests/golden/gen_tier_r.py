"""Capture Tier-R golden vectors by running the REFERENCE itself (this container only).

SURVEY.md §8c: ``utils.data_processing`` and ``models.crowd_density_model``
import and run from ``/root/reference`` here.  This script imports them
read-only (no bytecode written), runs the reference CPU path
(``preprocess_lidar_data`` -> ``CrowdDensityModel().analyze``,
``utils/data_processing.py:127-328``, ``models/crowd_density_model.py:23-98``)
on seeded synthetic frames and writes what it returned:

* ``tier_r.json`` — per case: sha256 + shape + dtype of every output array,
  float scalars as ``float.hex``, exception types for the edge cases;
* ``tier_r.npz`` — small arrays (labels of the <=16 384-point cases, ground
  planes, people positions, density maps, hotspots, downsample picks).

The reference never travels to the GPU box; only these files do.
Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_tier_r.py
"""
import hashlib
import json
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")

from utils.data_processing import (preprocess_lidar_data, extract_people_positions,  # noqa: E402
                                   downsample_point_cloud)
from models.crowd_density_model import CrowdDensityModel  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import (uniform_frame, crowd_frame,  # noqa: E402
                                                        blob_frame, lattice_frame,
                                                        stress_frame, STRESS_KINDS)


def sha(a):
    a = np.ascontiguousarray(a)
    return {"sha256": hashlib.sha256(a.tobytes()).hexdigest(), "shape": list(a.shape), "dtype": str(a.dtype)}


def fhex(v):
    return float(v).hex()


# Case table: name -> (points factory, keep full labels in the npz?)
CASES = {}
for n in (4096, 16384):
    for s in (0, 1, 2):
        CASES[f"uniform_{n}_s{s}"] = (lambda n=n, s=s: uniform_frame(n, s), True)
CASES["uniform_65536_s0"] = (lambda: uniform_frame(65536, 0), False)
CASES["uniform_65536_s1"] = (lambda: uniform_frame(65536, 1), False)
CASES["uniform_131072_s0"] = (lambda: uniform_frame(131072, 0), False)
CASES["crowd_10000_s42"] = (lambda: crowd_frame(10000, 42), True)
CASES["crowd_16384_s7"] = (lambda: crowd_frame(16384, 7), True)
CASES["crowd_65536_s3"] = (lambda: crowd_frame(65536, 3), False)
# clumpy frames: tens of clusters, border points, sub-min_samples blobs, noise
CASES["lattice_4293_s0"] = (lambda: lattice_frame(4, 60, 150, 0), True)
CASES["lattice_8163_s4"] = (lambda: lattice_frame(4, 120, 60, 4, 15, 0.4), True)
CASES["lattice_15636_s1"] = (lambda: lattice_frame(4, 250, 100, 1, 15, 0.3), True)
CASES["lattice_62978_s2"] = (lambda: lattice_frame(4, 1000, 100, 2, 15, 0.3), False)
CASES["blobs_4293_s0"] = (lambda: blob_frame(60, 60, 300, 0, 15, 0.6), True)
CASES["blobs_8980_s1"] = (lambda: blob_frame(200, 40, 500, 1, 15, 0.3), True)
# small / degenerate frames that still run (SURVEY §8b error table)
CASES["small_12"] = (lambda: uniform_frame(12, 5), True)
CASES["small_20"] = (lambda: uniform_frame(20, 5), True)
CASES["small_40"] = (lambda: uniform_frame(40, 11), True)
CASES["int_4096"] = (lambda: np.floor(uniform_frame(4096, 3) * 10).astype(np.int64), True)
CASES["dup_4096"] = (lambda: np.repeat(uniform_frame(1024, 4), 4, axis=0), True)
CASES["tight_2048"] = (lambda: uniform_frame(2048, 9, -1.0, 1.0) * np.array([1.0, 1.0, 0.01]), True)
# frames against the sequential-sum emulation and the lstsq(rcond=None) plane: far from the origin,
# tiny magnitudes and collinear ground make the design [x y 1] rank-deficient for gelsd (round 3)
# (not "int_big": its 2^32 m extent makes the reference's np.arange of grid edges take 34 GB)
for _k in STRESS_KINDS:
    if _k == "int_big":
        continue
    CASES[f"stress_{_k}"] = (lambda k=_k: stress_frame(k), True)

# frames on which the reference raises (type recorded)
ERROR_CASES = {
    "empty": lambda: np.zeros((0, 3)),
    "one": lambda: uniform_frame(1, 0),
    "const_col": lambda: np.column_stack([uniform_frame(100, 1)[:, :2], np.full(100, 2.5)]),
    "all_equal": lambda: np.ones((50, 3)),
    "nan": lambda: np.where(np.arange(300)[:, None] == 7, np.nan, uniform_frame(300, 2)),
}


def run_case(points):
    pd = preprocess_lidar_data(points)
    people = extract_people_positions(pd)
    try:
        res = CrowdDensityModel().analyze(pd)
    except MemoryError:  # a frame 1e12 m wide: np.arange of the density grid's edges cannot allocate
        res = None
    return pd, people, res


def main():
    meta = {"generator": "tests/golden/gen_tier_r.py", "numpy": np.__version__,
            "cases": {}, "errors": {}, "downsample": {}}
    import sklearn
    meta["sklearn"] = sklearn.__version__
    arrays = {}
    for name, (make, keep) in CASES.items():
        pts = make()
        pd, people, res = run_case(pts)
        d = pd["dimensions"]
        ent = {
            "input": sha(pts),
            "points": sha(pd["points"]), "colors": sha(pd["colors"]),
            "normals": sha(pd["normals"]), "clusters": sha(pd["clusters"]),
            "ground_plane": [fhex(v) for v in pd["ground_plane"]],
            "ground_plane_dtype": str(pd["ground_plane"].dtype),
            "dims": {k: [fhex(v) for v in d[k]] for k in ("x_range", "y_range", "z_range")},
            "dims_scalar": {k: fhex(d[k]) for k in ("width", "length", "height")},
            "dims_dtype": str(np.asarray(d["width"]).dtype),
            "n_clusters": int(pd["clusters"].max() + 1),
            "people": sha(people),
        }
        if res is None:
            ent["analyze_error"] = "MemoryError"
        else:
            ent.update({
                "total_people": int(res["total_people"]),
                "avg_density": fhex(res["avg_density"]), "avg_density_type": type(res["avg_density"]).__name__,
                "max_density": fhex(res["max_density"]), "max_density_type": type(res["max_density"]).__name__,
                "density_map": sha(res["density_map"]),
                "grid_x": sha(res["grid_coordinates"][0]), "grid_y": sha(res["grid_coordinates"][1]),
                "density_values": sha(res["density_values"]),
                "hotspots": [[fhex(h["x"]), fhex(h["y"]), fhex(h["density"])] for h in res["hotspots"]],
            })
            arrays[f"{name}/density_map"] = res["density_map"]
        meta["cases"][name] = ent
        arrays[f"{name}/ground_plane"] = pd["ground_plane"]
        arrays[f"{name}/people"] = people
        if keep:
            arrays[f"{name}/clusters"] = pd["clusters"].astype(np.int32)
        print(name, pts.shape, "clusters", ent["n_clusters"], "people", ent.get("total_people"),
              ent.get("analyze_error", ""), flush=True)
    for name, make in ERROR_CASES.items():
        try:
            run_case(make())
            meta["errors"][name] = None
        except Exception as e:  # record the reference's exception type
            meta["errors"][name] = type(e).__name__
        print(name, "->", meta["errors"][name])
    # downsample_point_cloud (dead code in the reference, A13): global legacy RNG
    base = np.arange(3000, dtype=np.float64).reshape(1000, 3)
    for seed in (0, 1, 2):
        for factor in (0.1, 0.5, 0.999, 1.0):
            np.random.seed(seed)
            out = downsample_point_cloud(base, factor)
            idx = (out[:, 0] // 3).astype(np.int64)
            key = f"s{seed}_f{factor}"
            arrays[f"downsample/{key}"] = idx
            meta["downsample"][key] = sha(out)
    np.savez_compressed(os.path.join(HERE, "tier_r.npz"), **arrays)
    with open(os.path.join(HERE, "tier_r.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
