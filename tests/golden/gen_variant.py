"""Capture golden vectors for the Streamlit apps' variant pipeline.

``app_simplified.py`` / ``app_with_db.py`` import ``streamlit`` at module level and it is not
installed here, so the apps themselves cannot be imported.  Their two pipeline functions use
only numpy and scikit-learn; this script re-expresses them step by step
(``preprocess_point_cloud``: app_simplified.py:76-137, ``analyze_crowd_density``: :234-316)
and runs the SAME third-party calls the apps make — ``sklearn.cluster.DBSCAN(eps=0.3,
min_samples=5).fit`` on the unscaled non-ground points and ``sklearn.neighbors.KDTree``
``query_radius(..., r=2.0)`` per grid cell — so the fixtures carry scikit-learn's own
results, not this repo's.

Writes ``variant.json`` (digests, float.hex scalars, hotspots, exception types) and
``variant.npz`` (labels of the small cases, density grids).
Run:  python tests/golden/gen_variant.py
"""
import hashlib
import json
import os
import sys

import numpy as np
from sklearn.cluster import DBSCAN
from sklearn.neighbors import KDTree

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from lidar_ai_recommendation_software_amd.synthetic import (uniform_frame, crowd_frame,  # noqa: E402
                                                        blob_frame, lattice_frame)


def sha(a):
    a = np.ascontiguousarray(a)
    return {"sha256": hashlib.sha256(a.tobytes()).hexdigest(), "shape": list(a.shape), "dtype": str(a.dtype)}


def fhex(v):
    return float(v).hex()


def variant_preprocess(points):
    """app_simplified.py:76-137 with sklearn's DBSCAN (eps 0.3 on unscaled coordinates)."""
    z = points[:, 2]
    lo, hi = np.min(z), np.max(z)
    h = (z - lo) / (hi - lo + 1e-10)
    colors = np.zeros((len(points), 3))
    colors[:, 0], colors[:, 1], colors[:, 2] = h, 0.5 * (1 - h), 0.5
    mu, sd = np.mean(points, axis=0), np.std(points, axis=0)
    keep = np.all(np.abs(points - mu) < 3 * sd, axis=1)
    inl = points[keep]
    zt = np.percentile(inl[:, 2], 30)
    above = ~(inl[:, 2] <= zt)
    ng = inl[above]
    if len(ng) > 10:
        lab = DBSCAN(eps=0.3, min_samples=5).fit(ng).labels_
    else:
        lab = np.zeros(len(ng), dtype=int)
    full = np.full(len(inl), -1, dtype=int)
    full[above] = lab
    mn, mx = np.min(inl, axis=0), np.max(inl, axis=0)
    dims = {"x_range": (mn[0], mx[0]), "y_range": (mn[1], mx[1]), "z_range": (mn[2], mx[2]),
            "width": mx[0] - mn[0], "length": mx[1] - mn[1], "height": mx[2] - mn[2]}
    return {"points": inl, "colors": colors[keep], "clusters": full, "dimensions": dims}


def variant_density(pd):
    """app_simplified.py:234-316 with sklearn's KDTree radius queries."""
    pts, cl = pd["points"], pd["clusters"]
    ids = np.unique(cl[cl >= 0])
    k = len(ids)
    area = pd["dimensions"]["width"] * pd["dimensions"]["length"]
    avg = k / max(1, area)
    if k == 0:
        return {"total_people": 0, "avg_density": avg, "max_density": 0, "density_grid": np.zeros((1, 1)),
                "hotspots": []}
    pos = np.array([np.mean(pts[cl == c], axis=0)[:2] for c in ids])
    xr, yr = pd["dimensions"]["x_range"], pd["dimensions"]["y_range"]
    xg = np.arange(xr[0], xr[1] + 1.0, 1.0)
    yg = np.arange(yr[0], yr[1] + 1.0, 1.0)
    grid = np.zeros((len(yg) - 1, len(xg) - 1))
    tree = KDTree(pos)
    for i in range(len(xg) - 1):
        for j in range(len(yg) - 1):
            c = np.array([(xg[i] + xg[i + 1]) / 2, (yg[j] + yg[j + 1]) / 2])
            grid[j, i] = len(tree.query_radius([c], r=2.0)[0]) / 4.0
    top = np.max(grid)
    thr = max(0.5, avg * 1.5)
    hs = []
    for j in range(grid.shape[0]):
        for i in range(grid.shape[1]):
            if grid[j, i] >= thr:
                hs.append({"x": (xg[i] + xg[i + 1]) / 2, "y": (yg[j] + yg[j + 1]) / 2, "density": grid[j, i]})
    hs = sorted(hs, key=lambda e: e["density"], reverse=True)[:5]
    return {"total_people": k, "avg_density": avg, "max_density": top, "density_grid": grid, "hotspots": hs}


CASES = {
    "crowd_10000_s42": (lambda: crowd_frame(10000, 42), True),
    "crowd_16384_s7": (lambda: crowd_frame(16384, 7), True),
    "crowd_65536_s3": (lambda: crowd_frame(65536, 3), False),
    "blobs_4293_s0": (lambda: blob_frame(60, 60, 300, 0, 15, 0.6), True),
    "blobs_8980_s1": (lambda: blob_frame(200, 40, 500, 1, 15, 0.3), True),
    "lattice_8163_s4": (lambda: lattice_frame(4, 120, 60, 4, 15, 0.4), True),
    "lattice_15636_s1": (lambda: lattice_frame(4, 250, 100, 1, 15, 0.3), True),
    "lattice_62978_s2": (lambda: lattice_frame(4, 1000, 100, 2, 15, 0.3), False),
    "uniform_4096_s0": (lambda: uniform_frame(4096, 0), True),
    "dense_4096_s1": (lambda: uniform_frame(4096, 1, -2.0, 2.0), True),
    "small_12": (lambda: uniform_frame(12, 5), True),
    "small_20": (lambda: uniform_frame(20, 5, -0.2, 0.2), True),
    "int_4096": (lambda: np.floor(uniform_frame(4096, 3, -3.0, 3.0) * 2).astype(np.int64), True),
    "dup_4096": (lambda: np.repeat(uniform_frame(1024, 4, -3.0, 3.0), 4, axis=0), True),
}
ERROR_CASES = {
    "empty": lambda: np.zeros((0, 3)),
    "one": lambda: uniform_frame(1, 0),
    "const_col": lambda: np.column_stack([uniform_frame(100, 1)[:, :2], np.full(100, 2.5)]),
    "all_equal": lambda: np.ones((50, 3)),
}


def main():
    import sklearn
    meta = {"generator": "tests/golden/gen_variant.py", "numpy": np.__version__, "sklearn": sklearn.__version__,
            "cases": {}, "errors": {}}
    arrays = {}
    for name, (make, keep) in CASES.items():
        pts = make()
        pd = variant_preprocess(pts)
        res = variant_density(pd)
        d = pd["dimensions"]
        meta["cases"][name] = {
            "input": sha(pts), "points": sha(pd["points"]), "colors": sha(pd["colors"]),
            "clusters": sha(pd["clusters"]),
            "dims": {k: [fhex(v) for v in d[k]] for k in ("x_range", "y_range", "z_range")},
            "dims_scalar": {k: fhex(d[k]) for k in ("width", "length", "height")},
            "dims_dtype": str(np.asarray(d["width"]).dtype),
            "total_people": int(res["total_people"]),
            "avg_density": fhex(res["avg_density"]), "avg_density_type": type(res["avg_density"]).__name__,
            "max_density": fhex(res["max_density"]), "max_density_type": type(res["max_density"]).__name__,
            "density_grid": sha(res["density_grid"]),
            "hotspots": [[fhex(h["x"]), fhex(h["y"]), fhex(h["density"])] for h in res["hotspots"]],
        }
        arrays[f"{name}/density_grid"] = res["density_grid"]
        if keep:
            arrays[f"{name}/clusters"] = pd["clusters"].astype(np.int32)
        print(name, pts.shape, "people", res["total_people"], "hotspots", len(res["hotspots"]), flush=True)
    for name, make in ERROR_CASES.items():
        try:
            variant_density(variant_preprocess(make()))
            meta["errors"][name] = None
        except Exception as e:
            meta["errors"][name] = type(e).__name__
        print(name, "->", meta["errors"][name])
    np.savez_compressed(os.path.join(HERE, "variant.npz"), **arrays)
    with open(os.path.join(HERE, "variant.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
