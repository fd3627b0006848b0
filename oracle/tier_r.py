"""CPU restatement of the reference density path (Tier R).  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module — as the checker / CPU baseline, never as the thing
measured or shipped.  The product path never imports ``oracle``.

Restates, step by step, ``utils/data_processing.py`` and
``models/crowd_density_model.py`` of the reference, with sklearn's DBSCAN
replaced by the order-independent formulation in ``lidar_oracle.c``
(``orc_dbscan_labels``).  Pinned bit-for-bit against ``tests/golden/tier_r.json``,
which ``tests/golden/gen_tier_r.py`` captured by running the reference itself.

Every scalar uses the numpy / sklearn arithmetic the reference goes through:
axis-0 sums of an (N, 3) C-contiguous array are sequential row sums; the
StandardScaler variance is sklearn's corrected two-pass form
(``sklearn/utils/extmath.py:_incremental_mean_and_var`` with a zero prior).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    """Load (building on first use when gcc is present) ``liblidar_oracle.so``."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liblidar_oracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE, "liblidar_oracle.so"])
        L = ctypes.CDLL(path)
        i64, i32, f32, f64 = ctypes.c_int64, ctypes.c_int32, ctypes.c_float, ctypes.c_double
        P = ctypes.c_void_p
        L.orc_eps_count.argtypes = [P, i64, f64, P]
        L.orc_dbscan_labels.argtypes = [P, i64, f64, i32, P, P]
        L.orc_fps.argtypes = [P, i64, i64, P, P]
        L.orc_ball_query.argtypes = [P, i64, P, i64, f32, i32, P]
        L.orc_eps_count.restype = ctypes.c_int
        L.orc_dbscan_labels.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def dbscan_labels(x, eps, min_samples=5, return_counts=False):
    """DBSCAN(eps, min_samples).fit(x).labels_ — order-independent restatement."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    n = len(x)
    labels = np.empty(n, dtype=np.int64)
    counts = np.empty(n, dtype=np.int32)
    rc = lib().orc_dbscan_labels(_ptr(x), n, float(eps), int(min_samples), _ptr(labels), _ptr(counts))
    if rc:
        raise MemoryError("orc_dbscan_labels failed")
    return (labels, counts) if return_counts else labels


def standard_scale(x):
    """StandardScaler().fit_transform(x) for a dense float64 array without NaN.

    sklearn/preprocessing/_data.py (partial_fit -> _incremental_mean_and_var with
    last_mean = last_var = 0, last_count = 0), then ``_handle_zeros_in_scale``
    with the near-constant mask, then transform ``(X - mean_) / scale_``.
    """
    x = np.asarray(x, dtype=np.float64)
    n = x.shape[0]
    new_sum = np.sum(x, axis=0)
    mean = new_sum / n
    temp = x - new_sum / n
    correction = np.sum(temp, axis=0)
    temp **= 2
    unnorm = np.sum(temp, axis=0)
    unnorm -= correction ** 2 / n
    var = unnorm / n
    eps64 = np.finfo(np.float64).eps
    constant = var <= n * eps64 * var + (n * mean * eps64) ** 2
    scale = np.sqrt(var)
    scale[constant] = 1.0
    out = x.copy()
    out -= mean
    out /= scale
    return out, mean, var, scale


def percentile30(z):
    """np.percentile(z, 30) ('linear'), written out (numpy _quantile / _lerp)."""
    n = z.shape[0]
    if n == 0:
        raise IndexError("index -1 is out of bounds for axis 0 with size 0")
    q = np.true_divide(30, np.float64(100))
    v = (n - 1) * q
    prev = np.floor(v)
    if v >= n - 1:
        lo_i = hi_i = n - 1
    else:
        lo_i, hi_i = int(prev), int(prev) + 1
    s = np.sort(z, kind="stable")
    a, b = s[lo_i], s[hi_i]
    t = v - prev
    diff = b - a
    r = a + diff * t
    if t >= 0.5:
        r = b - diff * (1 - t)
    return r


def preprocess_lidar_data(points, dbscan="c"):
    """Restates utils/data_processing.py:127-229 (``preprocess_lidar_data``).

    dbscan "c": the order-independent C DBSCAN (lidar_oracle.c) and the written-out scaler;
    "sklearn": scikit-learn's StandardScaler().fit_transform and DBSCAN(eps, min_samples=5).fit —
    the reference's own calls (:190-197), used as bench.py's CPU baseline of the density path."""
    points = np.asarray(points)
    # :143-147 height colours over ALL points
    z = points[:, 2]
    nh = (z - np.min(z)) / (np.max(z) - np.min(z) + 1e-10)
    colors = np.zeros((len(points), 3))
    colors[:, 0] = nh
    colors[:, 1] = 0.5 * (1 - nh)
    colors[:, 2] = 0.5
    # :151-157 3-sigma filter (strict <, all three axes)
    mean = np.mean(points, axis=0)
    std = np.std(points, axis=0)
    mask = np.all(np.abs(points - mean) < 3 * std, axis=1)
    inl = points[mask]
    inl_colors = colors[mask]
    # :160-161
    normals = np.zeros_like(inl)
    normals[:, 2] = 1.0
    # :164-166 30th percentile ground split
    zt = percentile30(inl[:, 2].astype(np.float64) if inl.dtype.kind != "f" else inl[:, 2])
    ground = inl[:, 2] <= zt
    nonground = ~ground
    # :169-183 ground plane
    if np.sum(ground) > 10:
        gp = inl[ground]
        A = np.column_stack((gp[:, 0], gp[:, 1], np.ones(len(gp))))
        pp, _, _, _ = np.linalg.lstsq(A, gp[:, 2], rcond=None)
        plane = np.array([pp[0], pp[1], -1, pp[2]])
    else:
        plane = np.array([0, 0, 1, -np.min(inl[:, 2])])
    # :186-200 DBSCAN on the scaled non-ground points
    ng = inl[nonground]
    if len(ng) > 10:
        if dbscan == "sklearn":
            from sklearn.cluster import DBSCAN
            from sklearn.preprocessing import StandardScaler
            scaled = StandardScaler().fit_transform(ng)
        else:
            scaled = standard_scale(ng)[0]
        avg = np.mean(np.std(scaled, axis=0)) * 0.5
        eps = max(0.2, min(0.5, avg))
        lab = DBSCAN(eps=eps, min_samples=5).fit(scaled).labels_ if dbscan == "sklearn" else dbscan_labels(scaled, eps, 5)
    else:
        lab = np.zeros(len(ng), dtype=int)
    # :203-204
    full = np.ones(len(inl), dtype=int) * -1
    full[nonground] = lab
    # :207-217
    x_min, y_min, z_min = np.min(inl, axis=0)
    x_max, y_max, z_max = np.max(inl, axis=0)
    dims = {"x_range": (x_min, x_max), "y_range": (y_min, y_max), "z_range": (z_min, z_max),
            "width": x_max - x_min, "length": y_max - y_min, "height": z_max - z_min}
    return {"points": inl, "colors": inl_colors, "normals": normals, "clusters": full,
            "ground_plane": plane, "dimensions": dims}


def extract_people_positions(pd):
    """Restates utils/data_processing.py:251-280 (sequential per-cluster mean)."""
    pts, lab = pd["points"], pd["clusters"]
    ids = np.unique(lab)
    ids = ids[ids >= 0]
    out = [np.mean(pts[lab == c], axis=0)[:2] for c in ids]
    return np.array(out)


def calculate_grid_density(pos, x_range, y_range, grid_size=1.0):
    """Restates utils/data_processing.py:282-328 (np.arange edges + histogram2d)."""
    if len(pos) == 0:
        return None, None, None
    x_min, x_max = x_range
    y_min, y_max = y_range
    m = grid_size * 2
    x_min -= m
    x_max += m
    y_min -= m
    y_max += m
    xe = np.arange(x_min, x_max + grid_size, grid_size)
    ye = np.arange(y_min, y_max + grid_size, grid_size)
    h, xe, ye = np.histogram2d(pos[:, 0], pos[:, 1], bins=[xe, ye])
    return (xe[:-1] + xe[1:]) / 2, (ye[:-1] + ye[1:]) / 2, h / (grid_size * grid_size)


def analyze(pd, grid_size=1.0):
    """Restates models/crowd_density_model.py:23-98 (``CrowdDensityModel.analyze``)."""
    people = extract_people_positions(pd)
    if len(people) == 0:
        return {"total_people": 0, "avg_density": 0.0, "max_density": 0.0,
                "density_map": np.zeros((1, 1)), "grid_coordinates": (np.array([0]), np.array([0])),
                "density_values": np.array([0]), "hotspots": []}
    gx, gy, dg = calculate_grid_density(people, pd["dimensions"]["x_range"],
                                        pd["dimensions"]["y_range"], grid_size)
    flat = dg.flatten()
    fx = np.repeat(gx, len(gy))
    fy = np.tile(gy, len(gx))
    mx = np.max(flat)
    avg = np.mean(flat[flat > 0]) if np.any(flat > 0) else 0
    thr = max(0.5, avg * 1.5)
    hs = [{"x": fx[i], "y": fy[i], "density": flat[i]} for i in np.where(flat >= thr)[0]]
    hs = sorted(hs, key=lambda h: h["density"], reverse=True)[:5]
    return {"total_people": len(people), "avg_density": avg, "max_density": mx, "density_map": dg,
            "grid_coordinates": (fx, fy), "density_values": flat, "hotspots": hs}


# ------------------------------------------------- Streamlit apps' variant
def variant_preprocess_point_cloud(points, eps=0.3):
    """Restates app_simplified.py:76-137 (== app_with_db.py:80-141): preprocess_lidar_data's
    colours / 3-sigma filter / 30th-percentile split, then DBSCAN(eps=0.3, min_samples=5) on
    the UNSCALED non-ground points; returns {points, colors, clusters, dimensions}."""
    points = np.asarray(points)
    z = points[:, 2]
    nh = (z - np.min(z)) / (np.max(z) - np.min(z) + 1e-10)
    colors = np.zeros((len(points), 3))
    colors[:, 0] = nh
    colors[:, 1] = 0.5 * (1 - nh)
    colors[:, 2] = 0.5
    mean = np.mean(points, axis=0)
    std = np.std(points, axis=0)
    mask = np.all(np.abs(points - mean) < 3 * std, axis=1)
    inl = points[mask]
    zt = percentile30(inl[:, 2].astype(np.float64) if inl.dtype.kind != "f" else inl[:, 2])
    nonground = ~(inl[:, 2] <= zt)
    ng = inl[nonground]
    lab = dbscan_labels(ng, eps, 5) if len(ng) > 10 else np.zeros(len(ng), dtype=int)
    full = np.ones(len(inl), dtype=int) * -1
    full[nonground] = lab
    x_min, y_min, z_min = np.min(inl, axis=0)
    x_max, y_max, z_max = np.max(inl, axis=0)
    dims = {"x_range": (x_min, x_max), "y_range": (y_min, y_max), "z_range": (z_min, z_max),
            "width": x_max - x_min, "length": y_max - y_min, "height": z_max - z_min}
    return {"points": inl, "colors": colors[mask], "clusters": full, "dimensions": dims}


def variant_analyze_crowd_density(pd):
    """Restates app_simplified.py:234-316: KDTree(people).query_radius([centre], r=2.0)
    counts are sklearn's rdist test ((cx-px)^2 + (cy-py)^2 <= 4.0, no FMA), here brute force."""
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
    cx = (xg[:-1] + xg[1:]) / 2
    cy = (yg[:-1] + yg[1:]) / 2
    dx = cx[None, :, None] - pos[None, None, :, 0]
    dy = cy[:, None, None] - pos[None, None, :, 1]
    grid = np.sum(dx * dx + dy * dy <= 4.0, axis=2) / 4.0
    top = np.max(grid)
    thr = max(0.5, avg * 1.5)
    jj, ii = np.nonzero(grid >= thr)
    order = np.argsort(-grid[jj, ii], kind="stable")[:5]
    hs = [{"x": cx[ii[o]], "y": cy[jj[o]], "density": grid[jj[o], ii[o]]} for o in order]
    return {"total_people": k, "avg_density": avg, "max_density": top, "density_grid": grid, "hotspots": hs}
