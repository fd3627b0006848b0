"""Drop-in for the Streamlit apps' own pipeline on MI355X.

``app_simplified.py`` and ``app_with_db.py`` do not call ``utils/data_processing.py``; they
carry a variant of it:

* ``preprocess_point_cloud(points)`` (``app_simplified.py:76-137``, ``app_with_db.py:80-141``):
  the same height colours / 3-sigma filter / 30th-percentile ground split as
  ``preprocess_lidar_data``, then ``DBSCAN(eps=0.3, min_samples=5)`` on the **unscaled**
  non-ground points (no StandardScaler, no eps heuristic) and a dict without normals or
  ground plane.
* ``analyze_crowd_density(processed_data)`` (``app_simplified.py:234-316``,
  ``app_with_db.py:238-320``): per-cluster centroids, then per 1 m grid cell the number of
  people within 2 m of the cell centre (``KDTree.query_radius``) / 4, and the hotspots.

Both run on the same gfx950 kernels as the drop-in path (``lidar_preprocess_eps_batch_f64``:
the preprocess phases with a fixed eps; ``lidar_people_f64``; ``lidar_cell_radius_density_f64``)
and return the reference's dicts, bit for bit (``tests/test_gpu_tier_r.py``).  Host work is
the reference's own scalar glue on tiny arrays (the grid edges ``np.arange``, the hotspot
sort over <= a few thousand cells).
"""
import ctypes

import numpy as np

from . import _native as nat
from .data_processing import _handle, _on_device, _reference_shape_errors, _remember

EPS = 0.3          # app_simplified.py:107
MIN_SAMPLES = 5    # the kernel's DBSCAN min_samples (fixed, as in the reference)
CELL_RADIUS = 2.0  # app_simplified.py:280
CELL_AREA = 4.0    # app_simplified.py:281


def preprocess_point_cloud(points, eps=EPS):
    """Replaces ``app_simplified.py:76-137``: {points, colors, clusters, dimensions}.

    Raises what the reference raises: ValueError on an empty frame, IndexError when no
    point survives the 3-sigma filter (``np.percentile`` of an empty array)."""
    import torch
    pts = np.asarray(points)
    _reference_shape_errors(pts)  # frames that are not (N >= 1, 3): app_simplified.py:80-117 raises the same
    n = len(pts)
    is_int = pts.dtype.kind in "iub"
    x = torch.from_numpy(np.ascontiguousarray(pts, dtype=np.float64)).cuda()
    dev = x.device
    mask = torch.empty(n, dtype=torch.uint8, device=dev)
    colors = torch.empty((n, 3), dtype=torch.float64, device=dev)
    normals = torch.empty((n, 3), dtype=torch.float64, device=dev)
    comp = torch.empty((n, 3), dtype=torch.float64, device=dev)
    labels = torch.empty(n, dtype=torch.int64, device=dev)
    scal = torch.empty(64, dtype=torch.float64, device=dev)
    nat.call("lidar_preprocess_eps_batch_f64", _handle(), nat.ptr(x), None, 1, n, float(eps), nat.ptr(mask),
             nat.ptr(colors), nat.ptr(normals), nat.ptr(comp), nat.ptr(labels), nat.ptr(scal), nat.stream_ptr())
    S = scal.cpu().numpy()
    if S[15] != 0:
        raise IndexError("index -1 is out of bounds for axis 0 with size 0")
    nin = int(S[0])
    comp_d, lab_d = comp[:nin], labels[:nin]
    inl = comp_d.cpu().numpy()
    if is_int:
        inl = inl.astype(pts.dtype)
    cols = colors[:nin].cpu().numpy()
    clusters = lab_d.cpu().numpy()
    mins, maxs = S[[5, 7, 9]], S[[6, 8, 10]]
    if is_int:
        mins, maxs = mins.astype(pts.dtype), maxs.astype(pts.dtype)
    (x_min, y_min, z_min), (x_max, y_max, z_max) = mins, maxs
    dims = {"x_range": (x_min, x_max), "y_range": (y_min, y_max), "z_range": (z_min, z_max),
            "width": x_max - x_min, "length": y_max - y_min, "height": z_max - z_min}
    _remember(inl, comp_d)
    _remember(clusters, lab_d)
    return {"points": inl, "colors": cols, "clusters": clusters, "dimensions": dims}


def _people(points, clusters):
    """(K, 2) centroids in ascending label order (labels dense 0..K-1, as DBSCAN emits)."""
    import torch
    n = len(points)
    if n == 0:
        return np.zeros((0, 2)), None
    x = _on_device(points, torch.float64)
    lbl = _on_device(clusters, torch.int64)
    people = torch.empty((n, 2), dtype=torch.float64, device=x.device)
    k = nat.I64(0)
    nat.call("lidar_people_f64", _handle(), nat.ptr(x), nat.ptr(lbl), n, nat.ptr(people), ctypes.byref(k),
             nat.stream_ptr())
    return people[:k.value], k.value


def analyze_crowd_density(processed_data):
    """Replaces ``app_simplified.py:234-316``: {total_people, avg_density, max_density,
    density_grid, hotspots} with the reference's types (``max_density`` a Python 0 and
    ``density_grid`` zeros((1, 1)) when nobody is found)."""
    import torch
    points = processed_data["points"]
    clusters = np.asarray(processed_data["clusters"])
    people_d, k = _people(points, clusters)
    num_people = int(k or 0)
    area = processed_data["dimensions"]["width"] * processed_data["dimensions"]["length"]
    avg_density = num_people / max(1, area)  # :243-244, the same Python expression
    if num_people == 0:
        return {"total_people": 0, "avg_density": avg_density, "max_density": 0,
                "density_grid": np.zeros((1, 1)), "hotspots": []}
    x_range = processed_data["dimensions"]["x_range"]
    y_range = processed_data["dimensions"]["y_range"]
    grid_size = 1.0
    x_grid = np.arange(x_range[0], x_range[1] + grid_size, grid_size)
    y_grid = np.arange(y_range[0], y_range[1] + grid_size, grid_size)
    nx, ny = len(x_grid) - 1, len(y_grid) - 1
    if nx == 0 or ny == 0:  # the reference's np.max over an empty grid
        raise ValueError("zero-size array to reduction operation maximum which has no identity")
    dev = people_d.device
    xg = torch.from_numpy(np.ascontiguousarray(x_grid, dtype=np.float64)).to(dev)
    yg = torch.from_numpy(np.ascontiguousarray(y_grid, dtype=np.float64)).to(dev)
    grid = torch.empty((ny, nx), dtype=torch.float64, device=dev)
    nat.call("lidar_cell_radius_density_f64", _handle(), nat.ptr(people_d.contiguous()), num_people, nat.ptr(xg),
             nx + 1, nat.ptr(yg), ny + 1, CELL_RADIUS, CELL_AREA, nat.ptr(grid), nat.stream_ptr())
    density_grid = grid.cpu().numpy()
    max_density = np.max(density_grid)
    hotspot_threshold = max(0.5, avg_density * 1.5)
    jj, ii = np.nonzero(density_grid >= hotspot_threshold)  # row-major = the reference's j, i loop order
    vals = density_grid[jj, ii]
    order = np.argsort(-vals, kind="stable")[:5]  # sorted(..., reverse=True) keeps ties in loop order
    hotspots = [{"x": (x_grid[ii[o]] + x_grid[ii[o] + 1]) / 2, "y": (y_grid[jj[o]] + y_grid[jj[o] + 1]) / 2,
                 "density": density_grid[jj[o], ii[o]]} for o in order]
    return {"total_people": num_people, "avg_density": avg_density, "max_density": max_density,
            "density_grid": density_grid, "hotspots": hotspots}
