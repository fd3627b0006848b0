"""Drop-in for the reference's ``utils/data_processing.py`` on MI355X.

Same function names, positional arguments, defaults, return types and exceptions as
the reference (FortuneMU2025/LIDAR_AI_Recommendation_Software ``utils/data_processing.py``);
the arithmetic runs in the gfx950 kernels of ``liblidar_amd.so`` and is bit-identical
to the reference's NumPy / scikit-learn CPU path (see DESIGN.md §2 and
``tests/test_gpu_tier_r.py``).  Inputs and outputs are NumPy, as the reference's
callers expect (``app.py:81``, ``visualization.py``); device copies of the last
results are cached so that ``extract_people_positions`` / ``CrowdDensityModel.analyze``
on a ``preprocess_lidar_data`` result do not re-upload the frame.

Extensions beyond the reference (north_star operators):
``voxel_downsample`` and ``farthest_point_sample``.
"""
import os
import re
import weakref

import numpy as np

from . import _native as nat

# ----------------------------------------------------------------- device cache
# Arrays this module returned keep their device copy, so that extract_people_positions /
# calculate_grid_density on a preprocess_lidar_data result do not re-upload the frame.  A
# hit needs the same object AND the same bytes: the entry stores an xxh3-128 digest of the
# array's contents, so a caller that edits pd["points"] (or the people array) in place gets
# the edited values uploaded, as the reference would read them.  Hashing a 65 k-point frame
# (1.5 MB) costs ~0.1 ms on the host with xxhash (optional), ~2 ms with the standard library's
# blake2b otherwise.
_cache = {}
try:
    import xxhash as _xxhash
except ImportError:  # xxhash is optional: the standard library's blake2b decides equally
    _xxhash = None


def _digest(arr):
    a = np.ascontiguousarray(arr)
    mv = memoryview(a.reshape(-1)).cast("B")
    if _xxhash is not None:
        return a.shape, a.dtype.str, _xxhash.xxh3_128_intdigest(mv)
    import hashlib
    return a.shape, a.dtype.str, hashlib.blake2b(mv, digest_size=16).digest()


def _remember(arr, tensor):
    key = id(arr)
    _cache[key] = (weakref.ref(arr, lambda _r, k=key: _cache.pop(k, None)), tensor, _digest(arr))


def _on_device(arr, dtype):
    import torch
    hit = _cache.get(id(arr))
    if (hit is not None and hit[0]() is arr and hit[1].dtype == dtype and isinstance(arr, np.ndarray)
            and hit[2] == _digest(arr)):
        return hit[1]
    npd = {torch.float64: np.float64, torch.int64: np.int64, torch.float32: np.float32}[dtype]
    return torch.from_numpy(np.ascontiguousarray(arr, dtype=npd)).cuda()


def _reference_shape_errors(pts):
    """The exceptions the reference raises for a frame that is not (N >= 1, 3), decided from the
    array's shape before any kernel runs (utils/data_processing.py:143-207; the Streamlit apps'
    preprocess_point_cloud, app_simplified.py:80-117, raises the same):
      * not 2-D, or fewer than 3 columns: ``points[:, 2]`` raises IndexError;
      * no rows: ``np.min`` of the empty z column raises ValueError;
      * k > 3 columns: the 3-sigma mask runs over all k columns; an empty inlier set raises
        IndexError from ``np.percentile`` (:164), otherwise unpacking ``np.min(inlier_points,
        axis=0)`` into three names raises ValueError (:207).  That decision is the reference's own
        numpy expression on the host: it selects the exception, it computes no result."""
    if pts.ndim != 2:
        raise IndexError(f"too many indices for array: array is {pts.ndim}-dimensional, but 2 were indexed")
    k = pts.shape[1]
    if k < 3:
        raise IndexError(f"index 2 is out of bounds for axis 1 with size {k}")
    if len(pts) == 0:
        raise ValueError("zero-size array to reduction operation minimum which has no identity")
    if k > 3:
        mean = np.mean(pts, axis=0)
        std = np.std(pts, axis=0)
        if not np.all(np.abs(pts - mean) < 3 * std, axis=1).any():
            raise IndexError("index -1 is out of bounds for axis 0 with size 0")
        raise ValueError("too many values to unpack (expected 3)")


def _handle():
    import torch
    return nat.handle(torch.cuda.current_device())


# ----------------------------------------------------------------------- I/O (L1)
def load_lidar_data(file_path):
    """Load an (n, 3) point array from CSV / XYZ / TXT / PCD (ascii) / PLY (ascii) / NPY.

    Mirrors ``utils/data_processing.py:8-125`` (the "next" input boundary of SURVEY §8f;
    host-side parsing, not accelerated): same formats and column rules, and every
    failure is re-raised as ``Exception("Failed to load point cloud file: ...")``.
    """
    try:
        ext = file_path.lower().split(".")[-1]
        if ext == "csv":
            import pandas as pd
            df = pd.read_csv(file_path)
            cols = [c for c in df.columns if c.lower() in ("x", "y", "z")]
            pts = df[cols[:3]].values if len(cols) >= 3 else df.iloc[:, :3].values
        elif ext in ("xyz", "txt"):
            pts = np.loadtxt(file_path, delimiter=None)[:, :3]
        elif ext == "npy":
            pts = np.load(file_path)[:, :3]
        elif ext == "pcd":
            pts = _read_ascii_body(file_path, _pcd_body_start)
        elif ext == "ply":
            pts = _read_ascii_body(file_path, _ply_body)
        else:
            raise ValueError(f"Unsupported file format: {ext}")
        if len(pts) == 0:
            raise ValueError("The loaded point cloud contains no points")
        return pts
    except Exception as e:
        raise Exception(f"Failed to load point cloud file: {str(e)}")


_PCD_HEADER = re.compile(r"([A-Z_]+)\s+([\w\s\.]+)")


def _pcd_body_start(lines):
    # header lines are "KEY value"; the first line that is neither a comment, blank,
    # nor such a header starts the data
    for i, ln in enumerate(lines):
        s = ln.strip()
        if ln.startswith("#") or not s or _PCD_HEADER.match(s):
            continue
        return i, len(lines)
    return 0, len(lines)


def _ply_body(lines):
    # utils/data_processing.py:87-97: the data lines are range(start, start + (n_points or
    # len(lines))), so an absent or zero "element vertex" count reads to the end of the file
    nvert = None
    for i, ln in enumerate(lines):
        if ln.strip() == "end_header":
            start = i + 1
            return start, start + (nvert or len(lines))
        if "element vertex" in ln:
            nvert = int(ln.split()[-1])
    return 0, (nvert or len(lines))


def _read_ascii_body(path, locate):
    with open(path, "rb") as f:
        raw = f.read()
    pts = _parse_fast(raw, locate)
    if pts is not None:
        return pts
    return _read_ascii_body_py(raw.decode(), locate)


def _read_ascii_body_py(text, locate):
    """The reference's loop (data_processing.py:74-80 / :98-104) on text-mode lines."""
    import io
    lines = io.StringIO(text, newline=None).readlines()
    a, b = locate(lines)
    rows = []
    for ln in lines[a:min(b, len(lines))]:
        vals = ln.strip().split()
        if len(vals) >= 3:
            rows.append([float(v) for v in vals[:3]])
    return np.array(rows)


_SLOW_BYTES = re.compile(rb"[\x80-\xff\x0b\x0c\x1c-\x1f]|\r(?!\n)")


def _parse_fast(raw, locate):
    """The data section parsed by liblidar_amd's C parser (lidar_parse_ascii_xyz), or None
    when the input needs Python's own text rules (non-ASCII / exotic whitespace, bare CR
    line breaks, a header beyond the first 64 KiB, or a token only float() parses)."""
    # the data section is checked by the C scanner; the window reaches one byte past the head
    # so that a CRLF split by the 64 KiB cut is not taken for a bare CR
    m = _SLOW_BYTES.search(raw, 0, 65537)
    if m and m.start() < 65536:
        return None
    head = raw[:65536].decode("ascii")
    lines = head.splitlines(keepends=True)
    if len(raw) > 65536:
        lines = lines[:-1]  # the last head line may be cut
    a, b = locate(lines)
    if a == 0 and (not lines or b >= len(lines)):
        # no data section located inside the head: let the Python path decide
        return None
    max_lines = -1
    if locate is _ply_body:  # the vertex count bounds the data lines; none: to the end
        nvert = None
        for ln in lines[:a]:
            if "element vertex" in ln:
                nvert = int(ln.split()[-1])
        max_lines = -1 if not nvert else max(0, nvert)  # None or 0: to the end (:97)
    pts = _parse_ascii_lines_or_none(raw, a, max_lines)
    if pts is None:
        return None
    return pts if len(pts) else np.array([])


def _parse_ascii_lines_or_none(raw, first, max_lines):
    """(n, 3) float64 rows of lines [first, first + max_lines) of `raw` (max_lines < 0: to the
    end) from liblidar_amd's C parser (lidar_parse_ascii_xyz), or None when a token needs
    Python's float() (the caller's own loop then decides)."""
    import ctypes
    lib = nat.load_library()
    cap = raw.count(b"\n") + 1
    out = np.empty((cap, 3), dtype=np.float64)
    n = ctypes.c_int64(0)
    rc = lib.lidar_parse_ascii_xyz(raw, len(raw), first, max_lines, out.ctypes.data_as(ctypes.c_void_p), cap,
                                   ctypes.byref(n))
    if rc != 0:
        return None
    return np.array(out[:n.value])


# ---------------------------------------------------------------- preprocess (L2)
def preprocess_lidar_data(points):
    """Replaces ``utils/data_processing.py:127-229`` — one frame on the GPU.

    Returns the reference's dict {points, colors, normals, clusters, ground_plane,
    dimensions} with the same dtypes; raises the reference's exceptions (ValueError
    on an empty frame, IndexError when no point survives the 3-sigma filter, and the
    shape errors of ``_reference_shape_errors`` for frames that are not (N, 3)).
    """
    import torch
    pts = np.asarray(points)
    _reference_shape_errors(pts)  # frames that are not (N >= 1, 3): the reference's exceptions
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
    nat.call("lidar_preprocess_f64", _handle(), nat.ptr(x), n, nat.ptr(mask), nat.ptr(colors),
             nat.ptr(normals), nat.ptr(comp), nat.ptr(labels), nat.ptr(scal), nat.stream_ptr())
    S = scal.cpu().numpy()
    if S[15] != 0:
        raise IndexError("index -1 is out of bounds for axis 0 with size 0")
    nin = int(S[0])
    comp_d, lab_d = comp[:nin], labels[:nin]
    inl = comp_d.cpu().numpy()
    if is_int:
        inl = inl.astype(pts.dtype)
    cols = colors[:nin].cpu().numpy()
    nrm = normals[:nin].cpu().numpy()
    if is_int:
        nrm = nrm.astype(pts.dtype)
    clusters = lab_d.cpu().numpy()
    kind = S[40]
    if kind == 1.0 and is_int:
        plane = np.array([0, 0, 1, -int(S[9])])
    elif kind == 1.0:
        plane = np.array([0.0, 0.0, 1.0, S[14]])
    else:
        plane = np.array([S[11], S[12], -1, S[14]], dtype=np.float64)
    mins, maxs = S[[5, 7, 9]], S[[6, 8, 10]]
    if is_int:
        mins, maxs = mins.astype(pts.dtype), maxs.astype(pts.dtype)
    (x_min, y_min, z_min), (x_max, y_max, z_max) = mins, maxs
    dims = {"x_range": (x_min, x_max), "y_range": (y_min, y_max), "z_range": (z_min, z_max),
            "width": x_max - x_min, "length": y_max - y_min, "height": z_max - z_min}
    out = {"points": inl, "colors": cols, "normals": nrm, "clusters": clusters,
           "ground_plane": plane, "dimensions": dims}
    _remember(inl, comp_d)
    _remember(clusters, lab_d)
    return out


def downsample_point_cloud(points, factor=0.1):
    """Replaces ``utils/data_processing.py:231-249``: identity for factor >= 1, else
    ``points[np.random.choice(n, max(1, int(n*factor)), replace=False)]``.

    The draw is the reference's own: ``np.random.choice`` on the GLOBAL legacy NumPy RNG (host
    RNG state: identical indices, identical RNG state afterwards).  A host array (or anything
    that is not a CUDA tensor) is indexed on the host, ``points[idx]``, exactly as the reference
    does (same result, same exceptions, e.g. TypeError for a Python list; uploading a host frame
    to gather rows would only add two PCIe copies).  A CUDA tensor in gives a CUDA tensor out:
    the gather runs on the GPU (``lidar_gather_rows`` moves rows as raw bytes) and only the
    indices cross PCIe (throughput mode)."""
    if factor >= 1.0:
        return points
    num = len(points)
    keep = max(1, int(num * factor))
    idx = np.random.choice(num, keep, replace=False)
    import torch
    if isinstance(points, torch.Tensor) and points.is_cuda:
        src = points.contiguous()
        out = torch.empty((keep,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        return _gather_rows(src, idx, out)
    return points[idx]


def _gather_rows(src, idx, out):
    """out[r] = src[idx[r]] on the GPU (rows of numel / len elements, copied as raw bytes)."""
    import torch
    n = len(src)
    row_bytes = src.element_size() * (src.numel() // max(n, 1))
    d_idx = torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int64)).to(src.device)
    nat.call("lidar_gather_rows", nat.handle(src.device.index), nat.ptr(src), n, row_bytes, nat.ptr(d_idx),
             len(idx), nat.ptr(out), nat.stream_ptr())
    d_idx.record_stream(torch.cuda.current_stream(src.device))
    return out


# ------------------------------------------------------------- people / density (L2)
def extract_people_positions(processed_data):
    """Replaces ``utils/data_processing.py:251-280``: (K, 2) per-cluster centroids
    (x, y) in ascending label order, ``np.array([])`` when there is no cluster."""
    import torch
    pts, lab = processed_data["points"], processed_data["clusters"]
    n = len(pts)
    if n == 0:
        return np.array([])
    x = _on_device(pts, torch.float64)
    lbl = _on_device(lab, torch.int64)
    people = torch.empty((n, 2), dtype=torch.float64, device=x.device)
    k = nat.I64(0)
    import ctypes
    nat.call("lidar_people_f64", _handle(), nat.ptr(x), nat.ptr(lbl), n, nat.ptr(people), ctypes.byref(k),
             nat.stream_ptr())
    k = k.value
    if k == 0:
        return np.array([])
    out = people[:k].cpu().numpy()
    _remember(out, people[:k])
    return out


def _grid(people_positions, x_range, y_range, grid_size):
    import torch
    x_min, x_max = x_range
    y_min, y_max = y_range
    nx, ny = nat.grid_dims(x_min, x_max, y_min, y_max, grid_size)
    p = _on_device(np.asarray(people_positions, dtype=np.float64).reshape(-1, 2), torch.float64)
    dev = p.device
    with nat.grid_alloc():
        gx = torch.empty(nx, dtype=torch.float64, device=dev)
        gy = torch.empty(ny, dtype=torch.float64, device=dev)
        buf = torch.empty(3 * nx * ny + 13, dtype=torch.float64, device=dev)
    nat.call("lidar_density_grid_f64", _handle(), nat.ptr(p), len(p), float(x_min), float(x_max),
             float(y_min), float(y_max), float(grid_size), nx, ny, nat.ptr(gx), nat.ptr(gy), nat.ptr(buf),
             nat.stream_ptr())
    b = buf.cpu().numpy()
    m = nx * ny
    dens = b[:m].reshape(nx, ny)
    stats = b[3 * m:3 * m + 8]
    hot = b[3 * m + 8:3 * m + 13].view(np.int64)[: int(stats[3])]
    return gx.cpu().numpy(), gy.cpu().numpy(), dens, b[m:2 * m], b[2 * m:3 * m], stats, hot


def calculate_grid_density(people_positions, x_range, y_range, grid_size=1.0):
    """Replaces ``utils/data_processing.py:282-328``: (grid_x, grid_y, density (nx, ny))
    in people per square metre; ``(None, None, None)`` when there are no positions."""
    if len(people_positions) == 0:
        return None, None, None
    gx, gy, dens, *_ = _grid(people_positions, x_range, y_range, grid_size)
    return gx, gy, dens


# ------------------------------------------------------------- north_star extensions
def voxel_downsample(points, voxel_size):
    """One point per occupied voxel (mean of its points, voxels in ascending key order)
    plus the voxel id of every input point.  Returns (centroids (V, 3) float32,
    voxel_id (N,) int32, counts (V,) int32).  SURVEY §8a N1.

    The voxels are ``calculate_grid_density``'s grid (``utils/data_processing.py:305-319``)
    extended to z: per axis ``np.arange(lo - 2v, (hi + 2v) + v, v)`` over the frame's extent,
    histogram2d's binning (searchsorted right, the last edge closed).  Summed over z, the
    counts are the reference's 2-D histogram of the points' (x, y) on its own edges.  Raises
    ValueError (as ``np.arange`` does) for a non-finite extent, or when the grid has 2^32 keys
    or more; a library failure (nvox <= -2: an in-launch wait timed out, or an inconsistent bucket
    table) raises LidarError instead, naming it."""
    import torch
    from .pointnet2 import voxel_downsample_batch
    if not 0 < voxel_size < np.inf:
        raise ValueError("voxel size must be finite and > 0")
    x = _on_device(np.asarray(points, dtype=np.float32).reshape(-1, 3), torch.float32)
    n = len(x)
    if n == 0:
        return np.zeros((0, 3), np.float32), np.zeros(0, np.int32), np.zeros(0, np.int32)
    # the chip-wide batched path with one frame (csrc/voxel_batch.hip; same results as the
    # single-workgroup lidar_voxel_downsample_f32)
    cent, vid, cnt, nv = voxel_downsample_batch(x[None].contiguous(), float(voxel_size))
    v = int(nv[0].item())  # (<= -2 raised LidarError inside voxel_downsample_batch)
    if v == -1:
        raise ValueError("voxel_downsample: the extent is not finite or the voxel grid has 2^32 keys or more")
    return cent[0, :v].cpu().numpy(), vid[0].cpu().numpy(), cnt[0, :v].cpu().numpy()


def farthest_point_sample(points, npoint):
    """Indices (npoint,) int32 of the farthest-point subset of an (N, 3) frame (start at
    index 0, ties to the lowest index).  SURVEY §8a N2 (no reference counterpart)."""
    import torch
    from .pointnet2 import farthest_point_sample as fps
    x = _on_device(np.asarray(points, dtype=np.float32).reshape(-1, 3), torch.float32)
    return fps(x[None], int(npoint))[0].cpu().numpy()


def radius_count(points, r=0.5):
    """``KDTree(points).query_radius(points, r=r, count_only=True)`` on the GPU: per point the
    number of points within r, itself included (the reference's density colouring,
    ``utils/visualization.py:41-48`` / ``:165-168``, ``app_simplified.py:156-159``; 2-D
    projections are passed as (n, 2)).  Exact: sklearn's fp64 rdist test
    ((dx*dx + dy*dy) + dz*dz <= r*r), shared with DBSCAN's neighbour count."""
    import torch
    p = np.asarray(points, dtype=np.float64)
    if p.ndim != 2 or p.shape[1] not in (2, 3):
        raise ValueError("radius_count expects (n, 2) or (n, 3) points")
    n = len(p)
    if n == 0:
        return np.zeros(0, dtype=np.intp)
    if p.shape[1] == 2:
        p = np.column_stack([p, np.zeros(n)])
    x = torch.from_numpy(np.ascontiguousarray(p)).cuda()
    out = torch.empty(n, dtype=torch.int64, device=x.device)
    nat.call("lidar_radius_count_f64", _handle(), nat.ptr(x), n, float(r), nat.ptr(out), nat.stream_ptr())
    return out.cpu().numpy().astype(np.intp)


def histogram2d(x, y, bins=10, range=None):
    """``np.histogram2d(x, y, bins=bins, range=range)`` with the counting on the GPU — the
    reference's projection heatmaps (``utils/visualization.py:125-137``,
    ``app_simplified.py:205-209``).  The edges are numpy's own (``np.linspace`` for an int
    bin count, or the given edge arrays); returns (H, xedges, yedges) like numpy."""
    import torch
    x = np.asarray(x, dtype=np.float64).ravel()
    y = np.asarray(y, dtype=np.float64).ravel()
    if len(x) != len(y):
        raise ValueError("x and y must have the same length")
    bxy = bins if isinstance(bins, (list, tuple)) and len(bins) == 2 else (bins, bins)
    rng = range if range is not None else [None, None]
    edges = []
    for v, b, r in zip((x, y), bxy, rng):
        if np.ndim(b) == 1:
            e = np.asarray(b, dtype=np.float64)
        else:
            lo, hi = (r if r is not None else ((v.min(), v.max()) if len(v) else (0.0, 1.0)))
            if lo == hi:  # numpy widens a degenerate range by 0.5 on both sides
                lo, hi = lo - 0.5, hi + 0.5
            e = np.linspace(lo, hi, int(b) + 1)
        edges.append(e)
    xe, ye = edges
    dev = torch.device("cuda", torch.cuda.current_device())
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    dx, dy, dxe, dye = T(x), T(y), T(xe), T(ye)
    H = torch.empty((len(xe) - 1, len(ye) - 1), dtype=torch.float64, device=dev)
    nat.call("lidar_histogram2d_f64", _handle(), nat.ptr(dx), nat.ptr(dy), len(x), nat.ptr(dxe), len(xe) - 1,
             nat.ptr(dye), len(ye) - 1, nat.ptr(H), nat.stream_ptr())
    return H.cpu().numpy(), xe, ye
