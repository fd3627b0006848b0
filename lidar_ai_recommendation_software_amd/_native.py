"""ctypes binding of liblidar_amd.so (the C-ABI declared in include/lidar_amd.h).

The shared library is built in-tree (``csrc/Makefile`` -> ``liblidar_amd.so`` next to
this file) by ``__graft_entry__.build()``.  There is NO fallback: if the library is
missing or cannot create a handle on the current GPU, every operator raises
``NativeUnavailable`` — the HIP path is the only compute path.

Handles are per (thread, device): the library's scratch workspace is shared by the
calls on one handle, so two threads never share one.
"""
import ctypes
import os
import sys
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# LIDAR_AMD_LIB: load another build of the library (kernel A/B experiments, tools/)
LIB_PATH = os.environ.get("LIDAR_AMD_LIB") or os.path.join(_HERE, "liblidar_amd.so")

LIDAR_ERRORS = {-1: "invalid argument", -2: "HIP runtime error", -3: "out of memory",
                -4: "unsupported device", -5: "needs the Python parser"}


class NativeUnavailable(RuntimeError):
    """liblidar_amd.so is missing, failed to load, or found no gfx950 device."""


class LidarError(RuntimeError):
    """A liblidar_amd call returned a negative status."""


_lib = None
_lib_lock = threading.Lock()
_tls = threading.local()

P = ctypes.c_void_p
I64, I32, F32, F64 = ctypes.c_int64, ctypes.c_int32, ctypes.c_float, ctypes.c_double

# name -> argtypes (restype int unless listed in _RESTYPES)
SIGNATURES = {
    "lidar_create": [ctypes.c_int, ctypes.POINTER(P)],
    "lidar_destroy": [P],
    "lidar_reserve": [P, ctypes.c_uint64],
    "lidar_trim": [P, P],
    "lidar_last_error": [],
    "lidar_version": [],
    "lidar_profile": [P, I32],
    "lidar_profile_read": [P, P, I64, P, I64, P],
    "lidar_gather_rows": [P, P, I64, I64, P, I64, P, P],
    "lidar_venue_counts_f64": [P, P, I64, F64, F64, F64, I64, I64, P, P],
    "lidar_fps_f32": [P, P, I64, I64, I64, P, P, P, P, P],
    "lidar_fps_ex_f32": [P, P, I64, I64, I64, P, P, P, P, I32, P],
    "lidar_ball_query_f32": [P, P, P, I64, I64, I64, F32, I32, P, P],
    "lidar_ball_query_mode_f32": [P, P, P, I64, I64, I64, F32, I32, I32, P, P],
    "lidar_ball_query_grid_bytes": [I64, I64],
    "lidar_ball_query_bin_f32": [P, P, I64, I64, F32, I32, P, P],
    "lidar_ball_query_binned_f32": [P, P, P, P, I64, I64, I64, F32, I32, P, P],
    "lidar_dense_relu_f32": [P, P, I64, I32, P, P, I32, I32, P, P],
    "lidar_dense_f32": [P, P, I64, I32, P, P, I32, I32, I32, P, P],
    "lidar_dense_x3_packed_size": [I32, I32],
    "lidar_dense_x3_pack_f32": [P, P, I32, I32, P, P],
    "lidar_dense_x1_pack_f32": [P, P, I32, I32, P, P],
    "lidar_dense_x3f_f32": [P, P, I32, I64, I32, P, P, I32, I32, I32, I32, P, I64, I64, P],
    "lidar_dense_h3p_f32": [P, P, I32, I64, I32, P, P, P, I32, I32, I32, I32, P, P, I64, F32, F32, P],
    "lidar_mlp_packed_size_x1": [I32, I32, I32],
    "lidar_fps_workspace_bytes": [I64, I64],
    "lidar_mlp_pack_x1_f32": [I32, I32, I32, P, P, P, P, P, P, P],
    "lidar_sa_group_mlp_bq_f32": [P, I32, P, P, P, I64, I64, I64, F32, I32, I32, I32, I32, P, P, I64, I64, P, P],
    "lidar_sa_group_mlp_x1_f32": [P, I32, P, I64, P, P, P, P, I64, I64, I64, I32, I32, I32, I32, P, P, I64, I64, P],
    "lidar_mlp_packed_size16": [I32, I32, I32, I32],
    "lidar_mlp_pack16_f32": [I32, I32, I32, I32, P, P, P, P, P, P, P],
    "lidar_sa_group_mlp16_f32": [P, I32, P, I64, P, P, I64, I64, I64, I32, I32, I32, I32, P, P, I64, I64, P],
    "lidar_mlp_packed_size_x3": [I32, I32, I32, I32],
    "lidar_mlp_pack_x3_f32": [I32, I32, I32, I32, P, P, P, P, P, P, P],
    "lidar_sa_group_mlp_x3_f32": [P, I32, P, I64, P, P, I64, I64, I64, I32, I32, I32, I32, P, P, I64, I64, P],
    "lidar_concat_xyz_pad_f32": [P, P, I64, P, I64, I64, P],
    "lidar_sa_group_rows_f32": [P, P, I64, I32, P, P, P, I64, I64, I64, I32, P, I64, I64, P],
    "lidar_group_max_f32": [P, P, I64, I64, I32, I32, P, I64, I64, P],
    "lidar_voxel_downsample_f32": [P, P, I64, F64, P, P, P, P, P],
    "lidar_voxel_batch_workspace_bytes": [I64, I64],
    "lidar_voxel_downsample_batch_f32": [P, P, I64, I64, F64, P, P, P, P, P],
    "lidar_dbscan_f64": [P, P, I64, F64, I32, P, P, P],
    "lidar_radius_count_f64": [P, P, I64, F64, P, P],
    "lidar_histogram2d_f64": [P, P, P, I64, P, I64, P, I64, P, P],
    "lidar_parse_ascii_xyz": [P, I64, I64, I64, P, I64, P],
    "lidar_preprocess_f64": [P, P, I64, P, P, P, P, P, P, P],
    "lidar_preprocess_batch_f64": [P, P, P, I32, I64, P, P, P, P, P, P, P],
    "lidar_preprocess_eps_batch_f64": [P, P, P, I32, I64, F64, P, P, P, P, P, P, P],
    "lidar_cell_radius_density_f64": [P, P, I64, P, I64, P, I64, F64, F64, P, P],
    "lidar_flow_field_f64": [P, I64, P, I64, F64, F64, I32, P, I32, F64, F64, P, P, P],
    "lidar_flow_bottlenecks_f64": [P, P, P, I64, F64, F64, F64, I32, I32, P, P, P, P, I64, P],
    "lidar_kdtree_order_f64": [P, I64, I32, I32, P],
    "lidar_people_batch_f64": [P, P, P, P, I32, I64, P, P, P, P],
    "lidar_density_batch_f64": [P, P, P, P, I32, P, P, I64, P],
    "lidar_people_f64": [P, P, P, I64, P, P, P],
    "lidar_grid_dims": [F64, F64, F64, F64, F64, P, P],
    "lidar_density_grid_f64": [P, P, I64, F64, F64, F64, F64, F64, I64, I64, P, P, P, P],
}
_RESTYPES = {"lidar_last_error": ctypes.c_char_p,
             "lidar_mlp_packed_size16": I64, "lidar_mlp_packed_size_x3": I64,
             "lidar_ball_query_grid_bytes": ctypes.c_uint64,
             "lidar_dense_x3_packed_size": I64, "lidar_mlp_packed_size_x1": I64,
             "lidar_fps_workspace_bytes": ctypes.c_uint64, "lidar_voxel_batch_workspace_bytes": ctypes.c_uint64}


def load_library(path=LIB_PATH):
    """Load and type the library (no GPU needed).  Raises NativeUnavailable."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NativeUnavailable(
                f"{path} not built — run __graft_entry__.build() (make -C csrc); "
                "there is no CPU fallback")
        try:
            lib = ctypes.CDLL(path)
        except OSError as e:  # pragma: no cover - depends on the box
            raise NativeUnavailable(f"cannot load {path}: {e}") from e
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue  # reported by missing_symbols(); calling it raises AttributeError
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = lib
        return lib


def missing_symbols():
    lib = load_library()
    return [n for n in SIGNATURES if getattr(lib, n, None) is None]


def check(rc, what):
    if rc != 0:
        msg = load_library().lidar_last_error().decode(errors="replace")
        raise LidarError(f"{what} failed ({rc}: {LIDAR_ERRORS.get(rc, '?')}): {msg}")


def grid_dims(x_min, x_max, y_min, y_max, grid_size):
    """(nx, ny) of calculate_grid_density's grid (lidar_grid_dims: np.arange's length of the
    margin-padded edges, utils/data_processing.py:305-313), with numpy's errors for grids it could
    never build: a non-finite extent or a length past what an array may hold raises ValueError
    ("Maximum allowed size exceeded"), more than 2^40 cells MemoryError (a frame 1e12 m wide).
    The grid's own allocation raises MemoryError too when the device has no room for it
    (grid_alloc)."""
    nx, ny = I64(0), I64(0)
    rc = load_library().lidar_grid_dims(float(x_min), float(x_max), float(y_min), float(y_max),
                                        float(grid_size), ctypes.byref(nx), ctypes.byref(ny))
    if rc == -3:
        raise MemoryError(f"Unable to allocate a density grid for x in [{x_min}, {x_max}], "
                          f"y in [{y_min}, {y_max}] at grid size {grid_size}")
    if rc == -1:
        raise ValueError("Maximum allowed size exceeded")
    check(rc, "lidar_grid_dims")
    return nx.value, ny.value


class grid_alloc:
    """Context for the device allocations of a density grid: torch's out-of-memory error becomes
    the MemoryError numpy raises for an array it cannot allocate."""

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        import torch
        if et is not None and issubclass(et, torch.cuda.OutOfMemoryError):
            raise MemoryError(f"Unable to allocate the density grid on the device: {ev}") from ev
        return False


class _ThreadHandles(dict):
    """This thread's handles, {(device, slot): handle}.  When the thread ends, its thread-local
    storage is released and the handles with it (lidar_destroy frees their workspaces); the main
    thread's live until exit, when the process's teardown reclaims the device memory."""

    # bound at definition: at interpreter exit module globals and imports may already be gone
    def __del__(self, _finalizing=sys.is_finalizing, _current=threading.current_thread,
                _main=threading.main_thread):
        try:
            if _finalizing() or _current() is _main():
                return
        except Exception:  # interpreter teardown
            return
        lib = _lib
        if lib is None:
            return
        for h in self.values():
            lib.lidar_destroy(h)
        self.clear()


def handle(device=None, slot=0):
    """The calling thread's handle for `device` (default: torch's current device).

    `slot` selects an independent handle (own scratch workspace) for work that runs
    concurrently on another stream — calls on one handle must not overlap."""
    import torch
    if not torch.cuda.is_available():
        raise NativeUnavailable("no GPU visible: the liblidar_amd HIP path needs a gfx950 device")
    if device is None:
        device = torch.cuda.current_device()
    hs = getattr(_tls, "handles", None)
    if hs is None:
        hs = _tls.handles = _ThreadHandles()
    key = (device, slot)
    h = hs.get(key)
    if h is None:
        lib = load_library()
        hp = P()
        check(lib.lidar_create(int(device), ctypes.byref(hp)), "lidar_create")
        h = hs[key] = hp
    return h


def trim(device=None):
    """Free the workspaces this thread's handles for `device` retired when they grew
    (lidar_trim).  Call only where the work queued with those handles has completed (after
    synchronising the streams it ran on).  Returns the bytes freed."""
    import torch
    if device is None:
        device = torch.cuda.current_device()
    freed = 0
    for (d, _), h in list((getattr(_tls, "handles", None) or {}).items()):
        if d == device:
            b = ctypes.c_uint64(0)
            call("lidar_trim", h, ctypes.byref(b))
            freed += b.value
    return freed


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return P(s.cuda_stream)


def ptr(t):
    """Device pointer of a contiguous torch tensor (None -> NULL)."""
    if t is None:
        return None
    return P(t.data_ptr())


def call(name, *args):
    lib = load_library()
    check(getattr(lib, name)(*args), name)


def profile(h, enable):
    """Start (True) or stop (False) per-phase HIP-event timing of handle h (lidar_profile)."""
    call("lidar_profile", h, 1 if enable else 0)


def profile_read(h, cap=4096):
    """[(phase name, ms)] recorded on h since the last read, in launch order (waits for them)."""
    names = ctypes.create_string_buffer(64 * cap)
    ms = (ctypes.c_float * cap)()
    n = I64(0)
    call("lidar_profile_read", h, names, len(names), ms, cap, ctypes.byref(n))
    return list(zip(names.value.decode().split("\n")[: n.value], ms[: n.value]))
