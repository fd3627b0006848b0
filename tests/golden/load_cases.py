"""Deterministic input files for the ``load_lidar_data`` fixtures (tests/golden/load.json).

``build(name)`` returns (file name, bytes); ``gen_load.py`` writes them, runs the REFERENCE's
``utils/data_processing.load_lidar_data`` (:8-125) on them and records the results;
``tests/test_loader_cpu.py`` rebuilds the same bytes and checks the drop-in against the record.

The PLY cases pin the header rules of :84-104: the data lines are
``range(data_start, data_start + (n_points or len(lines)))``, so ``element vertex 0`` or no
vertex line at all reads to the end of the file, a negative count reads nothing, the last
``element vertex`` line wins, and a missing ``end_header`` starts the data at line 0.  Large
bodies (past the drop-in's 64 KiB header window) exercise its C parser; the others its
Python loop.  PCD / CSV / XYZ / TXT / NPY cases pin the remaining branches.
"""
import io

import numpy as np


def _rows(n, seed, cols=3):
    rng = np.random.default_rng(seed)
    return [" ".join(repr(float(v)) for v in r) for r in rng.uniform(-20.0, 20.0, size=(n, cols))]


def _ply(body, count="keep", tail=(), nl="\n", extra_vertex=None, end=True):
    head = ["ply", "format ascii 1.0", "comment synthetic"]
    if count == "keep":
        head.append(f"element vertex {len(body)}")
    elif count is not None:
        head.append(f"element vertex {count}")
    if extra_vertex is not None:
        head.append(f"element vertex {extra_vertex}")
    head += ["property float x", "property float y", "property float z"]
    if end:
        head.append("end_header")
    return (nl.join(head + list(body) + list(tail)) + nl).encode()


def _pcd(body, nl="\n"):
    head = ["# .PCD v0.7", "VERSION 0.7", "FIELDS x y z", "SIZE 4 4 4", "TYPE F F F", "COUNT 1 1 1",
            f"WIDTH {len(body)}", "HEIGHT 1", f"POINTS {len(body)}", "DATA ascii"]
    return (nl.join(head + list(body)) + nl).encode()


def _npy(a):
    f = io.BytesIO()
    np.save(f, a, allow_pickle=False)
    return f.getvalue()


def _cases():
    c = {}
    small, big = _rows(7, 1), _rows(6000, 2)
    c["ply_vertex_count"] = ("a.ply", _ply(small))
    c["ply_vertex0"] = ("a.ply", _ply(small, count=0))
    c["ply_vertex0_big"] = ("a.ply", _ply(big, count=0))
    c["ply_no_vertex_line"] = ("a.ply", _ply(small, count=None))
    c["ply_no_vertex_line_big"] = ("a.ply", _ply(big, count=None))
    c["ply_vertex_negative"] = ("a.ply", _ply(small, count=-3))
    c["ply_vertex_fewer"] = ("a.ply", _ply(small, count=4))
    c["ply_vertex_fewer_big"] = ("a.ply", _ply(big, count=5000))
    c["ply_vertex_more"] = ("a.ply", _ply(small, count=50))
    c["ply_two_vertex_lines"] = ("a.ply", _ply(small, count=2, extra_vertex=5))
    c["ply_vertex0_crlf"] = ("a.ply", _ply(small, count=0, nl="\r\n"))
    c["ply_vertex0_tail_face"] = ("a.ply", _ply(small, count=0, tail=("3 0 1 2", "3 1 2 3")))
    c["ply_vertex0_short_rows"] = ("a.ply", _ply(small[:3] + ["1 2", ""] + small[3:], count=0))
    c["ply_no_end_header"] = ("a.ply", _ply(small, end=False))
    c["ply_empty_vertex0"] = ("a.ply", _ply([], count=0))
    c["ply_vertex0_underscore"] = ("a.ply", _ply(small[:2] + ["1_0.5 2 3"] + small[2:], count=0))
    c["pcd_basic"] = ("a.pcd", _pcd(small))
    c["pcd_big"] = ("a.pcd", _pcd(big))
    c["pcd_nan_paren"] = ("a.pcd", _pcd(small[:2] + ["nan(1) 2 3"] + small[2:]))
    c["pcd_nan_paren_big"] = ("a.pcd", _pcd(big[:3000] + ["1 nan() 3"] + big[3000:]))
    c["pcd_empty"] = ("a.pcd", _pcd([]))
    c["csv_xyz"] = ("a.csv", ("i,X,y,Z\n" + "".join(f"{k},{r.replace(' ', ',')}\n"
                                                    for k, r in enumerate(small))).encode())
    c["csv_other"] = ("a.csv", ("a,b,c,d\n" + "".join(f"{r.replace(' ', ',')},9\n" for r in small)).encode())
    c["xyz_space"] = ("a.xyz", ("\n".join(small) + "\n").encode())
    c["txt_four_cols"] = ("a.txt", ("\n".join(r + " 1.0" for r in small) + "\n").encode())
    c["npy_f64"] = ("a.npy", _npy(np.random.default_rng(3).uniform(-5, 5, (9, 4))))
    c["npy_i32"] = ("a.npy", _npy(np.arange(30, dtype=np.int32).reshape(10, 3)))
    c["unsupported"] = ("a.las", b"LASF")
    return c


CASES = _cases()
NAMES = sorted(CASES)


def build(name):
    return CASES[name]
