"""Deterministic input files for the desktop-loader fixtures (tests/golden/loader.json).

``build(name)`` returns (file name, bytes); ``gen_loader.py`` writes them, runs the REFERENCE's
``windows_implementation/core/data_loader.py`` on them and records the results;
``tests/test_loader_cpu.py`` rebuilds the same bytes and checks ``desktop_loader`` against the
record. The cases cover ASCII PCD / PLY bodies (C-parser path and Python fallbacks), binary
PCD / PLY (rejected), LAS (record cap, short final record, bad signature, truncated header,
records shorter than X, Y, Z), LAZ, XYZ delimiters and CSV column rules.
"""
import struct

import numpy as np


def _rows(n, seed, cols=3, fmt="repr"):
    rng = np.random.default_rng(seed)
    a = rng.uniform(-50.0, 50.0, size=(n, cols))
    out = []
    for r in a:
        if fmt == "repr":
            out.append(" ".join(repr(float(v)) for v in r))
        else:
            out.append(" ".join(f"{v:.6f}" for v in r))
    return out


def _pcd(body_lines, data="ascii", fields="x y z", nl="\n", extra_header=()):
    head = ["# .PCD v0.7 - Point Cloud Data file format", "VERSION 0.7", f"FIELDS {fields}",
            "SIZE 4 4 4", "TYPE F F F", "COUNT 1 1 1", f"WIDTH {len(body_lines)}", "HEIGHT 1",
            "VIEWPOINT 0 0 0 1 0 0 0", f"POINTS {len(body_lines)}", *extra_header, f"DATA {data}"]
    return (nl.join(head + list(body_lines)) + nl).encode("utf-8")


def _ply(body_lines, n_vertex=None, fmt="ascii 1.0", props=("float x", "float y", "float z"), tail=()):
    n_vertex = len(body_lines) if n_vertex is None else n_vertex
    head = ["ply", f"format {fmt}", "comment synthetic", f"element vertex {n_vertex}",
            *[f"property {p}" for p in props], "element face 0", "property list uchar int vertex_indices",
            "end_header"]
    return ("\n".join(head + list(body_lines) + list(tail)) + "\n").encode("utf-8")


def _las(n_records, present, rec_len=20, offset=227, sig=b"LASF", fmt_id=0, extra=b"", seed=5):
    hdr = bytearray(offset)
    hdr[0:4] = sig
    hdr[24:26] = bytes([1, 2])  # version 1.2
    hdr[94:96] = struct.pack("<H", 227)
    hdr[96:100] = struct.pack("<I", offset)
    hdr[104] = fmt_id
    hdr[105:107] = struct.pack("<H", rec_len)
    hdr[107:111] = struct.pack("<I", n_records)
    rng = np.random.default_rng(seed)
    recs = bytearray()
    for _ in range(present):
        xyz = rng.integers(-2 ** 31, 2 ** 31 - 1, size=3, dtype=np.int64)
        rec = struct.pack("<iii", *[int(v) for v in xyz]) + bytes(rng.integers(0, 256, size=max(rec_len - 12, 0),
                                                                             dtype=np.uint8))
        recs += rec[:rec_len] if rec_len < 12 else rec
    return bytes(hdr) + bytes(recs) + extra


def _cases():
    c = {}
    c["pcd_ascii_4col"] = ("a.pcd", _pcd(_rows(300, 1, cols=4), fields="x y z intensity"))
    c["pcd_ascii_65536"] = ("big.pcd", _pcd(_rows(65536, 2)))
    c["pcd_ascii_fixed6"] = ("f.pcd", _pcd(_rows(1000, 3, fmt="f6")))
    bad = _rows(50, 4) + ["nan 1 2", "a b c", "1 2", "", "   ", "1_0 2 3", "0x10 1 2", "inf -inf 3e-320",
                          "4 5 6 extra tokens"] + _rows(20, 5)
    c["pcd_bad_rows"] = ("bad.pcd", _pcd(bad))
    c["pcd_crlf"] = ("crlf.pcd", _pcd(_rows(200, 6), nl="\r\n"))
    # strtod reads "nan(1)" / "nan()", Python's float() does not: the row is the
    # reference loop's to judge, in a small file (Python path) and past the C parser's window
    c["pcd_nan_paren"] = ("np.pcd", _pcd(_rows(20, 18) + ["nan(1) 2 3", "1 nan() 3"] + _rows(5, 19)))
    c["pcd_nan_paren_big"] = ("npb.pcd", _pcd(_rows(4000, 20) + ["nan(7) 2 3"] + _rows(100, 21)))
    c["pcd_nbsp"] = ("nbsp.pcd", _pcd(_rows(10, 7) + ["1.5 2.5 3.5", "7 8 9"]))
    c["pcd_binary"] = ("bin.pcd", _pcd([], data="binary") + bytes(range(256)))
    c["pcd_binary_compressed"] = ("binc.pcd", _pcd([], data="binary_compressed") + bytes(64))
    c["pcd_no_data_line"] = ("nodata.pcd", b"VERSION 0.7\nFIELDS x y z\n1 2 3\n")
    c["pcd_all_bad"] = ("allbad.pcd", _pcd(["x y z", "1 2"]))
    c["ply_ascii"] = ("a.ply", _ply(_rows(500, 8, cols=6), props=("float x", "float y", "float z", "uchar red",
                                                                   "uchar green", "uchar blue"),
                                  tail=["3 0 1 2", "3 1 2 3"]))
    c["ply_double"] = ("d.ply", _ply(_rows(64, 9), props=("double x", "double y", "double z")))
    c["ply_count_short"] = ("s.ply", _ply(_rows(40, 10), n_vertex=100))
    c["ply_count_less"] = ("l.ply", _ply(_rows(40, 11), n_vertex=25))
    c["ply_binary"] = ("b.ply", _ply([], n_vertex=10, fmt="binary_little_endian 1.0") + bytes(120))
    c["ply_missing_z"] = ("m.ply", _ply(_rows(5, 12), props=("float x", "float y", "float w")))
    c["ply_no_end_header"] = ("n.ply", b"ply\nformat ascii 1.0\nelement vertex 2\nproperty float x\n"
                                        b"property float y\nproperty float z\n1 2 3\n4 5 6\n")
    c["las_capped"] = ("cap.las", _las(12000, 12000))
    c["las_short_tail"] = ("tail.las", _las(50, 30, extra=bytes(13)))
    c["las_short_tail_small"] = ("tails.las", _las(50, 30, extra=bytes(11)))
    c["las_reclen_28"] = ("r28.las", _las(300, 300, rec_len=28, offset=375, fmt_id=1))
    c["las_reclen_8"] = ("r8.las", _las(10, 10, rec_len=8))
    c["las_bad_signature"] = ("sig.las", _las(10, 10, sig=b"LASX"))
    c["las_truncated_header"] = ("trunc.las", b"LASF" + bytes(60))
    c["las_empty_body"] = ("empty.las", _las(10, 0))
    c["laz"] = ("x.laz", _las(10, 10))
    c["xyz_space_4col"] = ("s.xyz", ("\n".join(_rows(200, 13, cols=4)) + "\n").encode())
    c["txt_comma"] = ("c.txt", ("\n".join(r.replace(" ", ",") for r in _rows(100, 14))).encode())
    c["xyz_semicolon"] = ("s2.xyz", ("\n".join(r.replace(" ", ";") for r in _rows(100, 15))).encode())
    c["csv_named"] = ("n.csv", ("id,Z,y,X,i\n" + "\n".join(f"{k}," + r.replace(" ", ",")
                                                           for k, r in enumerate(_rows(100, 16, cols=4)))).encode())
    c["csv_unnamed"] = ("u.csv", ("a,b,c,d\n" + "\n".join(r.replace(" ", ",") for r in _rows(80, 17, cols=4))
                                  ).encode())
    c["csv_two_columns"] = ("t.csv", b"a,b\n1,2\n3,4\n")
    c["unsupported_ext"] = ("x.bin", b"1 2 3\n")
    return c


CASES = _cases()
NAMES = sorted(CASES)


def build(name):
    return CASES[name]
