"""Reduce rocprofv3 --pmc passes of bench.py to memory-side bytes per launch per kernel.

Input: the FETCH_SIZE and WRITE_SIZE counter CSVs of `tools/pmc_passes.sh` (one pass per
counter, `--kernel-trace` only beside `--pmc`) plus its calibration passes (a 1 GiB
device copy).  Units and the gfx950 correction follow MI355X_MICROARCH.md §HBM:
FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE reports exactly half of a wide
coalesced read on gfx950, so it is doubled; the calibration pass checks both factors
on this box (copy of 2^30 bytes -> expected read and write 2^30 bytes).  The counters sit
on the L2's memory side, so Infinity-Cache hits are included: "traffic" is bytes that
left the L2, an upper bound on HBM bytes.

Output JSON (profiles/<round>/pmc_traffic.json): {"config": ..., "calibration": ...,
"kernels": {label: {"fetch_bytes": F, "write_bytes": W, "traffic_bytes": F + W,
"launches": n}}}; bench.py copies traffic_bytes into roofline["traffic"].

usage: python tools/pmc_traffic.py gpurun_out/pmc_calib_f gpurun_out/pmc_calib_w \
           gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/<round>/pmc_traffic.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

GIB = 1 << 30


def rows(d):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    return list(csv.DictReader(open(f[0])))


FRAMES_PER_LAUNCH = 96  # bench.py defaults: 32 frames per batch x 3 batches per group (one launch per group)


def label(name, grid, F=FRAMES_PER_LAUNCH):
    """Kernel label of the SSG stack (N = 65536) for F frames per launch (grid = threads).
    The split-plane GEMMs of SA2's per-point layer 1 (fp32 rows in, mode 0) and group_all's
    layers are told apart by their template arguments <mode, fp32-input, x1>."""
    if "fps_bucket_kernel" in name:
        return "fps"  # split into sa1/sa2 by duration below
    if "ball_query_kernel" in name:
        return {F * 4096 * 8: "sa1_ball_query", F * 1024 * 8: "sa2_ball_query"}.get(grid)
    if "bq_grid_kernel" in name:  # one wavefront per centre
        return {F * 4096 * 64: "sa1_ball_query", F * 1024 * 64: "sa2_ball_query"}.get(grid)
    if "bq_bin_kernel" in name:
        return "bq_bin"  # one 1024-thread workgroup per frame: SA1 (65536 pts) vs SA2 (4096) by duration
    # sa_x3_kernel<C1, C2, C3, NS, layer-1 mode (0 xyz, 1 pre, 2 px), R, X1, BQ> (BQ: the SA1 kernel
    # that answers its own ball queries); sa_x3_lean_kernel<C1, C2, C3, NS> (SA2);
    # sa16_kernel<C1, C2, C3, NS, XYZ> (the native fp32-MFMA leg)
    if "sa_x3_kernel<64, 64, 128, 32, 0, 2, false" in name or "sa16_kernel<64, 64, 128, 32, true" in name:
        return "sa1_group_mlp"
    if ("sa_x3_lean_kernel<128, 128, 256, 64>" in name or "sa_x3_kernel<128, 128, 256, 64, 1, 2, false" in name
            or "sa16_kernel<128, 128, 256, 64, false" in name):
        return "sa2_group_mlp"
    if "dense_x3s_kernel<" in name:  # split-plane GEMM: <mode, fp32-input, x1>
        for key, lab in (("<0, true, false>", "sa2_layer1_points"), ("<1, true, false>", "sa3_dense1"),
                         ("<1, false, false>", "sa3_dense2"), ("<2, false, false>", "sa3_dense3_pool")):
            if key in name:
                return lab
        return None
    if "dense_relu_kernel" in name:
        return {F * 4096 * 2: "dense_shared", F * 1024 * 2: "sa2_layer1_points", F * 1024 * 4: "sa3_dense1",
                F * 1024 * 16: "sa3_dense3_pool"}.get(grid)
    if "concat_xyz_pad" in name:
        return "concat"
    return None


def per_label(rs, counter):
    acc = defaultdict(list)
    fps, bins = [], []
    nsh = 0
    for r in sorted(rs, key=lambda r: int(r["Dispatch_Id"])):
        if r["Counter_Name"] != counter:
            continue
        v = float(r["Counter_Value"]) * 1024.0  # KiB -> bytes
        lab = label(r["Kernel_Name"], int(r["Grid_Size"]))
        if lab == "fps":
            fps.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), v))
        elif lab == "bq_bin":
            bins.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), v))
        elif lab == "dense_shared":
            acc["sa2_layer1_points" if nsh % 2 == 0 else "sa3_dense2"].append(v)
            nsh += 1
        elif lab:
            acc[lab].append(v)
    if fps:  # SA1 FPS (65536 -> 4096, long) vs SA2's nested-prefix FPS (short)
        fps.sort()
        half = len(fps) // 2
        acc["sa2_fps"] = [v for _, v in fps[:half]]
        acc["sa1_fps"] = [v for _, v in fps[half:]]
    if bins:  # SA1's binning (65536-point frames, side stream) vs SA2's (4096 points, inside its query)
        bins.sort()
        half = len(bins) // 2
        acc["sa2_bq_bin"] = [v for _, v in bins[:half]]
        acc["sa1_bq_bin"] = [v for _, v in bins[half:]]
    # sa2_layer1_points = its two GEMMs (point rows, centre rows) per pass: report their sum
    if "sa2_layer1_points" in acc:
        v = acc["sa2_layer1_points"]
        passes = max(1, len(v) // 2)
        acc["sa2_layer1_points"] = [sum(v) / passes]
    return acc


def calib(rs, counter):
    v = [float(r["Counter_Value"]) * 1024.0 for r in rs
         if r["Counter_Name"] == counter and "copyBuffer" in r["Kernel_Name"] and int(r["Grid_Size"]) >= 65536]
    return sum(v) / len(v) if v else None


def main(cf, cw, pf, pw, out):
    fetch_scale = 2.0  # gfx950: FETCH_SIZE = half the bytes of a wide coalesced read
    c_read, c_write = calib(rows(cf), "FETCH_SIZE"), calib(rows(cw), "WRITE_SIZE")
    cal = {"copy_bytes": GIB, "fetch_size_raw_bytes": c_read, "write_size_raw_bytes": c_write,
           "fetch_scale": fetch_scale,
           "fetch_check": None if c_read is None else fetch_scale * c_read / GIB,
           "write_check": None if c_write is None else c_write / GIB}
    fa, wa = per_label(rows(pf), "FETCH_SIZE"), per_label(rows(pw), "WRITE_SIZE")
    kern = {}
    for lab in sorted(set(fa) | set(wa)):
        f = fetch_scale * sum(fa.get(lab, [0])) / max(1, len(fa.get(lab, [])))
        w = sum(wa.get(lab, [0])) / max(1, len(wa.get(lab, [])))
        kern[lab] = {"fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w,
                     "launches": len(fa.get(lab, []))}
    res = {"config": {"workload": "ssg", "points_per_frame": 65536, "frames_per_gpu": 32,
                      "frames_per_launch": FRAMES_PER_LAUNCH},
           "source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes) of "
                     "bench.py --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --no-standalone "
                     "--steps 6 --warmup 1",
           "calibration": cal, "kernels": kern}
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in kern.items():
        print(f"{k:18s} fetch {v['fetch_bytes'] / 1e6:10.2f} MB  write {v['write_bytes'] / 1e6:10.2f} MB")
    print("calibration", cal)


if __name__ == "__main__":
    main(*sys.argv[1:6])
