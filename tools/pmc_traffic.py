"""Reduce rocprofv3 --pmc passes of bench.py to memory-side bytes per frame per kernel.

Input: the FETCH_SIZE and WRITE_SIZE counter CSVs of `tools/profile_round.sh` (one pass per
counter, `--kernel-trace` only beside `--pmc`) plus its calibration passes (a 1 GiB device copy),
and the bench line each pass printed (its `pipeline.frames_per_launch` F).  The passes run
`bench.py --no-verify` at the driver's settings (--steps 20: G = 4 batches of 32 frames, 128-frame
launches), so every library launch is a pipeline launch of F frames: the one-batch forward()
references that the timed bench compares against are not issued.

Labels come from the kernel's template prefix (`label`).  Each dispatch's frames are derived from
its Grid_Size with the launch geometry of its kernel (`frames_of`): one workgroup per frame for
FPS and the ball-query binning, one wavefront per centre for the SA kernels and the grid query,
128-row tiles x 128-column tiles of 256 threads for the split-plane GEMMs.  A dispatch whose
geometry does not give exactly F frames is reported under "unmatched" and left out, so a label
never averages launches of different sizes.  Units and the gfx950 correction follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE reports half of a wide
coalesced read on gfx950, so it is doubled; the calibration pass checks both factors on this box
(copy of 2^30 bytes -> expected read and write 2^30 bytes).  The counters sit on the L2's memory
side, so Infinity-Cache hits are included: "traffic" is bytes that left the L2, an upper bound on
HBM bytes.

Output JSON (profiles/<round>/pmc_traffic.json): {"config": {..., "frames_per_launch": F},
"calibration": ..., "kernels": {label: {"fetch_bytes", "write_bytes", "traffic_bytes" (per launch
of F frames), "traffic_per_frame", "launches"}}, "unmatched": {...}}; bench.py scales
traffic_per_frame to its own launches.

usage: python tools/pmc_traffic.py CALIB_F CALIB_W PMC_FETCH PMC_WRITE BENCH_JSON OUT_JSON
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

GIB = 1 << 30
N_POINTS = 65536
M1, M2 = N_POINTS // 16, N_POINTS // 64  # SA1 / SA2 centres per frame


def rows(d):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    return list(csv.DictReader(open(f[0])))


# (template prefix, label).  First match wins; the prefixes carry the template arguments that
# tell the levels apart.  Kernels of one name that serve two levels (the ball-query binning, the
# split-plane GEMM in mode 0) are split by `frames_of`'s geometry or by duration below.
PREFIXES = (
    ("fps_bucket_kernel<512,", "sa1_fps"),  # the pipeline's SA1 FPS (--fps-threads 512)
    ("fps_bucket_kernel<1024, 1, false>", "fps_1024"),  # SA2's nested FPS (and SA1 at --fps-threads 1024)
    ("fps_bucket_kernel<1024, 1, true>", "fps_1024"),
    ("fps_bucket_kernel<1024, 1, false, 1>", "fps_1024"),  # round 5: + points per lane
    ("fps_bucket_kernel<1024, 1, true, 1>", "fps_1024"),
    ("bq_bin_kernel", "bq_bin"),
    ("bq_grid_kernel", "sa2_ball_query"),  # SA1's queries run inside its MLP kernel (bq="bin")
    ("ball_query_kernel", "ball_query_scan"),
    ("sa_x3_kernel<64, 64, 128, 32, 0, 2, false, true>", "sa1_group_mlp"),
    ("sa_x3_kernel<64, 64, 128, 32, 0, 2, false>", "sa1_group_mlp"),
    ("sa_x3_lean_kernel<128, 128, 256, 64,", "sa2_group_mlp"),
    ("sa16_kernel<64, 64, 128, 32, true", "sa1_group_mlp"),
    ("sa16_kernel<128, 128, 256, 64, false", "sa2_group_mlp"),
    ("dense_x3_kernel<0, false, false>", "dense_rows"),  # round 4: SA2's layer 1 (points, centres), by grid
    ("dense_x3_kernel<1, false, false>", "sa3_dense1"),  # fp32 rows in, h3 planes out
    ("dense_x3_kernel<1, false, true>", "sa3_dense2"),  # h3 planes in and out
    ("dense_x3_kernel<2, false, true>", "sa3_dense3_pool"),  # h3 planes in, max-pool out
    ("dense_x3_kernel<0, true, false>", "dense_x1"),
    ("dense_x3_kernel<0, false>", "dense_rows"),  # round 4 before the planes: layer 1, dense1, dense2 by grid
    ("dense_x3_kernel<2, false>", "sa3_dense3_pool"),
    ("dense_x3_kernel<0, true>", "dense_x1"),  # the bf16 spec's per-point layer 1 (MSG)
    ("dense_x3s_kernel<0, true, false>", "sa2_layer1"),  # round-3 names (split planes)
    ("dense_x3s_kernel<1, true, false>", "sa3_dense1"),
    ("dense_x3s_kernel<1, false, false>", "sa3_dense2"),
    ("dense_x3s_kernel<2, false, false>", "sa3_dense3_pool"),
    ("dense_x3_pack_kernel", "weight_pack"),
    ("dense_pack_kernel", "weight_pack"),
    ("dense_absmax_kernel", "weight_pack"),
    ("vb_", "voxel_batch"),
    ("vx_", "voxel_batch"),
    ("group_rows_kernel", "sa_generic"),
    ("group_max_kernel", "sa_generic"),
    ("concat_xyz_pad_kernel", "concat"),
    ("dense_relu_kernel", "dense_relu_fp32"),
    ("__amd_rocclr_", "runtime_copy"),
    ("at::native::", "torch"),
)


def label(name):
    """The label of a kernel name (rocprofv3's Kernel_Name), or None."""
    short = name.split("::", 1)[1] if name.startswith("void (anonymous namespace)::") else name
    short = short.replace("(anonymous namespace)::", "")
    for prefix, lab in PREFIXES:
        if short.startswith(prefix) or (prefix.startswith("at::") and prefix in name):
            return lab
    return None


def _tiles(rows_per_frame, cout, F):
    """Threads of a dense_x3s launch over F frames (128 x 128 tiles of 256 threads, grid rounded
    up to a multiple of 8 workgroups for the XCD-affine order)."""
    total = (F * rows_per_frame // 128) * (cout // 128)
    return ((total + 7) // 8) * 8 * 256


def frames_of(lab, name, grid, wg, F):
    """(label, frames) of a dispatch when its grid is that of an F-frame pipeline launch, else
    (label, None).  `lab` may be refined (the two GEMMs of SA2's per-point layer 1)."""
    if lab in ("sa1_fps", "fps_1024", "bq_bin"):
        return lab, (grid // wg if grid // wg == F else None)
    if lab == "sa1_group_mlp":
        return lab, (F if grid == F * M1 * 64 else None)
    if lab == "sa2_group_mlp":
        return lab, (F if grid == F * M2 * 64 else None)
    if lab == "sa2_ball_query":
        blocks = (F * M2 + 3) // 4
        return lab, (F if grid == ((blocks + 7) // 8) * 8 * 256 else None)
    if lab == "dense_rows":
        for rows, cout, name_ in ((M1, 128, "sa2_layer1_points"), (M2, 128, "sa2_layer1_centres"),
                                  (M2, 256, "sa3_dense1"), (M2, 512, "sa3_dense2")):
            if grid == _tiles(rows, cout, F):
                return name_, F
        return lab, None
    if lab == "sa2_layer1":
        if grid == _tiles(M1, 128, F):
            return "sa2_layer1_points", F
        if grid == _tiles(M2, 128, F):
            return "sa2_layer1_centres", F
        return lab, None
    if lab == "sa3_dense1":
        return lab, (F if grid == _tiles(M2, 256, F) else None)
    if lab == "sa3_dense2":
        return lab, (F if grid == _tiles(M2, 512, F) else None)
    if lab == "sa3_dense3_pool":
        return lab, (F if grid == _tiles(M2, 1024, F) else None)
    return lab, None


def per_label(rs, counter, F):
    """{label: [bytes of each F-frame dispatch]} and {kernel: count} of dispatches left out."""
    acc, unmatched = defaultdict(list), defaultdict(int)
    by_dur = defaultdict(list)  # same geometry, two levels: split by duration
    for r in sorted(rs, key=lambda r: int(r["Dispatch_Id"])):
        if r["Counter_Name"] != counter:
            continue
        v = float(r["Counter_Value"]) * 1024.0  # KiB -> bytes
        name = r["Kernel_Name"]
        lab = label(name)
        if lab in (None, "torch", "runtime_copy", "weight_pack", "concat", "voxel_batch", "dense_x1"):
            unmatched[(lab or "unlabelled") + ": " + name[:80]] += 1
            continue
        lab, frames = frames_of(lab, name, int(r["Grid_Size"]), int(r["Workgroup_Size"]), F)
        if frames is None:
            unmatched[lab + ": " + name[:80]] += 1
            continue
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if lab in ("fps_1024", "bq_bin"):
            by_dur[lab].append((dur, v))
        else:
            acc[lab].append(v)
    # SA2's nested FPS (prefix shortcut: microseconds) is the only 1024-thread FPS of the pipeline at
    # --fps-threads 512; the binning runs once per level per group (SA1: 65 536-point frames, long;
    # SA2: 4 096-point frames, short)
    if by_dur.get("fps_1024"):
        acc["sa2_fps"] = [v for _, v in by_dur["fps_1024"]]
    if by_dur.get("bq_bin"):
        b = sorted(by_dur["bq_bin"])
        half = len(b) // 2
        acc["sa2_bq_bin"] = [v for _, v in b[:half]]
        acc["sa1_bq_bin"] = [v for _, v in b[half:]]
    return acc, dict(unmatched)


def calib(rs, counter):
    v = [float(r["Counter_Value"]) * 1024.0 for r in rs
         if r["Counter_Name"] == counter and "copyBuffer" in r["Kernel_Name"] and int(r["Grid_Size"]) >= 65536]
    return sum(v) / len(v) if v else None


def bench_frames_per_launch(path):
    with open(path) as f:
        line = [ln for ln in f if ln.startswith("{")][-1]
    d = json.loads(line)  # the full record (--detail) or the compact last line
    return int(d["pipeline"]["frames_per_launch"] if "pipeline" in d else d["chains_ms_per_group"]["frames_per_launch"])


def main(cf, cw, pf, pw, bench_json, out):
    F = bench_frames_per_launch(bench_json)
    fetch_scale = 2.0  # gfx950: FETCH_SIZE = half the bytes of a wide coalesced read
    c_read, c_write = calib(rows(cf), "FETCH_SIZE"), calib(rows(cw), "WRITE_SIZE")
    cal = {"copy_bytes": GIB, "fetch_size_raw_bytes": c_read, "write_size_raw_bytes": c_write,
           "fetch_scale": fetch_scale,
           "fetch_check": None if c_read is None else fetch_scale * c_read / GIB,
           "write_check": None if c_write is None else c_write / GIB}
    (fa, fu), (wa, wu) = per_label(rows(pf), "FETCH_SIZE", F), per_label(rows(pw), "WRITE_SIZE", F)
    kern = {}
    for lab in sorted(set(fa) | set(wa)):
        f = fetch_scale * sum(fa.get(lab, [0])) / max(1, len(fa.get(lab, [])))
        w = sum(wa.get(lab, [0])) / max(1, len(wa.get(lab, [])))
        kern[lab] = {"fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w, "traffic_per_frame": (f + w) / F,
                     "launches": len(fa.get(lab, []))}
    # SA2's per-point layer 1 is two GEMMs per pass (point rows, centre rows): bench.py times them as one
    if "sa2_layer1_points" in kern and "sa2_layer1_centres" in kern:
        p, c = kern.pop("sa2_layer1_points"), kern.pop("sa2_layer1_centres")
        kern["sa2_layer1_points"] = {k: p[k] + c[k] for k in ("fetch_bytes", "write_bytes", "traffic_bytes",
                                                              "traffic_per_frame")}
        kern["sa2_layer1_points"]["launches"] = p["launches"]
    res = {"config": {"workload": "ssg", "points_per_frame": N_POINTS, "frames_per_gpu": 32,
                      "frames_per_launch": F},
           "source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes) of bench.py "
                     "--no-verify --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --no-standalone "
                     "--steps 20 --warmup 5 (the driver's G = 4: 128-frame launches); every dispatch whose grid is "
                     "not an F-frame pipeline launch is listed under 'unmatched' and left out",
           "calibration": cal, "kernels": kern, "unmatched": {"fetch": fu, "write": wu}}
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in kern.items():
        print(f"{k:20s} fetch {v['fetch_bytes'] / 1e6:10.2f} MB  write {v['write_bytes'] / 1e6:10.2f} MB  "
              f"per frame {v['traffic_per_frame'] / 1e6:8.3f} MB  ({v['launches']} launches)")
    print("F =", F, "calibration", cal)
    print("unmatched", fu)


if __name__ == "__main__":
    main(*sys.argv[1:7])
