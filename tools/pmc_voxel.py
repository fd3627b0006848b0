"""Reduce the voxel leg's rocprofv3 --pmc passes (tools/profile_round.sh step 5: FETCH_SIZE and WRITE_SIZE,
separate passes, over tools/voxel_micro.py = one warm-up-free run of 20 lidar_voxel_downsample_batch_f32
calls on 32 x 65 536-point unit frames at voxel 0.05, the bench's voxel leg shape) to memory-side bytes per
call and per kernel.  Units and the gfx950 correction as tools/pmc_traffic.py (FETCH_SIZE in KiB, doubled;
WRITE_SIZE in KiB); the calibration passes of the same profile_round.sh call check both factors.  A call is
the dispatches from one call's first launch to the next's.

usage: python tools/pmc_voxel.py gpurun_out/<tag> profiles/<round>/pmc_voxel.json
"""
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import calib, rows  # noqa: E402

FRAMES, N = 32, 65536


def per_call(rs, counter):
    calls, cur = [], None
    for r in sorted(rs, key=lambda r: int(r["Dispatch_Id"])):
        if r["Counter_Name"] != counter or "vx_" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].split("vx_", 1)[1].split("(", 1)[0].split("<", 1)[0]
        # a call starts at its first launch: bbox (round 4), extent (frames above 16 tiles) or keys
        if name in ("bbox_kernel", "extent_kernel") or (name == "keys_kernel" and (cur is None or "keys_kernel" in cur)):
            if not (name == "keys_kernel" and cur is not None and "extent_kernel" in cur and "keys_kernel" not in cur):
                cur = defaultdict(float)
                calls.append(cur)
        if cur is not None:
            cur[name] += float(r["Counter_Value"]) * 1024.0
    return calls[1:] if len(calls) > 1 else calls  # the first call also pays first-touch effects


def main(tagdir, out):
    fetch_scale = 2.0
    cf = calib(rows(os.path.join(tagdir, "pmc_calib_f")), "FETCH_SIZE")
    cw = calib(rows(os.path.join(tagdir, "pmc_calib_w")), "WRITE_SIZE")
    f = per_call(rows(os.path.join(tagdir, "vpmc_fetch")), "FETCH_SIZE")
    w = per_call(rows(os.path.join(tagdir, "vpmc_write")), "WRITE_SIZE")
    kern = {}
    for k in sorted(set().union(*f, *w)):
        fb = fetch_scale * sum(c.get(k, 0.0) for c in f) / len(f)
        wb = sum(c.get(k, 0.0) for c in w) / len(w)
        kern[k] = {"fetch_bytes": fb, "write_bytes": wb}
    tot = sum(v["fetch_bytes"] + v["write_bytes"] for v in kern.values())
    res = {"config": {"workload": "voxel_downsample_batch", "frames": FRAMES, "points_per_frame": N, "voxel": 0.05},
           "source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes) of tools/voxel_micro.py",
           "calibration": {"fetch_check": None if cf is None else fetch_scale * cf / 2 ** 30,
                           "write_check": None if cw is None else cw / 2 ** 30},
           "calls": min(len(f), len(w)), "traffic_bytes_per_call": tot, "traffic_bytes_per_point": tot / (FRAMES * N),
           "kernels": kern}
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: res[k] for k in ("calls", "traffic_bytes_per_call", "traffic_bytes_per_point")}))
    for k, v in kern.items():
        print(f"{k:20s} fetch {v['fetch_bytes'] / 1e6:8.2f} MB  write {v['write_bytes'] / 1e6:8.2f} MB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
