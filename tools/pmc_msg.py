"""Memory-side bytes per frame of configs[4]'s MSG kernels (roofline_configs[4].traffic).

Input: the FETCH_SIZE and WRITE_SIZE passes (rocprofv3 --kernel-trace --pmc, one counter each) of
`tools/msg_pipe.py 30 0 3,3,0` — the bench's MSG leg (32 x 131 072-point batches, depth 3, G = 3: 96-frame
launches, every branch's SA1 queries inside its fused kernel), no one-batch references, so every dispatch of
these kernels is a pipeline launch.  Labels from the template prefix; a dispatch's frames from its grid (one
wavefront per centre: grid = frames x M x 64, M = N/16 at level 1, N/64 at level 2); only F-frame launches
are kept.  FETCH_SIZE is doubled (gfx950, MI355X_MICROARCH.md §HBM; checked by tools/profile_round.sh's copy
calibration), KiB -> bytes.  Output: profiles/<round>/pmc_traffic_msg.json, read by bench.py's MSG leg.

usage: python tools/pmc_msg.py PMC_FETCH_DIR PMC_WRITE_DIR OUT_JSON [F]
       python tools/pmc_msg.py --cfg1 PMC_FETCH_DIR PMC_WRITE_DIR OUT_JSON [F]  (configs[1]'s SA1 kernel, F = 256)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

N = 131072
M = {1: N // 16, 2: N // 64}
# configs[1] (SA1 only, 16 384-point frames, fp32 contract): `python tools/pmc_msg.py --cfg1 FETCH WRITE OUT [F]`
N_CFG1 = 16384
KERNELS_CFG1 = (("sa_x3_kernel<64, 64, 128, 32, 0, 2, false, true>", "sa1_group_mlp", 1),)
KERNELS = (  # (template prefix, label, level)
    ("sa_x3_kernel<32, 32, 64, 16, 0, 1, true, true>", "sa1_b0_group_mlp", 1),
    ("sa_x3_kernel<64, 64, 128, 32, 0, 2, true, true>", "sa1_b1_group_mlp", 1),
    ("sa_x3_kernel<64, 96, 128, 128, 0, 2, true, true>", "sa1_b2_group_mlp", 1),
    ("sa_x3_kernel<64, 64, 128, 32, 2, 2, true, false>", "sa2_b0_group_mlp", 2),
    ("sa_x3_kernel<128, 128, 256, 64, 2, 2, true, false>", "sa2_b1_group_mlp", 2),
    ("sa_x3_kernel<128, 128, 256, 128, 2, 2, true, false>", "sa2_b2_group_mlp", 2),
)


def rows(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    return list(csv.DictReader(open(f[0])))


def per_label(rs, counter, F, kernels=None, m=None):
    kernels, m = kernels or KERNELS, m or M
    acc, skipped = defaultdict(list), defaultdict(int)
    for r in rs:
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        hit = next(((lab, lv) for pre, lab, lv in kernels if name.startswith(pre)), None)
        if hit is None:
            continue
        lab, lv = hit
        if int(r["Grid_Size"]) != F * m[lv] * 64:
            skipped[lab] += 1
            continue
        acc[lab].append(float(r["Counter_Value"]) * 1024.0)
    return acc, dict(skipped)


def main(pf, pw, out, F=96, cfg1=False):
    F = int(F)
    kern_set, m = (KERNELS_CFG1, {1: N_CFG1 // 16}) if cfg1 else (KERNELS, M)
    (fa, fs), (wa, ws) = (per_label(rows(pf), "FETCH_SIZE", F, kern_set, m),
                          per_label(rows(pw), "WRITE_SIZE", F, kern_set, m))
    kern = {}
    for lab in sorted(set(fa) | set(wa)):
        f = 2.0 * sum(fa.get(lab, [0])) / max(1, len(fa.get(lab, [])))
        w = sum(wa.get(lab, [0])) / max(1, len(wa.get(lab, [])))
        kern[lab] = {"fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w, "traffic_per_frame": (f + w) / F,
                     "launches": len(fa.get(lab, []))}
        print(f"{lab:18s} fetch {f / 1e6:9.1f} MB  write {w / 1e6:8.1f} MB per {F}-frame launch  "
              f"({(f + w) / F / 1e6:.2f} MB per frame, {len(fa.get(lab, []))} launches)")
    src = ("tools/msg_pipe.py --cfg1 40 (configs[1]: SA1 only, 32 x 16 384-point batches, depth 3, G = 8: the bench's "
           "configs[1] leg settings" if cfg1 else
           "tools/msg_pipe.py 30 0 3,3,0 (the bench's MSG leg settings")
    res = {"config": {"workload": "sa1_16k_f32" if cfg1 else "msg_bf16", "points_per_frame": N_CFG1 if cfg1 else N,
                      "frames_per_launch": F},
           "source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes) of " + src +
                     ", no one-batch references); FETCH_SIZE x 2 (gfx950)",
           "kernels": kern, "skipped_other_sizes": {"fetch": fs, "write": ws}}
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--cfg1":
        main(*sys.argv[2:5], *(sys.argv[5:6] or [256]), cfg1=True)
    else:
        main(*sys.argv[1:5])
