"""Reduce one rocprofv3 --pmc pass of SQ / GRBM counters of bench.py to per-kernel VALU activity.

Counters (one pass, tools/profile_round.sh): SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES,
SQ_BUSY_CYCLES, SQ_INSTS_SALU, SQ_INSTS_VMEM_RD, GRBM_GUI_ACTIVE.  Units per MI355X_MICROARCH.md:
SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES count quad-cycles summed over waves; GRBM_GUI_ACTIVE is the
GPU-busy clock summed over the 8 XCDs, so a dispatch lasts GRBM_GUI_ACTIVE / 8 cycles.  Per kernel:

  valu_busy       = 4 * SQ_ACTIVE_INST_VALU / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
                    (the share of all SIMD-cycles of the dispatch spent issuing VALU)
  valu_issue_frac = 2 * SQ_INSTS_VALU / (1024 * GRBM_GUI_ACTIVE / 8)
                    (a wave64 VALU instruction takes 2 SIMD-32 cycles: the VALU-throughput roofline)

rocprofv3 serialises dispatches while collecting counters, so each row is the kernel alone.

usage: python tools/pmc_valu.py gpurun_out/<tag>/pmc_valu gpurun_out/<tag>/pmc_valu.json profiles/<round>/pmc_valu.json
"""
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import bench_frames_per_launch, frames_of, label, rows  # noqa: E402

SIMDS = 1024


def main(d, bench_json, out):
    F = bench_frames_per_launch(bench_json)
    per = defaultdict(lambda: defaultdict(float))  # (dispatch) -> counter -> value
    meta = {}
    for r in rows(d):
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[k] = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["Workgroup_Size"]),
                   int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    acc = defaultdict(list)
    bins = []
    unmatched = defaultdict(int)
    for k in sorted(per):
        name, grid, wg, dur = meta[k]
        lab = label(name)
        if lab in (None, "torch", "runtime_copy", "weight_pack", "concat"):
            unmatched[(lab or "unlabelled") + ": " + name[:80]] += 1
            continue
        lab, frames = frames_of(lab, name, grid, wg, F)
        if frames is None:
            unmatched[lab + ": " + name[:80]] += 1
        elif lab == "bq_bin":
            bins.append((dur, per[k]))
        else:
            acc["sa2_fps" if lab == "fps_1024" else lab].append(per[k])
    bins.sort(key=lambda t: t[0])
    half = len(bins) // 2
    acc["sa2_bq_bin"] += [c for _, c in bins[:half]]
    acc["sa1_bq_bin"] += [c for _, c in bins[half:]]
    kern = {}
    for lab, cs in acc.items():
        if not cs:
            continue
        m = {c: sum(x.get(c, 0.0) for x in cs) / len(cs) for c in cs[0]}
        cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        kern[lab] = {"launches": len(cs), **{c.lower(): v for c, v in m.items()},
                     "valu_busy": 4 * m.get("SQ_ACTIVE_INST_VALU", 0.0) / (SIMDS * cyc) if cyc else None,
                     "valu_issue_frac": 2 * m.get("SQ_INSTS_VALU", 0.0) / (SIMDS * cyc) if cyc else None,
                     "valu_insts_per_frame": m.get("SQ_INSTS_VALU", 0.0) / F}
    res = {"config": {"workload": "ssg", "points_per_frame": 65536, "frames_per_gpu": 32,
                      "frames_per_launch": F},
           "source": "rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES "
                     "SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE of bench.py --no-verify (SSG leg only, the "
                     "driver's --steps 20: F-frame pipeline launches; other dispatches under 'unmatched')",
           "kernels": kern, "unmatched": dict(unmatched)}
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in sorted(kern.items()):
        print(f"{k:18s} valu_busy {v['valu_busy'] or 0:.3f}  issue {v['valu_issue_frac'] or 0:.3f}  "
              f"valu insts/frame {v['valu_insts_per_frame']:.3e}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
