"""Reduce the three SQ / GRBM passes of the round-3 PMC script (history at f4fc716) (the SSG kernels alone, tools/ssg_alone.py)
to per-kernel shares: MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x GRBM_GUI_ACTIVE / 8), and the
disjoint wave-cycle shares SQ_WAIT_ANY (parked at s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stall, a busy
matrix pipe included) and SQ_ACTIVE_INST_ANY, per MI355X_MICROARCH.md's units.

usage: python tools/pmc_sq_alone.py gpurun_out/alone profiles/<round>/pmc_sq_alone.json"""
import collections
import csv
import glob
import json
import sys

LABELS = [("sa_x3_lean", "sa2_group_mlp"), ("sa_x3_kernel", "sa1_group_mlp"), ("dense_x3s_kernel<2", "sa3_dense3_pool"),
          ("dense_x3_kernel<2", "sa3_dense3_pool"), ("dense_x3_kernel<1", "sa3_dense1_dense2"),
          ("dense_x3_kernel<0", "sa2_layer1_points_and_centres"),
          ("dense_x3s_kernel<1", "sa3_dense1_dense2"), ("dense_x3s_kernel<0", "sa2_layer1_points_and_centres"),
          ("fps_bucket", "fps"), ("bq_bin", "bq_bin"), ("bq_grid", "sa2_ball_query")]


def label(name):
    for key, lab in LABELS:
        if key in name:
            return lab
    return None


def main(prefix, out):
    rows = []
    for p in (1, 2, 3):
        rows += list(csv.DictReader(open(glob.glob(f"{prefix}_p{p}/p_counter_collection.csv")[0])))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        lab = label(r["Kernel_Name"])
        if lab:
            agg[lab][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[lab].add(r["Dispatch_Id"])
    res = {"source": "rocprofv3 --kernel-trace --pmc, three SQ/GRBM passes (tools/pmc_kern.sh TAG tools/ssg_alone.py): two SSG "
                     "forward() calls over one 128-frame group, nothing else on the chip", "kernels": {}}
    for lab, a in agg.items():
        wc = a["SQ_WAVE_CYCLES"] or 1.0
        res["kernels"][lab] = {
            "dispatches": len(disp[lab]),
            "mfma_busy": a["SQ_VALU_MFMA_BUSY_CYCLES"] / (a["GRBM_GUI_ACTIVE"] / 8 * 1024) if a["GRBM_GUI_ACTIVE"] else None,
            "wait_any": a["SQ_WAIT_ANY"] / wc, "wait_inst_any": a["SQ_WAIT_INST_ANY"] / wc,
            "active_inst_any": a["SQ_ACTIVE_INST_ANY"] / wc, "wait_inst_lds": a["SQ_WAIT_INST_LDS"] / wc,
            "insts_mfma": a["SQ_INSTS_MFMA"], "insts_valu": a["SQ_INSTS_VALU"], "insts_lds": a["SQ_INSTS_LDS"]}
    json.dump(res, open(out, "w"), indent=1)
    for lab, v in res["kernels"].items():
        print(f"{lab:30s}", {k: round(x, 3) for k, x in v.items() if k in ("mfma_busy", "wait_any", "wait_inst_any", "active_inst_any")})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
