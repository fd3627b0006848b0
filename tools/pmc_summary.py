"""Summarise tools/pmc_kern.sh passes: per-dispatch mean of every counter, kernels matching a substring.
python tools/pmc_summary.py TAG SUBSTR [SUBSTR...]"""
import collections
import csv
import glob
import sys

tag, subs = sys.argv[1], sys.argv[2:]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"gpurun_out/{tag}_p*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if subs and not any(s in k for s in subs):
            continue
        vals[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    print(k)
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    busy = m.get("SQ_BUSY_CYCLES", 0) or 1
    for c in sorted(m):
        extra = ""
        if c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE"):
            extra = f"  ({m[c] / wc * 100:.1f}% of wave-cycles)"
        print(f"   {c:28s} {m[c]:16.0f}{extra}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        print(f"   MFMA busy / (GUI_ACTIVE/8 * 256 CUs * 4 SIMDs): "
              f"{m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
