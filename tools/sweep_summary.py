"""python tools/sweep_summary.py TAG: one line per gpu_sweep.sh result"""
import glob
import json
import sys

for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}_*.json"), key=lambda s: int(s.rsplit("_", 1)[1][:-5])):
    try:
        r = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    p, k = r["pipeline"], r["kernel_ms"]
    print(f"{f.rsplit('/', 1)[1]:14s} {r['value']:7.1f}  side {p['side_ms_per_group']:.2f} main {p['main_ms_per_group']:.2f}  "
          f"g{p['batches_per_group']} d{p['side_streams']} bq:{p['ball_query_stream']}  "
          + " ".join(f"{a}={b:.2f}" for a, b in k.items()))
