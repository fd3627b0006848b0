"""Summarise a rocprofv3 --kernel-trace CSV of a pipelined run: wall span, per-kernel busy time,
and how many SA1-FPS launches overlap (python tools/timeline.py <kernel_trace.csv> [skip_first_ms])."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
t0 = min(s for s, _, _ in ev) + skip * 1e6
ev = [e for e in ev if e[0] >= t0]
t1 = max(e for _, e, _ in ev)
span = (t1 - t0) / 1e6
print(f"span {span:.2f} ms, {len(ev)} kernels")
busy = defaultdict(float)
for s, e, n in ev:
    busy[n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]] += (e - s) / 1e6
for n, b in sorted(busy.items(), key=lambda x: -x[1])[:14]:
    print(f"  {b:9.2f} ms  {b / span * 100:5.1f}%  {n}")
# concurrency of the big FPS launches and of everything else
pts = []
for s, e, n in ev:
    fps = "fps_bucket_kernel" in n and (e - s) > 1e6
    pts.append((s, 1, fps))
    pts.append((e, -1, fps))
pts.sort()
cur_f = cur_o = 0
last = pts[0][0]
hist = defaultdict(float)
other_idle = 0.0
for t, d, fps in pts:
    dt = (t - last) / 1e6
    hist[cur_f] += dt
    if cur_o == 0:
        other_idle += dt
    last = t
    if fps:
        cur_f += d
    else:
        cur_o += d
print("time by number of concurrent SA1-FPS launches:", {k: round(v, 2) for k, v in sorted(hist.items())})
print(f"time with no non-FPS kernel running: {other_idle:.2f} ms ({other_idle / span * 100:.1f}%)")
