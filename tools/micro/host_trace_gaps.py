"""What the main stream waits for, pass by pass, in a kernel + memory-copy trace of tools/host_feed_probe.py
(rocprofv3 --kernel-trace --memory-copy-trace --output-format csv).  Each StreamingSSG run pairs its k-th SA1
FPS launch (side streams) with its k-th SA1 MLP launch (main stream): a main pass starts when the main stream is
free (the previous pass's last kernel ended), its group's side work is done (the last side kernel after the
group's FPS on that stream) and the host has issued it.  Per run: main-stream idle time before each pass,
split by which of the three came last (idle ~0 = main-bound).
usage: python tools/micro/host_trace_gaps.py TRACE_DIR"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"],
           r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", ""))
          for r in csv.DictReader(open(kt))]
    mt = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    ms = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], "H2D")
          for r in csv.DictReader(open(mt[0]))] if mt else []
    return sorted(ks + ms)


def main(d):
    ev = load(d)
    main_sid = next(s for _, _, s, n in ev if n.startswith("sa_x3_lean"))
    # every run builds a fresh pipeline and drains it, and the probe runs no other FPS or SA1 launches, so the
    # k-th SA1 FPS launch of the trace and its k-th SA1 MLP launch belong to the same group
    fps = [e for e in ev if e[2] != main_sid and e[3].startswith("fps_bucket_kernel<512")]
    sa1 = [e for e in ev if e[2] == main_sid and e[3].startswith("sa_x3_kernel<64, 64, 128, 32")]
    main_k = [e for e in ev if e[2] == main_sid]
    side_by = defaultdict(list)
    for e in ev:
        if e[2] != main_sid:
            side_by[e[2]].append(e)
    done, host = [], []
    for f in fps:  # the last side kernel on f's stream before that stream's next group (copy or FPS)
        st = side_by[f[2]]
        before = [e for e in st if e[1] <= f[0] + 1000]
        host.append(bool(before) and before[-1][3] == "H2D")
        after = [e for e in st if e[0] >= f[0]]
        nxt = next((e for e in after[1:] if e[3].startswith("fps_bucket_kernel<512") or e[3] == "H2D"
                    or e[3].startswith("__amd_rocclr_copyBuffer")), None)
        grp = [e for e in after if nxt is None or e[0] < nxt[0]]
        done.append(max(e[1] for e in grp))
    n = min(len(done), len(sa1))
    tot, cnt, passes = defaultdict(float), defaultdict(int), defaultdict(list)
    for k in range(1, n):
        s0 = sa1[k][0]
        prev_end = max((e[1] for e in main_k if e[1] <= s0 + 1000), default=s0)
        idle = (s0 - prev_end) / 1e6
        if idle > 20:  # a pipeline boundary (setup, warm-up sync)
            continue
        feed = "host" if host[k] else "device"
        if idle < 0.05:
            cls = "main-bound"
        elif done[k] > prev_end and abs(s0 - done[k]) < 0.1e6:
            cls = "side work"
        else:
            cls = "host issue"
        tot[feed, cls] += max(0.0, idle)
        cnt[feed, cls] += 1
        passes[feed].append((sa1[k][0], prev_end))
    for feed in ("device", "host"):
        m = sum(cnt[feed, c] for c in ("main-bound", "side work", "host issue"))
        print(f"{feed} feed: {m} passes; main idle before a pass: "
              + ", ".join(f"{c} {cnt[feed, c]} x / {tot[feed, c]:.1f} ms"
                          for c in ("main-bound", "side work", "host issue")))


if __name__ == "__main__":
    main(sys.argv[1])
