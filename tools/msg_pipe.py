"""configs[4] (MSG, bf16 spec, 131 072-point frames, 32 per step) through StreamingSSG at several
(depth, group) settings: wall ms per 32-frame batch in the steady state, timed as bench.py does (the window
starts and ends with `depth` groups in flight; its extras leg uses depth 3 and G = pick_group(steps, 3)).  usage: python tools/msg_pipe.py [steps [unused [depth,G[,unused] ...]]]
       python tools/msg_pipe.py --cfg1 [steps]  (configs[1] at the bench's leg settings: depth 3, G 8)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

CFG1 = len(sys.argv) > 1 and sys.argv[1] == "--cfg1"  # configs[1] (SA1 only, fp32 contract) at the bench's leg settings
if CFG1:
    sys.argv = sys.argv[:1] + sys.argv[2:3] + ["0", "3,8"]
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
settings = [tuple(int(v) for v in a.split(',')) + ((128,) if a.count(',') == 1 else ()) for a in sys.argv[3:]] or [(3, 3, 128), (3, 2, 128), (4, 2, 128), (2, 3, 128)]
dev = torch.device("cuda:0")
B, N = (32, 16384) if CFG1 else (32, 131072)
bb = pn.PointNet2Backbone(pn.SA1_ONLY, device=dev, seed=0) if CFG1 else pn.PointNet2Backbone(pn.MSG, device=dev, seed=0, dtype="bf16")
xs = [torch.from_numpy(unit_frames(B, N, seed=s)).to(dev) for s in range(4)]
ready = torch.cuda.Event()
ready.record()
# MSG_SKIP_STREAMS=k: take k pool streams first (the bench's MSG leg runs after three other
# StreamingSSG legs took 9); MSG_PRIO=-1: side streams from the high-priority pool
_skip = [torch.cuda.Stream(device=dev) for _ in range(int(os.environ.get("MSG_SKIP_STREAMS", "0")))]
prio = int(os.environ.get("MSG_PRIO", "0"))
for depth, G, sq in settings:
    pipe = pn.StreamingSSG(bb, B, N, depth=depth, fps_group=G, fps_threads=512, side_priority=prio, ramp=False, bq="bin", l2_side=True)
    feed = pipe.feed()
    for i in range((depth + 1) * G):
        feed.push(xs[i % 4], ready)
    # no sync here (as bench.py): the window starts and ends with `depth` groups in flight
    n = (steps // G) * G
    t0 = time.perf_counter()
    for i in range(n):
        feed.push(xs[i % 4], ready)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    print(f"side_ns {sq} prio {prio} skip {len(_skip)} depth {depth} G {G}: {ms:.3f} ms per batch, {B * N / ms / 1e3:.1f} M points/s", flush=True)
    feed.flush()
    del feed, pipe
    torch.cuda.synchronize()
    time.sleep(float(os.environ.get("MSG_SLEEP", "0")))  # idle between settings (clock / power recovery probe)
