"""Where the main-chain slowdown in the SSG pipeline comes from: time the MFMA levels of one
128-frame group (forward_from_sa1_fps, main stream) alone and while side streams run
(a) SA1 FPS launches, (b) FPS + the level-0 ball queries (the pipeline's side chain),
(c) only the ball queries.  Prints per-kernel ms per pass for each side load.
usage: python tools/contention.py [frames] [threads]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 128
TH = int(sys.argv[2]) if len(sys.argv) > 2 else 512
N, M1 = 65536, 4096
dev = torch.device("cuda:0")
bb = pn.PointNet2Backbone(pn.SSG, device=dev, seed=0)
xs = [torch.from_numpy(unit_frames(F, N, seed=s)).to(dev) for s in range(4)]
idx, nx = pn.farthest_point_sample(xs[0], M1, return_xyz=True, threads=TH)
fz = torch.empty(F, dtype=torch.int32, device=dev)
pn.farthest_point_sample(xs[0], M1, first_zero=fz, threads=TH)
gi = pn.ball_query(0.2, 32, xs[0], nx)
side = [torch.cuda.Stream(device=dev) for _ in range(3)]
side_out = [(torch.empty((F, M1), dtype=torch.int32, device=dev), torch.empty((F, M1, 3), device=dev),
             torch.empty((F, M1, 32), dtype=torch.int32, device=dev)) for _ in range(3)]
torch.cuda.synchronize()


def load(mode, reps=3):
    for j, s in enumerate(side):
        with torch.cuda.stream(s):
            oi, ox, og = side_out[j]
            for r in range(reps):
                x = xs[1 + j]
                if mode in ("fps", "fps+bq"):
                    pn.farthest_point_sample(x, M1, return_xyz=True, slot=1 + j, out_idx=oi, out_xyz=ox, threads=TH)
                if mode in ("fps+bq", "bq"):
                    for _ in range(1 if mode == "fps+bq" else 12):
                        pn.ball_query(0.2, 32, x, nx, out=og, slot=1 + j)


for mode in ("none", "fps", "fps+bq", "bq", "none"):
    torch.cuda.synchronize()
    load(mode)
    t = pn._Timers()
    bb.timers = t
    for _ in range(3):
        bb.forward_from_sa1_fps(xs[0], idx, nx, fz, [gi])
    bb.timers = None
    e = torch.cuda.Event()
    e.record()
    busy = [s.query() for s in side]
    torch.cuda.synchronize()
    tot = t.totals()
    ms = {k: round(v[2] / v[0], 3) for k, v in tot.items()}
    print(f"{mode:7s} main pass {sum(ms.values()):.2f} ms  side still busy at main end: {busy}  {ms}", flush=True)
