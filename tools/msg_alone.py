"""configs[4] (MSG, bf16 spec, 131 072-point frames) kernels alone: one forward() over F frames with
HIP-event timers per launch, then SA1's branches decomposed into the grid query and the MLP on given
indices.  usage: python tools/msg_alone.py [F]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 96
N = 131072
dev = torch.device("cuda:0")
bb = pn.PointNet2Backbone(pn.MSG, device=dev, seed=0, dtype="bf16")
x = torch.from_numpy(unit_frames(F, N, 3)).to(dev)
bb.forward(x)
torch.cuda.synchronize()
t = pn._Timers()
bb.timers = t
for _ in range(3):
    bb.forward(x)
torch.cuda.synchronize()
bb.timers = None
for k, (c, f, ms) in sorted(t.totals().items(), key=lambda kv: -kv[1][2]):
    print(f"{k:22s} {ms / c:8.3f} ms per launch ({f // c} frames)")
lvl = bb.levels[0]
M = N // lvl["div"]
idx, nx = pn.farthest_point_sample(x, M, return_xyz=True)
t2 = pn._Timers()
for bi, br in enumerate(lvl["branches"]):
    out = torch.empty((F, M, br["widths"][-1]), dtype=torch.float32, device=dev)
    for _ in range(3):
        gi = pn._call(t2, f"b{bi}_query", F, pn.ball_query, br["r"], br["ns"], x, nx)
        pn._call(t2, f"b{bi}_mlp_given_idx", F, pn.group_mlp_x1, x, gi, N, br["packed_x1"], br["widths"], out,
                 centres=nx)
torch.cuda.synchronize()
for k, (c, f, ms) in sorted(t2.totals().items()):
    print(f"{k:22s} {ms / c:8.3f} ms per launch ({f // c} frames)")
