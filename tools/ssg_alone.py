"""One SSG forward() over a 128-frame group (the driver's launch size), nothing else on the chip:
the kernels alone, for per-kernel PMC passes (tools/pmc_kern.sh TAG tools/ssg_alone.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

dev = torch.device("cuda:0")
bb = pn.PointNet2Backbone(pn.SSG, device=dev, seed=0)
x = torch.cat([torch.from_numpy(unit_frames(32, 65536, seed=s)).to(dev) for s in range(4)])
for _ in range(2):
    bb.forward(x)
torch.cuda.synchronize()
print("ok")
