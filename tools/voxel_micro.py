"""Voxel batch micro (python tools/voxel_micro.py [B] [voxel] [scale] [N]): 20 launches on 32 x 65536 frames
(scale: the unit frames stretched by (scale, scale, scale / 200) — a LiDAR-like sparse grid at scale 100-200)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
voxel = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
scale = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
N = int(sys.argv[4]) if len(sys.argv) > 4 else 65536
f = unit_frames(B, N, 0)
if scale != 1.0:
    f = (f * [scale, scale, scale / 200]).astype("float32")
x = torch.from_numpy(f).to("cuda:0")
res = pn.voxel_downsample_batch(x, voxel)
for _ in range(19):
    pn.voxel_downsample_batch(x, voxel, check=False, out=res)
torch.cuda.synchronize()
pn.check_voxel_counts(res[3])
print("ok")
