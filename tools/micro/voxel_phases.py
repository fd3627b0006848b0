"""Phase cycles of the voxel bucket kernel (diagnostic build -DVX_DIAG_PHASES: s_memtime stamps of
workgroup thread 0, written into the scratch tail of the counts output).  usage:
LIDAR_AMD_LIB=tools/ablib/liblidar_vx_PHASES.so python tools/micro/voxel_phases.py [B] [voxel]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
voxel = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
N = 65536
x = torch.from_numpy(unit_frames(B, N, 0)).to("cuda:0")
for _ in range(3):
    c, vid, cnt, nv = pn.voxel_downsample_batch(x, voxel)
torch.cuda.synchronize()
nb = (N + 1535) // 1536
cnt = cnt.cpu().numpy()
ph = np.stack([cnt[:, N - 1 - (8 * b + np.arange(8))] for b in range(nb)], 1).astype(np.float64)  # (B, nb, 8)
names = ["range", "load+sort", "xyz gather", "count", "look-back", "emit"]
print(f"B={B} voxel={voxel} buckets/frame={nb}: mean cycles per phase " +
      ", ".join(f"{k} {v:.0f}" for k, v in zip(names, ph.mean(axis=(0, 1)))))
print("look-back cycles by bucket index (mean over frames):", np.round(ph[:, :, 4].mean(0)).astype(int).tolist())
print("spins by bucket index (mean):", np.round(ph[:, :, 6].mean(0), 1).tolist())
t = ph[:, :, 7]
print("frame 0: look-back start relative to bucket 0's (cycles):", (t[0] - t[0, 0]).astype(int).tolist())
print("frame 8: look-back start relative to bucket 0's (cycles):", (t[8] - t[8, 0]).astype(int).tolist())
