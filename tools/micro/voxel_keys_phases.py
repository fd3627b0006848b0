"""Phase cycles of the fused voxel keys launch (diagnostic build -DVX_DIAG_KEYS: s_memtime stamps of
workgroup thread 0, written into the tail rows of each frame's centroids).  usage:
LIDAR_AMD_LIB=tools/ablib/liblidar_vx_KEYS.so python tools/micro/voxel_keys_phases.py [B] [voxel]"""
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
T = (N + 8191) // 8192
x = torch.from_numpy(unit_frames(B, N, 0)).to("cuda:0")
for _ in range(3):
    c, vid, cnt, nv = pn.voxel_downsample_batch(x, voxel)
torch.cuda.synchronize()
raw = c.cpu().numpy().reshape(B, -1).view(np.uint64)  # (B, 1.5 N) words
st = np.stack([raw[:, raw.shape[1] - 12 * (t + 1): raw.shape[1] - 12 * t] for t in range(T)], 1).astype(np.int64)
rt = st[:, :, 10:12].astype(np.float64) * 0.01  # s_memrealtime (100 MHz): start, end in us
st = st[:, :, :10]
d = np.diff(st, axis=2).astype(np.float64)  # (B, T, 9)
names = ["extent publish", "extent poll", "grid+tables", "keys+hist", "hist publish", "hist poll", "scan+offsets",
         "bucket table", "scatter"]
print(f"B={B}: mean cycles per phase " + ", ".join(f"{k} {v:.0f}" for k, v in zip(names, d.mean(axis=(0, 1)))))
print("total per tile (mean, max):", round(float(d.sum(2).mean())), round(float(d.sum(2).max())))
for k, nm in enumerate(names):
    print(f"{nm:14s} by tile:", np.round(d[:, :, k].mean(0)).astype(int).tolist())
t0 = rt[:, :, 0].min()
print("realtime: span us %.1f, start spread us %.1f, tile life us mean %.1f max %.1f, clock GHz %.2f" % (
    rt[:, :, 1].max() - t0, rt[:, :, 0].max() - t0, (rt[:, :, 1] - rt[:, :, 0]).mean(), (rt[:, :, 1] - rt[:, :, 0]).max(),
    d.sum(2).mean() / (rt[:, :, 1] - rt[:, :, 0]).mean() / 1e3))
