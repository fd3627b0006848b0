"""SA1 FPS alone at growing batch sizes (512-thread workgroups, 65 536-point frames): launch
time and us per step, to price a time-multiplexed schedule (FPS for many frames on the whole
chip, then the MFMA levels) against the pipelined one."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

dev = torch.device("cuda:0")
N = int(os.environ.get('FPS_N', 65536))
M = N // 16
# usage: python tools/fps_scale.py [THREADS,... [B,...]]
THREADS = [int(t) for t in sys.argv[1].split(",")] if len(sys.argv) > 1 else [512]
BATCHES = [int(t) for t in sys.argv[2].split(",")] if len(sys.argv) > 2 else [128, 256, 384, 512, 768]
for T, B in [(t, b) for b in BATCHES for t in THREADS]:
    x = torch.from_numpy(unit_frames(B, N, seed=B)).to(dev)
    pn.farthest_point_sample(x, M, threads=T)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(2):
        pn.farthest_point_sample(x, M, threads=T)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 2
    print(f"N={N} T={T:4d} B={B:4d}  {ms:7.2f} ms  {ms * 1e3 / M:5.2f} us/step  {B / ms * 1e3:8.0f} frames/s", flush=True)
    del x
