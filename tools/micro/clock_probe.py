"""Shader clock (MHz) while (a) idle, (b) the main chain (MFMA levels) runs alone, (c) the full SSG
pipeline runs: clock probes on a side stream.  usage: python tools/micro/clock_probe.py"""
import ctypes
import os
import subprocess
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

LIB = os.path.join(HERE, "libclockprobe.so")
lib = ctypes.CDLL(LIB)
lib.clock_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")
out = torch.zeros(2 * 4096, dtype=torch.float64, device=dev)
ps = torch.cuda.Stream(device=dev)


def probes(k0, count, gap_s):
    for j in range(count):
        lib.clock_probe(ctypes.c_void_p(out.data_ptr()), k0 + j, 100, ctypes.c_void_p(ps.cuda_stream))
        time.sleep(gap_s)


def mhz(k0, count):
    torch.cuda.synchronize()
    o = out.cpu().numpy().reshape(-1, 2)[k0:k0 + count]
    r = [c / w * 100.0 for c, w in o if w > 0]
    r.sort()
    return r[len(r) // 2], r[0], r[-1]


B, N = 32, 65536
bb = pn.PointNet2Backbone(pn.SSG, device=dev, seed=0)
xs = [torch.from_numpy(unit_frames(B, N, seed=s)).to(dev) for s in range(8)]
# (a) idle
probes(0, 20, 0.002)
print("idle            MHz median/min/max %.0f %.0f %.0f" % mhz(0, 20))
# (b) main chain alone: forward_from_sa1_fps over a 128-frame group, repeated
x = torch.cat(xs[:4])
idx, nx = pn.farthest_point_sample(x, N // 16, return_xyz=True, threads=512)
fz = torch.empty(4 * B, dtype=torch.int32, device=dev)
pn.farthest_point_sample(x, N // 16, first_zero=fz, threads=512)
torch.cuda.synchronize()
for _ in range(2):
    bb.forward_from_sa1_fps(x, idx, nx, fz, None)
torch.cuda.synchronize()
for _ in range(40):
    bb.forward_from_sa1_fps(x, idx, nx, fz, None)
probes(100, 20, 0.004)
print("main chain      MHz median/min/max %.0f %.0f %.0f" % mhz(100, 20))
torch.cuda.synchronize()
# (c) the pipeline (bench settings)
pipe = pn.StreamingSSG(bb, B, N, depth=3, fps_group=4, fps_threads=512, ramp=False, bq="bin", l2_side=True)
feed = pipe.feed()
for i in range(400):
    feed.push(xs[i % 8])
    if i == 40:
        probes(200, 30, 0.004)
feed.flush()
print("SSG pipeline    MHz median/min/max %.0f %.0f %.0f" % mhz(200, 30))
