"""Contention experiment (GPU box): how much do the main-stream MFMA kernels slow down next to
the SA1 FPS launches of StreamingSSG, and is it the CU resources FPS holds or what it does?

  python tools/contend.py
Scenarios for SA2's fused MLP (16-row and 32-row kernels, one 64-frame pair per launch):
alone; beside lidar_diag_occupy (sleeping 1024-thread workgroups with FPS's VGPR/LDS
footprint, 64 or 128 of them); beside two FPS launches (64 frames each, 2 side streams, as the
pipeline runs them).  Also the FPS launch time alone vs beside a loop of SA2 MLPs.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import _native as nat  # noqa: E402
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

dev = torch.device("cuda:0")
lib = nat.load_library()
lib.lidar_diag_occupy.argtypes = [nat.P, nat.I64, nat.I64, nat.P, nat.P]
rng = np.random.default_rng(0)
w = pn.init_weights(pn.SSG, 0)
B, N1, N, M, ns, widths = 64, 65536, 4096, 1024, 64, [128, 128, 256]
layers = w[1][0]
P = torch.from_numpy(rng.standard_normal((B * N, 128)).astype(np.float32)).to(dev)
Q = torch.from_numpy(rng.standard_normal((B * M, 128)).astype(np.float32)).to(dev)
x = torch.from_numpy(unit_frames(B, N1, 0)).to(dev)
c = pn.farthest_point_sample(x[:, :N].contiguous(), M, return_xyz=True)[1]
gi = pn.ball_query(0.4, ns, x[:, :N].contiguous(), c)
pk16 = torch.from_numpy(pn.pack_branch16(layers, False)).to(dev)
pk32 = torch.from_numpy(pn.pack_branch(layers, 128)).to(dev)
out = torch.empty((B, M, 256), dtype=torch.float32, device=dev)
sink = torch.zeros(1, dtype=torch.int32, device=dev)
sides = [torch.cuda.Stream(dev) for _ in range(2)]
xs = [torch.from_numpy(unit_frames(B, N1, 1 + i)).to(dev) for i in range(2)]

mlps = {"mlp16": lambda: pn.group_mlp16(P, Q, gi, N, pk16, widths, out),
        "mlp32": lambda: pn.group_mlp_pre(P, Q, gi, N, pk32, 128, widths, out)}


def ev():
    return torch.cuda.Event(enable_timing=True)


def timed_loop(fn, k):
    es = [(ev(), ev()) for _ in range(k)]
    for a, b in es:
        a.record()
        fn()
        b.record()
    return es


def occupy(blocks, ms):
    iters = int(ms * 1e-3 * 2.4e9 / (127 * 64))
    for s in sides:
        with torch.cuda.stream(s):
            nat.check(lib.lidar_diag_occupy(nat.handle(0), blocks // 2, iters, nat.ptr(sink), nat.stream_ptr()),
                      "occupy")


def fps_side():
    es = []
    for s, xx in zip(sides, xs):
        with torch.cuda.stream(s):
            a, b = ev(), ev()
            a.record(s)
            pn.farthest_point_sample(xx, N1 // 16, return_xyz=True, slot=1 + sides.index(s))
            b.record(s)
            es.append((a, b))
    return es


def med(es):
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in es]))


for name, fn in mlps.items():
    fn()
    torch.cuda.synchronize()
    alone = med(timed_loop(fn, 5))
    occupy(64, 40.0)
    o64 = med(timed_loop(fn, 5))
    torch.cuda.synchronize()
    occupy(128, 40.0)
    o128 = med(timed_loop(fn, 5))
    torch.cuda.synchronize()
    f_es = fps_side()
    beside = med(timed_loop(fn, 3))
    fps_busy = med(f_es)
    print(f"{name}: alone {alone:.3f} ms | beside 64 sleeping FPS-shaped WGs {o64:.3f} | beside 128 {o128:.3f} | "
          f"beside 2x64-frame FPS {beside:.3f} ms (FPS then took {fps_busy:.2f} ms)", flush=True)

torch.cuda.synchronize()
fa = med(fps_side())
print(f"FPS 2 x 64 frames alone: {fa:.2f} ms", flush=True)
