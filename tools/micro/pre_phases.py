"""Per-section shader-clock stamps of preprocess_kernel (a LIDAR_PRE_DIAG build of liblidar_amd.so,
selected with LIDAR_AMD_LIB): one 65 536-point uniform frame.  usage:
LIDAR_AMD_LIB=lidar_ai_recommendation_software_amd/liblidar_amd_diag.so python tools/micro/pre_phases.py
(`make -C lidar_ai_recommendation_software_amd/csrc diag` builds it)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lidar_ai_recommendation_software_amd.density_stream import DensityStream  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import uniform_frame  # noqa: E402

ds = DensityStream("cuda:0", workers=1)
x = torch.from_numpy(uniform_frame(65536, 1000)).cuda()
for _ in range(3):
    ds.analyze_frame(x)
torch.cuda.synchronize()
st = ds._bufs[0]["scal"].cpu().numpy()[48:58]
names = "A colours,B mean/std,C mask,D percentile,E plane,F non-ground,G scaler,H transform,I eps".split(",")
for i, nm in enumerate(names):
    print(f"{nm:14s} {(st[i + 1] - st[i]) / 2.4e3:8.1f} us")
print(f"total          {st[9] / 2.4e3:8.1f} us (clock64 at 2.4 GHz)")
