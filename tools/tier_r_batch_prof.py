"""Tier R batch path only (for rocprofv3 --stats): 32 uniform 65 536-point frames, 5 runs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd.density_stream import DensityStream  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import uniform_frame  # noqa: E402

dev = torch.device("cuda:0")
xs = [torch.from_numpy(uniform_frame(65536, 1000 + i)).to(dev) for i in range(32)]
ds = DensityStream(dev, workers=4)
for _ in range(5):
    ds.run_batch(xs)
torch.cuda.synchronize()
print("ok")
