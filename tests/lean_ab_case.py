"""Helper of tests/test_gpu_tier_n.py::test_sa2_lean_kernel_bit_identical: runs one SA2-shaped
x3 grouped MLP (128 -> 128 -> 256, nsample 64 and 128) and writes the outputs to argv[1] (.npy).
The caller runs it under LIDAR_SA_LEAN=0 (the 160-VGPR sa_x3_kernel) and compares with the
default lean kernel, bit for bit."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402


def run(dev):
    outs = []
    for ns, seed in ((64, 3), (128, 4)):
        rng = np.random.default_rng(seed)
        B, N, M = 2, 1500, 203  # 406 centres: the last workgroup has dead waves
        x = unit_frames(B, N, seed)
        c = np.ascontiguousarray(x[:, :M])
        w2 = (rng.standard_normal((128, 128)) * 0.1).astype(np.float32)
        w3 = (rng.standard_normal((128, 256)) * 0.1).astype(np.float32)
        b1, b2, b3 = [(rng.standard_normal(k) * 0.1).astype(np.float32) for k in (128, 128, 256)]
        w1 = (rng.standard_normal((131, 128)) * 0.1).astype(np.float32)
        packed = torch.from_numpy(pn.pack_branch_x3([(w1, b1), (w2, b2), (w3, b3)], False)).to(dev)
        P = torch.from_numpy(rng.standard_normal((B * N, 128)).astype(np.float32)).to(dev)
        Q = torch.from_numpy(rng.standard_normal((B * M, 128)).astype(np.float32) * 0.5).to(dev)
        idx = torch.from_numpy(rng.integers(0, N, (B, M, ns)).astype(np.int32)).to(dev)
        out = torch.full((B, M, 260), -7.0, dtype=torch.float32, device=dev)
        pn.group_mlp_x3(P, Q, idx, N, packed, [128, 128, 256], out, 2)
        outs.append(out.cpu().numpy())
    return outs


if __name__ == "__main__":
    o = run(torch.device("cuda:0"))
    np.save(sys.argv[1], np.concatenate([a.ravel() for a in o]))
