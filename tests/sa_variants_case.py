"""Helper of tests/test_gpu_tier_n.py::test_sa_kernel_variants_bit_identical.  Runs the grouped
MLPs that have a second kernel form — the wide feature level (128 -> 128 -> 256, nsample 64 and
128: the lean kernel) — and writes every output to argv[1] (.npy).  The caller runs it under
LIDAR_SA_LEAN=0 (the 160-VGPR sa_x3_kernel) and compares with the default, bit for bit."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402


def _weights(rng, widths, cin):
    out, k = [], cin
    for c in widths:
        out.append(((rng.standard_normal((k, c)) * (1.5 / np.sqrt(k))).astype(np.float32),
                    (rng.standard_normal(c) * 0.1).astype(np.float32)))
        k = c
    return out


def run(dev):
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    outs = []
    B, N, M = 2, 1500, 203  # 406 centres: partial workgroups / waves
    for ns, seed in ((64, 3), (128, 4)):  # feature level (lean kernel)
        rng = np.random.default_rng(seed)
        layers = _weights(rng, [128, 128, 256], 131)
        packed = T(pn.pack_branch_x3(layers, False))
        P = T(rng.standard_normal((B * N, 128)).astype(np.float32))
        Q = T(rng.standard_normal((B * M, 128)).astype(np.float32) * 0.5)
        idx = T(rng.integers(0, N, (B, M, ns)).astype(np.int32))
        out = torch.full((B, M, 260), -7.0, dtype=torch.float32, device=dev)
        pn.group_mlp_x3(P, Q, idx, N, packed, [128, 128, 256], out, 2)
        outs.append(out.cpu().numpy())
    return outs


if __name__ == "__main__":
    o = run(torch.device("cuda:0"))
    np.save(sys.argv[1], np.concatenate([a.ravel() for a in o]))
