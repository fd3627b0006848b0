"""Freeze Tier-N golden vectors (north_star operators; parity UNPINNED by the reference).

The reference has no FPS / ball query / SA-MLP / voxel code, so these
vectors come from the build's own CPU restatement (``oracle/tier_n.py``) and freeze its
spec: any later change to the restatement that alters them fails
``tests/test_oracle.py::test_tier_n_frozen_vectors``.
Run:  python tests/golden/gen_tier_n.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import tier_n  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

CASES = ["fps_4096", "fps_dups_2000", "bq_4096", "voxel_4096", "mlp_sa1", "sa_ssg_4096"]


def _weights(cfg_name, seed=0):
    from lidar_ai_recommendation_software_amd.pointnet2 import CONFIGS, init_weights
    return CONFIGS[cfg_name], init_weights(CONFIGS[cfg_name], seed)


def compute(name):
    if name == "fps_4096":
        return {"idx": tier_n.fps(unit_frames(1, 4096, 0)[0], 512)}
    if name == "fps_dups_2000":
        x = unit_frames(1, 2000, 1)[0]
        x[1000:] = x[:1000]
        return {"idx": tier_n.fps(x, 1200)}
    if name == "bq_4096":
        x = unit_frames(1, 4096, 2)[0]
        return {"idx": tier_n.ball_query(x, x[:256], 0.2, 32)}
    if name == "voxel_4096":
        c, vid, cnt = tier_n.voxel_downsample(unit_frames(1, 4096, 3)[0], 0.1)
        return {"cent": c, "vid": vid, "cnt": cnt}
    if name == "mlp_sa1":
        cfg, w = _weights("ssg")
        x = unit_frames(1, 2048, 4)[0]
        c = x[:64]
        gi = tier_n.ball_query(x, c, 0.2, 32)
        return {"feat": tier_n.mlp_maxpool(tier_n.group(x, None, c, gi), w[0][0], 32)}
    if name == "sa_ssg_4096":
        from lidar_ai_recommendation_software_amd.pointnet2 import resolve
        cfg, w = _weights("ssg")
        g, _ = tier_n.sa_stack(unit_frames(1, 4096, 5)[0], {"levels": resolve(cfg, 4096)}, w)
        return {"global": g}
    raise KeyError(name)


def main():
    arrays = {}
    for name in CASES:
        for k, v in compute(name).items():
            arrays[f"{name}/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "tier_n.npz"), **arrays)


if __name__ == "__main__":
    main()
