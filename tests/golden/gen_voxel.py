"""Pin voxel_downsample's x/y binning to the REFERENCE (this container only).

SURVEY.md §8a N1: the voxel key is the grid hash of ``calculate_grid_density``
(``utils/data_processing.py:282-328``) extended to 3-D: per axis the edges are
``np.arange(lo - 2v, (hi + 2v) + v, v)`` of the frame's own extent ``lo = min, hi = max``
(the reference's 2-cell margin and arange fill), binned by histogram2d's rule (searchsorted
right, the last edge closed).  Summing a frame's voxel counts over z therefore gives the 2-D
histogram of its (x, y) columns on exactly the reference's edges, and so
``counts_xy / (v * v) == calculate_grid_density(points[:, :2], (min x, max x), (min y, max y), v)``
bit for bit.  This script runs the reference's function on seeded float32 frames (widened to
float64 exactly) and writes what it returned to ``voxel.npz`` (density grid + cell centres per
case, plus the sha256 of the input frame so drift in the generators is caught).

The reference never travels to the GPU box; only voxel.npz does.
Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_voxel.py
"""
import hashlib
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.path.insert(0, "/root/reference")

from utils.data_processing import calculate_grid_density  # noqa: E402
from voxel_cases import VOXEL_CASES  # noqa: E402


def main():
    out = {}
    for name, (make, v) in VOXEL_CASES.items():
        x = make()
        pos = x[:, :2].astype(np.float64)
        xr = (float(pos[:, 0].min()), float(pos[:, 0].max()))
        yr = (float(pos[:, 1].min()), float(pos[:, 1].max()))
        gx, gy, dens = calculate_grid_density(pos, xr, yr, v)
        out[f"{name}__density"] = dens
        out[f"{name}__grid_x"] = gx
        out[f"{name}__grid_y"] = gy
        out[f"{name}__sha"] = np.frombuffer(hashlib.sha256(np.ascontiguousarray(x).tobytes()).digest(), np.uint8)
        print(name, dens.shape, int(dens.sum() * v * v + 0.5), len(x))
    np.savez_compressed(os.path.join(HERE, "voxel.npz"), **out)


if __name__ == "__main__":
    main()
