"""Synthetic LiDAR frames used by the tests, the golden-vector generator and bench.py.

There is no dataset on the GPU box, so every workload is generated from a seed:

* ``uniform_frame(n, seed)`` — ``np.random.default_rng(seed).uniform(-15, 15, (n, 3))``
  float64, the frame SURVEY.md §6/§8d times the reference on (a ±15 m box, the
  extent of the reference's demo generator, ``app_simplified.py:999-1000``).
* ``crowd_frame(n, seed)`` — a vectorised restatement of the reference demo's
  crowd generator (``app_simplified.py:994-1024``): flat terrain
  ``0.1·sin(x/2)·cos(y/2)`` plus "people", i.e. points within 0.3 m of one of
  ``n_people`` centres lifted to a uniform height in [0.1, 1.8].  The legacy
  ``RandomState`` draws are taken in the same order as the reference loop
  (x, y, centres, then one height per person-point in index order), so the
  reference's 10 000-point demo frame is ``crowd_frame(10000, 42)``.
* ``unit_frames(b, n, seed)`` — ``default_rng(seed).uniform(-1, 1, (b, n, 3))``
  float32, the normalised frames the SetAbstraction stack runs on (§8d:
  r = 0.2 is meaningless in metres).
"""
import numpy as np


def uniform_frame(n, seed=0, lo=-15.0, hi=15.0):
    return np.random.default_rng(seed).uniform(lo, hi, (n, 3))


def crowd_frame(n, seed=42, n_people=50):
    rs = np.random.RandomState(seed)
    x = rs.uniform(-15, 15, n)
    y = rs.uniform(-15, 15, n)
    z = np.zeros(n)
    z += 0.1 * np.sin(x * 0.5) * np.cos(y * 0.5)
    centres = rs.uniform(-10, 10, (n_people, 2))
    d = np.sqrt((x[:, None] - centres[None, :, 0]) ** 2 + (y[:, None] - centres[None, :, 1]) ** 2)
    inside = d.min(axis=1) < 0.3
    z[inside] = rs.uniform(0.1, 1.8, int(inside.sum()))
    return np.column_stack((x, y, z))


def unit_frames(b, n, seed=0):
    return np.random.default_rng(seed).uniform(-1.0, 1.0, (b, n, 3)).astype(np.float32)


def blob_frame(n_blobs, mean_pts, n_noise, seed=0, spread=15.0, sigma=0.6):
    """Gaussian blobs of random size (some below min_samples) plus uniform noise,
    shuffled: gives DBSCAN many clusters, border points and noise (label
    coverage the uniform frames, which form one cluster, do not give)."""
    rng = np.random.default_rng(seed)
    centres = rng.uniform(-spread, spread, (n_blobs, 3))
    sizes = rng.integers(2, 2 * mean_pts, n_blobs)
    parts = [c + rng.normal(0.0, sigma, (k, 3)) for c, k in zip(centres, sizes)]
    parts.append(rng.uniform(-spread, spread, (n_noise, 3)))
    pts = np.concatenate(parts)
    return pts[rng.permutation(len(pts))]


def lattice_frame(per_axis, mean_pts, n_noise, seed=0, spread=15.0, sigma=0.8):
    """Blobs on a jittered ``per_axis``³ lattice (spacing > the reference's
    eps, which is ~0.29·spread in raw units after StandardScaler) so DBSCAN
    yields tens of clusters, plus tiny blobs (< min_samples) and noise."""
    rng = np.random.default_rng(seed)
    g = np.linspace(-spread, spread, per_axis)
    centres = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    centres = centres + rng.uniform(-0.1 * spread / per_axis, 0.1 * spread / per_axis, centres.shape)
    sizes = rng.integers(2, 2 * mean_pts, len(centres))
    parts = [c + rng.normal(0.0, sigma, (k, 3)) for c, k in zip(centres, sizes)]
    parts.append(rng.uniform(-spread, spread, (n_noise, 3)))
    pts = np.concatenate(parts)
    return pts[rng.permutation(len(pts))]
