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
* ``stress_frame(kind, n, seed)`` — frames built against the preprocess's parallel emulation
  of numpy's sequential fp64 sums and against the ground-plane fit (``lstsq(rcond=None)``
  truncates a singular value of ``[x y 1]`` far from the origin, at tiny magnitudes, or when
  the ground points are collinear).
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


STRESS_KINDS = ("offset_ties", "cancel", "tiny", "int_big", "powers", "collinear", "far_1e8", "xy_line")


def stress_frame(kind, n=16384, seed=0):
    """Frames whose axis-0 sums stress the sequential-chain emulation (exact ties at the
    accumulator's grid, sums crossing powers of two, heavy cancellation, tiny magnitudes, large
    integers) and whose ground designs ``[x y 1]`` are numerically rank-deficient for LAPACK
    gelsd's rcond (``cancel``, ``tiny``, ``offset_ties``, ``far_1e8``, ``collinear``) or nearly
    so (``xy_line``)."""
    rng = np.random.default_rng(seed)
    if kind == "offset_ties":  # sums reach 2^54+: increments land on exact half-ulp ties
        x = 2.0 ** 40 + rng.integers(0, 1000, n) * 0.25
        y = -(2.0 ** 39) + rng.integers(0, 1000, n) * 0.125
        z = rng.uniform(0.0, 3.0, n)
    elif kind == "cancel":  # +-1e12 alternating: the accumulator jumps between ~1e12 and ~0
        s = np.where(np.arange(n) % 2 == 0, 1.0, -1.0)
        x = s * 1e12 + rng.uniform(-1.0, 1.0, n)
        y = rng.uniform(-5.0, 5.0, n)
        z = s * 1e6 + rng.uniform(0.0, 2.0, n)
    elif kind == "tiny":  # centred random walks at 1e-140
        x, y = rng.uniform(-1e-140, 1e-140, n), rng.uniform(-1e-140, 1e-140, n)
        z = rng.uniform(0.0, 1e-140, n)
    elif kind == "int_big":
        x = rng.integers(-2 ** 31, 2 ** 31, n).astype(np.float64)
        y = rng.integers(-2 ** 20, 2 ** 20, n).astype(np.float64)
        z = rng.integers(0, 1000, n).astype(np.float64)
    elif kind == "collinear":  # every point on the line y = 2x: [x y 1] has rank 2 exactly
        x = rng.uniform(-5.0, 5.0, n)
        y = 2.0 * x
        z = rng.uniform(0.0, 3.0, n)
    elif kind == "far_1e8":  # a +-15 m scene 1e8 m from the origin
        p = rng.uniform(-15.0, 15.0, (n, 3)) + np.array([1e8, -3e7, 0.0])
        x, y, z = p.T
    elif kind == "xy_line":  # nearly collinear: y = 2x + 1e-9 noise (full rank, ill-conditioned)
        x = rng.uniform(-5.0, 5.0, n)
        y = 2.0 * x + 1e-9 * rng.standard_normal(n)
        z = rng.uniform(0.0, 3.0, n)
    else:  # "powers": +-2^k and +-1.5 * 2^k: ties in many binades
        k = rng.integers(-20, 20, (n, 3))
        m = rng.choice([1.0, 1.5, -1.0, -1.5], (n, 3))
        x, y, z = (m * np.ldexp(1.0, k)).T
        z = np.abs(z)
    return np.ascontiguousarray(np.stack([x, y, z], axis=1))
