"""Optional cross-frame / cross-GPU people density on a fixed venue grid.

The reference computes a density grid per frame, with edges derived from that frame's extent
(``models/crowd_density_model.py:49-54`` -> ``utils/data_processing.py:282-328``).  A venue
watched by several LiDAR feeds (one GPU each, frames sharded per rank) wants ONE grid over a
fixed extent: every frame's people binned into it, summed over frames and over GPUs.

Binning is ``calculate_grid_density``'s own (``lidar_venue_counts_f64``: np.arange edges with
the 2-grid margin, searchsorted right, the last edge closed, outside dropped).  Histogram
counts add, so after all frames of all ranks are added and the per-rank int32 grids are summed
by one RCCL all-reduce (``torch.distributed`` backend "nccl" = RCCL over xGMI on MI355X; a
nx*ny*4-byte message, 4.6 KB for a 34 x 34 venue: latency-bound), ``density()`` equals
``calculate_grid_density(all those people, x_range, y_range, grid_size)[2]`` bit for bit.
"""

import numpy as np
import torch
import torch.distributed as dist

from . import _native as nat


class VenueGrid:
    def __init__(self, x_range, y_range, grid_size=1.0, device=None):
        """x_range / y_range: the venue's extent (the (min, max) a frame's dimensions would give);
        the grid is the one calculate_grid_density builds for that extent."""
        self.x_range = (float(x_range[0]), float(x_range[1]))
        self.y_range = (float(y_range[0]), float(y_range[1]))
        self.grid_size = float(grid_size)
        self.nx, self.ny = nat.grid_dims(self.x_range[0], self.x_range[1], self.y_range[0], self.y_range[1],
                                         self.grid_size)
        self.x0 = self.x_range[0] - self.grid_size * 2.0  # data_processing.py:305-309's margin
        self.y0 = self.y_range[0] - self.grid_size * 2.0
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.counts = torch.zeros((self.nx, self.ny), dtype=torch.int32, device=self.device)

    def add(self, people):
        """Bin people (K, 2) float64 — a CUDA tensor (device-resident, e.g. DensityStream's) or a
        NumPy array (uploaded) — into the venue counts on the GPU."""
        if not isinstance(people, torch.Tensor):
            people = torch.from_numpy(np.ascontiguousarray(np.asarray(people, dtype=np.float64).reshape(-1, 2)))
        p = people.to(self.device, torch.float64).contiguous()
        if p.shape[0]:
            nat.call("lidar_venue_counts_f64", nat.handle(self.device.index), nat.ptr(p), p.shape[0], self.x0,
                     self.y0, self.grid_size, self.nx, self.ny, nat.ptr(self.counts), nat.stream_ptr())
        return self

    @staticmethod
    def backend():
        return dist.get_backend() if dist.is_available() and dist.is_initialized() else None

    def all_reduce(self, group=None):
        """Sum the venue counts over all ranks: one all_reduce(int32, SUM) — RCCL when the process
        group is "nccl"; gloo reduces a host copy (CPU tests, ranks sharing a GPU).  A one-rank
        group still runs the collective (an identity; one per reporting interval, never per frame),
        so the RCCL branch is the same code at every world size."""
        if self.backend() is None:
            return self
        if self.backend() == "nccl":
            dist.all_reduce(self.counts, op=dist.ReduceOp.SUM, group=group)
        else:
            host = self.counts.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            self.counts.copy_(host)
        return self

    def density(self):
        """(nx, ny) float64 people per square metre (calculate_grid_density's `h / g^2`)."""
        g = self.grid_size
        return self.counts.cpu().numpy().astype(np.float64) / (g * g)

    def centres(self):
        """(grid_x, grid_y) cell centres, as calculate_grid_density returns them."""
        xe = np.arange(self.x0, (self.x_range[1] + self.grid_size * 2.0) + self.grid_size, self.grid_size)
        ye = np.arange(self.y0, (self.y_range[1] + self.grid_size * 2.0) + self.grid_size, self.grid_size)
        return (xe[:-1] + xe[1:]) / 2, (ye[:-1] + ye[1:]) / 2
