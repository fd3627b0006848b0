"""Throughput executor for the reference density path (Tier R) on device-resident frames.

The drop-in API (``data_processing`` + ``CrowdDensityModel``) takes and returns host
NumPy arrays, one frame at a time, exactly like the reference.  A LiDAR feed wants
frames already in HBM and many of them in flight: the per-frame chain (preprocess ->
DBSCAN -> people -> density grid, ``utils/data_processing.py:127-328`` +
``models/crowd_density_model.py:23-98``) has three small host read-backs (the scalars
that size the next step, K, the grid), so one frame alone leaves the GPU idle between
them.  ``DensityStream`` runs ``workers`` frames concurrently, each worker thread on its
own HIP stream with its own library handle (workspace), and returns per frame the
reference's ``analyze`` result (the big per-point arrays stay on the device and are
returned as tensors).  Results are the drop-in path's, bit for bit (same kernels).
"""
import ctypes
import threading

import numpy as np
import torch

from . import _native as nat


class DensityStream:
    def __init__(self, device="cuda", workers=4, grid_size=1.0):
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.workers = workers
        self.grid_size = float(grid_size)
        self._streams = [torch.cuda.Stream(device=self.device) for _ in range(workers)]
        self._bufs = [{} for _ in range(workers)]

    def _buffers(self, w, n):
        b = self._bufs[w]
        if b.get("n", 0) < n:
            d = self.device
            b.update(n=n, mask=torch.empty(n, dtype=torch.uint8, device=d),
                     colors=torch.empty((n, 3), dtype=torch.float64, device=d),
                     normals=torch.empty((n, 3), dtype=torch.float64, device=d),
                     comp=torch.empty((n, 3), dtype=torch.float64, device=d),
                     labels=torch.empty(n, dtype=torch.int64, device=d),
                     people=torch.empty((n, 2), dtype=torch.float64, device=d),
                     scal=torch.empty(64, dtype=torch.float64, device=d))
        return b

    def analyze_frame(self, x, w=0):
        """x: (n, 3) float64 CUDA tensor -> (result dict of CrowdDensityModel.analyze,
        device tensors {points, colors, normals, clusters} of the preprocessed frame)."""
        n = x.shape[0]
        if n == 0:
            raise ValueError("zero-size array to reduction operation minimum which has no identity")
        b = self._buffers(w, n)
        s = self._streams[w]
        h = nat.handle(self.device.index, slot=8 + w)
        sp = s.cuda_stream
        nat.call("lidar_preprocess_f64", h, nat.ptr(x), n, nat.ptr(b["mask"]), nat.ptr(b["colors"]),
                 nat.ptr(b["normals"]), nat.ptr(b["comp"]), nat.ptr(b["labels"]), nat.ptr(b["scal"]), sp)
        S = np.empty(64)
        with torch.cuda.stream(s):
            S[:] = b["scal"].cpu().numpy()
        if S[15] != 0:
            raise IndexError("index -1 is out of bounds for axis 0 with size 0")
        nin = int(S[0])
        frame = {"points": b["comp"][:nin], "colors": b["colors"][:nin], "normals": b["normals"][:nin],
                 "clusters": b["labels"][:nin]}
        k = nat.I64(0)
        nat.call("lidar_people_f64", h, nat.ptr(b["comp"]), nat.ptr(b["labels"]), nin, nat.ptr(b["people"]),
                 ctypes.byref(k), sp)
        k = k.value
        if k == 0:
            return {"total_people": 0, "avg_density": 0.0, "max_density": 0.0, "density_map": np.zeros((1, 1)),
                    "grid_coordinates": (np.array([0]), np.array([0])), "density_values": np.array([0]),
                    "hotspots": []}, frame
        x_min, x_max, y_min, y_max = S[5], S[6], S[7], S[8]
        nx, ny = nat.I64(0), nat.I64(0)
        nat.call("lidar_grid_dims", float(x_min), float(x_max), float(y_min), float(y_max), self.grid_size,
                 ctypes.byref(nx), ctypes.byref(ny))
        nx, ny = nx.value, ny.value
        m = nx * ny
        with torch.cuda.stream(s):
            gx = torch.empty(nx, dtype=torch.float64, device=self.device)
            gy = torch.empty(ny, dtype=torch.float64, device=self.device)
            buf = torch.empty(3 * m + 13, dtype=torch.float64, device=self.device)
        nat.call("lidar_density_grid_f64", h, nat.ptr(b["people"]), k, float(x_min), float(x_max), float(y_min),
                 float(y_max), self.grid_size, nx, ny, nat.ptr(gx), nat.ptr(gy), nat.ptr(buf), sp)
        with torch.cuda.stream(s):
            hb = buf.cpu().numpy()
        dens = hb[:m].reshape(nx, ny)
        flat_x, flat_y, stats = hb[m:2 * m], hb[2 * m:3 * m], hb[3 * m:3 * m + 8]
        hot = hb[3 * m + 8:3 * m + 13].view(np.int64)[: int(stats[3])]
        flat = dens.flatten()
        res = {"total_people": k, "avg_density": np.float64(stats[1]), "max_density": np.float64(stats[0]),
               "density_map": dens, "grid_coordinates": (flat_x, flat_y), "density_values": flat,
               "hotspots": [{"x": flat_x[i], "y": flat_y[i], "density": flat[i]} for i in hot]}
        return res, frame

    def run(self, frames):
        """frames: list of (n_i, 3) float64 CUDA tensors -> list of analyze results, in order.
        Worker w takes frames w, w + workers, ...; exceptions are re-raised in order."""
        out = [None] * len(frames)

        def work(w):
            torch.cuda.set_device(self.device)
            for i in range(w, len(frames), self.workers):
                try:
                    out[i] = self.analyze_frame(frames[i], w)[0]
                except Exception as e:  # reported per frame, like the reference per call
                    out[i] = e
            self._streams[w].synchronize()

        ts = [threading.Thread(target=work, args=(w,)) for w in range(min(self.workers, len(frames)))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for r in out:
            if isinstance(r, Exception):
                raise r
        return out
