"""Throughput executor for the reference density path (Tier R) on device-resident frames.

The drop-in API (``data_processing`` + ``CrowdDensityModel``) takes and returns host
NumPy arrays, one frame at a time, exactly like the reference.  A LiDAR feed wants
frames already in HBM and many of them in flight: the per-frame chain (preprocess ->
DBSCAN -> people -> density grid, ``utils/data_processing.py:127-328`` +
``models/crowd_density_model.py:23-98``) has three small host read-backs (the scalars
that size the next step, K, the grid), so one frame alone leaves the GPU idle between
them.  ``DensityStream.run`` runs ``workers`` frames concurrently, each worker thread on its
own HIP stream with its own library handle (workspace).  ``DensityStream.run_batch``
processes a whole batch of frames with one launch per phase instead (frames in CSR
layout: ``lidar_preprocess_batch_f64`` / ``lidar_people_batch_f64`` /
``lidar_density_batch_f64``), three small host read-backs per batch.  Both
return per frame the reference's ``analyze`` result (the big per-point arrays stay on
the device).  Results are the drop-in path's, bit for bit (same kernels).
"""
import ctypes
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from . import _native as nat
from .streams import side_streams


class DensityStream:
    def __init__(self, device="cuda", workers=4, grid_size=1.0):
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.workers = workers
        self.grid_size = float(grid_size)
        self._streams = side_streams(self.device, workers)
        self._bufs = [{} for _ in range(workers)]
        # one persistent host thread per lane: the library's handles (workspaces) are per thread,
        # so a lane keeps its handles from call to call instead of creating them per call
        self._lanes = []
        self._last_people = None

    def _lane(self, j):
        while len(self._lanes) <= j:
            self._lanes.append(ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"density-lane{len(self._lanes)}"))
        return self._lanes[j]

    def close(self):
        """Stop the lane threads (their handles are destroyed with them)."""
        for ex in self._lanes:
            ex.shutdown(wait=True)
        self._lanes = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

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
        nx, ny = nat.grid_dims(x_min, x_max, y_min, y_max, self.grid_size)
        m = nx * ny
        with torch.cuda.stream(s), nat.grid_alloc():
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
            nat.trim(self.device.index)  # this lane's work is done: free retired workspaces

        for f in [self._lane(w).submit(work, w) for w in range(min(self.workers, len(frames)))]:
            f.result()
        for r in out:
            if isinstance(r, Exception):
                raise r
        return out

    # ------------------------------------------------------------------ batched mode
    BATCH_SLOT = 7  # run_batch's library handle slot

    def profile(self, enable):
        """Per-phase HIP-event timing of run_batch's launches (lidar_profile): phases preprocess,
        dbscan_grid, dbscan_count, dbscan_union, dbscan_labels, label_scatter, people, density_grid."""
        nat.profile(nat.handle(self.device.index, slot=self.BATCH_SLOT), enable)

    def profile_read(self):
        """{phase: (launches, total ms)} since the last read (waits for the events)."""
        out = {}
        for name, ms in nat.profile_read(nat.handle(self.device.index, slot=self.BATCH_SLOT)):
            n, t = out.get(name, (0, 0.0))
            out[name] = (n + 1, t + ms)
        return out

    def run_batches(self, batches, lanes=3):
        """batches: list of frame lists -> list of per-batch result lists, in order, with `lanes`
        batches in flight: each lane is a host thread with its own HIP stream and library handle
        (handles are per thread), so one lane's host read-backs and latency-bound phases (the
        sequential preprocess / people chains run one workgroup per frame) overlap the other
        lanes' kernels.  Three lanes measured best (a process has 4 hardware queues; 32 x 65 536-point
        batches: 663-704 M points/s vs 602-650 with four).  Results equal run_batch's batch by batch; the first failing batch's
        exception (in batch order) is raised."""
        out = [None] * len(batches)
        lanes = max(1, min(int(lanes), len(batches)))
        caller = torch.cuda.current_stream(self.device)
        streams = side_streams(self.device, lanes)
        for st in streams:
            st.wait_stream(caller)  # the frames exist on the caller's stream

        people = [None] * len(batches)

        def work(j):
            torch.cuda.set_device(self.device)
            with torch.cuda.stream(streams[j]):
                for i in range(j, len(batches), lanes):
                    try:
                        out[i] = self._run_batch(batches[i])
                        people[i] = out[i][1]
                        out[i] = out[i][0]
                    except Exception as e:  # reported in batch order below
                        out[i] = e
            streams[j].synchronize()
            nat.trim(self.device.index)  # this lane's work is done: free retired workspaces

        for f in [self._lane(j).submit(work, j) for j in range(lanes)]:
            f.result()
        for r in out:
            if isinstance(r, Exception):
                raise r
        if batches and people[-1] is not None:  # the last batch in batch order (an empty one keeps the previous)
            self._last_people = people[-1]
        return out

    def people_of_last_batch(self):
        """The people positions of every frame of the last batch of run_batch / run_batches (in
        batch order), concatenated in frame order: a (sum K_f, 2) float64 CUDA tensor (what
        extract_people_positions returns per frame)."""
        if self._last_people is None:
            return torch.empty((0, 2), dtype=torch.float64, device=self.device)
        people, offs, K = self._last_people
        rows = [people[int(o):int(o) + int(k)] for o, k in zip(offs[:-1], K) if k > 0]
        return torch.cat(rows) if rows else people[:0]

    def run_batch(self, frames):
        """frames: list of (n_i, 3) float64 CUDA tensors -> list of analyze results, one
        launch per phase for the whole list.  Raises the reference's exception of the first
        failing frame (ValueError empty, IndexError no inlier), like `run`."""
        res, people = self._run_batch(frames)
        if people is not None:
            self._last_people = people
        torch.cuda.current_stream(self.device).synchronize()
        nat.trim(self.device.index)
        return res

    def _run_batch(self, frames):
        """run_batch's work -> (results, (people, offsets, K) or None); no shared state is
        written, so lanes of run_batches may call it concurrently."""
        F = len(frames)
        if F == 0:
            return [], None
        dev = self.device
        sizes = [int(x.shape[0]) for x in frames]
        offs_h = np.zeros(F + 1, dtype=np.int64)
        offs_h[1:] = np.cumsum(sizes)
        total, max_n = int(offs_h[-1]), max(1, max(sizes))
        x = torch.cat([t.reshape(-1, 3) for t in frames]) if F > 1 else frames[0].reshape(-1, 3)
        x = x.contiguous()
        rows = max(1, total)
        f64 = dict(dtype=torch.float64, device=dev)
        offs = torch.from_numpy(offs_h).to(dev)
        mask = torch.empty(rows, dtype=torch.uint8, device=dev)
        colors, normals, comp = (torch.empty((rows, 3), **f64) for _ in range(3))
        labels = torch.empty(rows, dtype=torch.int64, device=dev)
        scal = torch.empty((F, 64), **f64)
        h = nat.handle(self.device.index, slot=self.BATCH_SLOT)
        sp = torch.cuda.current_stream(dev).cuda_stream
        nat.call("lidar_preprocess_batch_f64", h, nat.ptr(x), nat.ptr(offs), F, max_n, nat.ptr(mask),
                 nat.ptr(colors), nat.ptr(normals), nat.ptr(comp), nat.ptr(labels), nat.ptr(scal), sp)
        people = torch.empty((rows, 2), **f64)
        kdev = torch.empty(F, dtype=torch.int64, device=dev)
        nat.call("lidar_people_batch_f64", h, nat.ptr(comp), nat.ptr(labels), nat.ptr(offs), F, max_n,
                 nat.ptr(scal), nat.ptr(people), nat.ptr(kdev), sp)
        S = scal.cpu().numpy()  # read-back 1 (also waits for people)
        for f in range(F):
            if S[f, 15] == 2.0:
                raise ValueError("zero-size array to reduction operation minimum which has no identity")
            if S[f, 15] != 0.0:
                raise IndexError("index -1 is out of bounds for axis 0 with size 0")
        K = kdev.cpu().numpy()  # read-back 2
        last_people = (people, offs_h, K)
        jobs = np.zeros((F, 8), dtype=np.float64)
        out_off = scr_off = 0
        dims = []
        for f in range(F):
            if K[f] <= 0:
                dims.append(None)
                continue
            x_min, x_max, y_min, y_max = S[f, 5], S[f, 6], S[f, 7], S[f, 8]
            nx, ny = nat.grid_dims(x_min, x_max, y_min, y_max, self.grid_size)
            m = nx * ny
            g2 = self.grid_size * 2.0
            jobs[f] = (x_min - g2, y_min - g2, self.grid_size, nx, ny, out_off, scr_off, 0)
            dims.append((nx, ny, out_off))
            out_off += nx + ny + 3 * m + 13
            scr_off += m + (m + 1) // 2 + nx + ny + 2
        res = [None] * F
        if out_off:
            jd = torch.from_numpy(jobs).to(dev)
            with nat.grid_alloc():
                out = torch.empty(out_off, **f64)
            nat.call("lidar_density_batch_f64", h, nat.ptr(people), nat.ptr(offs), nat.ptr(kdev), F, nat.ptr(jd),
                     nat.ptr(out), scr_off, sp)
            ob = out.cpu().numpy()  # read-back 3
        for f in range(F):
            if dims[f] is None:
                res[f] = {"total_people": 0, "avg_density": 0.0, "max_density": 0.0,
                          "density_map": np.zeros((1, 1)), "grid_coordinates": (np.array([0]), np.array([0])),
                          "density_values": np.array([0]), "hotspots": []}
                continue
            nx, ny, o = dims[f]
            m = nx * ny
            b = ob[o:o + nx + ny + 3 * m + 13]
            dens = b[nx + ny:nx + ny + m].reshape(nx, ny)
            flat_x, flat_y = b[nx + ny + m:nx + ny + 2 * m], b[nx + ny + 2 * m:nx + ny + 3 * m]
            stats = b[nx + ny + 3 * m:nx + ny + 3 * m + 8]
            hot = b[nx + ny + 3 * m + 8:nx + ny + 3 * m + 13].view(np.int64)[: int(stats[3])]
            flat = dens.flatten()
            res[f] = {"total_people": int(K[f]), "avg_density": np.float64(stats[1]),
                      "max_density": np.float64(stats[0]), "density_map": dens,
                      "grid_coordinates": (flat_x, flat_y), "density_values": flat,
                      "hotspots": [{"x": flat_x[i], "y": flat_y[i], "density": flat[i]} for i in hot]}
        return res, last_people
