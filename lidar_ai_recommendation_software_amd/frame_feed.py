"""Host frames to the density path with the host work and the PCIe copy off the critical path
(the input step before the hot path).

The drop-in API takes one host NumPy frame per call, uploads it, runs the kernels and reads the
result back: each frame pays its parse, its copy and its kernels one after the other
(``app.py:78-84`` -> ``utils/data_processing.py:8-229``).  ``HostFrameFeed`` pipelines a stream of
frames in batches: staging threads parse (``load_lidar_data``'s multithreaded C parser for
PCD / PLY) or take the frames, pack the next `lanes` batches into pinned host buffers and issue their
H2D copies on a copy stream, while the GPU runs the current `lanes` batches through
``DensityStream.run_batches`` (one launch per phase over each CSR batch, the batches in flight at once).  Results are the drop-in API's, frame for frame (same kernels); the
reference's exceptions are raised for the first bad frame.
"""
import concurrent.futures

import numpy as np
import torch

from .data_processing import _reference_shape_errors, load_lidar_data
from .density_stream import DensityStream
from .streams import side_streams


class HostFrameFeed:
    def __init__(self, device=None, batch=32, grid_size=1.0, lanes=3):
        """batch: frames per density launch (32: the latency-bound per-frame phases then run 32 workgroups
        at once; 8 / 16 / 32 measured 133-135 / 235-236 / 290-329 M points/s on 65 536-point frames).
        lanes: batches run at once through DensityStream.run_batches (one host thread, HIP stream and
        handle each; the next `lanes` batches are staged meanwhile, one staging thread per batch);
        1: one batch at a time through run_batch."""
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.batch = max(1, int(batch))
        self.lanes = max(1, int(lanes))
        self.ds = DensityStream(self.device, workers=1, grid_size=grid_size)
        # the copies on a stream of their own, past the lanes' (run_batches takes side streams 0 .. lanes - 1)
        self.copy_stream = side_streams(self.device, 1, start=self.lanes)[0]
        nslot = 2 * self.lanes  # host staging, double-buffered per lane
        self._pinned = [None] * nslot
        self._dev = [None] * nslot
        self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=self.lanes)  # one batch each
        self._win = concurrent.futures.ThreadPoolExecutor(max_workers=1)  # stages a window of batches

    def _buffers(self, slot, rows):
        if self._pinned[slot] is None or self._pinned[slot].shape[0] < rows:
            cap = max(rows, 1 << 16)
            self._pinned[slot] = torch.empty((cap, 3), dtype=torch.float64, pin_memory=True)
            self._dev[slot] = torch.empty((cap, 3), dtype=torch.float64, device=self.device)
        return self._pinned[slot], self._dev[slot]

    def _stage(self, items, slot, from_files):
        """(staging thread) frames -> pinned rows -> H2D on the copy stream; returns the device
        frames (views) and the copy's completion event."""
        torch.cuda.set_device(self.device)
        frames = [load_lidar_data(p) if from_files else p for p in items]
        arrs = []
        for f in frames:
            a = np.asarray(f)
            _reference_shape_errors(a)
            arrs.append(a)
        sizes = [len(a) for a in arrs]
        total = sum(sizes)
        pin, dev = self._buffers(slot, total)
        host = pin.numpy()
        o = 0
        for a in arrs:
            host[o:o + len(a)] = a  # int frames convert to float64 here, as the drop-in does
            o += len(a)
        ev = torch.cuda.Event()
        with torch.cuda.stream(self.copy_stream):
            dev[:total].copy_(pin[:total], non_blocking=True)
            ev.record(self.copy_stream)
        views, o = [], 0
        for n in sizes:
            views.append(dev[o:o + n])
            o += n
        return views, ev

    def _stage_window(self, window, half, from_files):
        """(window thread) the window's batches staged in parallel into half `half` of the slots; per batch
        (views, event) or the exception its staging raised."""
        futs = [self._pool.submit(self._stage, b, half * self.lanes + j, from_files) for j, b in enumerate(window)]
        out = []
        for f in futs:
            try:
                out.append(f.result())
            except Exception as e:  # noqa: BLE001 — raised in batch order by _run
                out.append(e)
        return out

    def _run(self, items, from_files):
        batches = [items[i:i + self.batch] for i in range(0, len(items), self.batch)]
        out = []
        if not batches:
            return out
        L = self.lanes
        windows = [batches[i:i + L] for i in range(0, len(batches), L)]
        fut = self._win.submit(self._stage_window, windows[0], 0, from_files)
        for w in range(len(windows)):
            staged = fut.result()
            # window w - 1 (the other half of the slots) is complete: run_batch(es) end with host read-backs
            if w + 1 < len(windows):
                fut = self._win.submit(self._stage_window, windows[w + 1], (w + 1) % 2, from_files)
            bad = next((j for j, st in enumerate(staged) if isinstance(st, Exception)), len(staged))
            cur = torch.cuda.current_stream(self.device)
            for views, ev in staged[:bad]:
                cur.wait_event(ev)
            ok = [views for views, _ in staged[:bad]]
            if L == 1 or len(ok) == 1:
                for views in ok:
                    out += self.ds.run_batch(views)
            elif ok:
                out += [r for res in self.ds.run_batches(ok, lanes=L) for r in res]
            if bad < len(staged):  # the batches before it ran (and raised first, if one of them fails)
                raise staged[bad]
        return out

    def run(self, frames):
        """frames: host (n_i, 3) arrays -> CrowdDensityModel(grid_size).analyze dict per frame."""
        return self._run(list(frames), False)

    def run_files(self, paths):
        """point-cloud files (any format load_lidar_data reads) -> analyze dict per file; the next
        batch's files are parsed while the current batch's kernels run."""
        return self._run(list(paths), True)
