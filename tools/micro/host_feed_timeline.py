"""Where push_host's host time goes, per call: the wait for the ring buffer's previous device copy
(copied.synchronize), the pinned fill, and _issue (the side-stream FPS work and, every G-th call once `depth`
groups are in flight, the main-stream pass).  Same pipeline as tools/host_feed_probe.py (32 x 65 536, depth 3,
G 4); the ring's events are wrapped to time their host waits.
usage: python tools/micro/host_feed_timeline.py [steps] [threads] [host|device]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lidar_ai_recommendation_software_amd import pointnet2 as pn  # noqa: E402
from lidar_ai_recommendation_software_amd.synthetic import unit_frames  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 80
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 4
mode = sys.argv[3] if len(sys.argv) > 3 else "host"
B, N, depth, G = 32, 65536, 3, 4
dev = torch.device("cuda:0")
bb = pn.PointNet2Backbone(pn.SSG, device=dev, seed=0)
hx = [unit_frames(B, N, seed=300 + i) for i in range(8)]
xs = [torch.from_numpy(h).to(dev) for h in hx]
ready = torch.cuda.Event()
ready.record()
WAIT = [0.0]


class _TimedEvent:
    def __init__(self):
        self.ev = torch.cuda.Event()

    def record(self, stream=None):
        self.ev.record(stream) if stream is not None else self.ev.record()

    def wait(self, stream):
        self.ev.wait(stream)

    def synchronize(self):
        a = time.perf_counter()
        self.ev.synchronize()
        WAIT[0] += time.perf_counter() - a


class _TimedHostGroup(pn._HostGroup):
    def __init__(self, pinned):
        self.pinned = pinned
        self.copied = _TimedEvent()
        self.copied.record()


pn._HostGroup = _TimedHostGroup
ISSUE = [0.0]
_orig_issue = pn._Feed._issue


def _timed_issue(self, xs, readies=None):
    a = time.perf_counter()
    r = _orig_issue(self, xs, readies)
    ISSUE[0] += time.perf_counter() - a
    return r


pn._Feed._issue = _timed_issue
PARTS = {"fps": [], "rest": []}
_orig_fps, _orig_rest = pn.StreamingSSG._fps, pn.StreamingSSG._rest


def _timed_fps(self, *a):
    t = time.perf_counter()
    r = _orig_fps(self, *a)
    PARTS["fps"].append((CALL[0], time.perf_counter() - t))
    return r


def _timed_rest(self, *a):
    t = time.perf_counter()
    r = _orig_rest(self, *a)
    PARTS["rest"].append((CALL[0], time.perf_counter() - t))
    return r


CALL = [-1]
SUB = {}
_orig_call = pn._call


def _timed_call(timers, name, frames, fn, *a, **k):
    t = time.perf_counter()
    r = _orig_call(timers, name, frames, fn, *a, **k)
    SUB.setdefault(name, []).append((CALL[0], time.perf_counter() - t))
    return r


pn._call = _timed_call


def _wrap(owner, attr, name):
    orig = getattr(owner, attr)

    def w(*a, **k):
        t = time.perf_counter()
        r = orig(*a, **k)
        SUB.setdefault(name, []).append((CALL[0], time.perf_counter() - t))
        return r
    setattr(owner, attr, w)


_wrap(torch.Tensor, "copy_", "tensor.copy_")
_wrap(torch.cuda.Stream, "wait_event", "stream.wait_event")
_wrap(torch.cuda.Event, "record", "event.record")
pn.StreamingSSG._fps, pn.StreamingSSG._rest = _timed_fps, _timed_rest

pipe = pn.StreamingSSG(bb, B, N, depth=depth, fps_group=G, fps_threads=512, ramp=False, bq="bin", l2_side=True)
feed = pipe.feed()
push = (lambda i: feed.push_host(hx[i % 8], threads=threads)) if mode == "host" else (lambda i: feed.push(xs[i % 8], ready))
for i in range((depth + 2) * G):
    push(i)
torch.cuda.synchronize()
WAIT[0] = ISSUE[0] = 0.0
calls = []
t0 = time.perf_counter()
for k in PARTS:
    PARTS[k].clear()
SUB.clear()
for i in range(steps):
    CALL[0] = i
    a = time.perf_counter()
    w0, i0 = WAIT[0], ISSUE[0]
    push(i)
    d = time.perf_counter() - a
    calls.append((d, WAIT[0] - w0, ISSUE[0] - i0))
t_push = time.perf_counter() - t0
torch.cuda.synchronize()
wall = time.perf_counter() - t0
feed.flush()
c = np.array(calls) * 1e3
print(f"{mode} feed, {steps} pushes: {t_push * 1e3 / steps:.3f} ms per push issued, {wall * 1e3 / steps:.3f} ms per batch to drain")
print(f"per call: total {c[:, 0].mean():.3f} (max {c[:, 0].max():.3f}), ring wait {c[:, 1].mean():.3f} "
      f"(max {c[:, 1].max():.3f}), issue {c[:, 2].mean():.3f} (max {c[:, 2].max():.3f}), "
      f"fill+rest {(c[:, 0] - c[:, 1] - c[:, 2]).mean():.3f}")
print("per call ms (total/wait/issue):", " ".join(f"{x:.1f}/{y:.1f}/{z:.1f}" for x, y, z in c[:24]), flush=True)
for k, v in list(PARTS.items()) + sorted(SUB.items()):
    slow = [(i, round(d * 1e3, 2)) for i, d in v if d > 1e-3]
    print(f"{k}: {len(v)} calls, mean {np.mean([d for _, d in v]) * 1e3:.3f} ms, slower than 1 ms (call, ms): {slow}")
