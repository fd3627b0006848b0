"""Side streams that keep their hardware queues from one pipeline to the next.

HIP multiplexes every stream of a process onto GPU_MAX_HW_QUEUES (4) hardware queues per priority
level, and a stream takes its queue when it is first used: the least-loaded one at that moment.
Two streams on one queue run their kernels one after the other.  A pipeline built from fresh
``torch.cuda.Stream()`` objects therefore overlaps its streams only as well as the queue
assignment of the moment allows: the first StreamingSSG of a process gets three queues apart from
the caller's, and a second one, created later in the same process, gets one side stream on the
caller's queue, so its FPS launches serialise with the main stream's MFMA levels
(``tools/micro/queue_probe.py``; configs[4]'s MSG pipeline measured 540 -> 498 -> 403 M points/s for
three successive StreamingSSG objects in one process, ``profiles/r06/queue_probe.json``).

``side_streams(device, n)`` hands out the same n streams to every caller on the device, so a
process keeps the assignment its first pipeline got.  Work on one stream stays in order, so two
executors that take the same streams one after the other stay correct; run side by side they
share the queues (pass ``start`` to take streams beyond another executor's)."""
import torch

_POOL = {}


def side_streams(device, n, start=0, priority=0):
    """Streams start .. start + n - 1 of the device's process-wide list (created on first request)."""
    device = torch.device(device)
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    pool = _POOL.setdefault((device.index, int(priority)), [])
    while len(pool) < start + n:
        pool.append(torch.cuda.Stream(device=device, priority=priority))
    return pool[start:start + n]
