"""Which torch streams share a hardware queue?  HIP maps every stream onto one of GPU_MAX_HW_QUEUES
(4) hardware queues per priority level; two streams on one queue run their kernels in order, not
side by side.  For the caller's stream (the null stream) and each of the first `n` pool streams
(torch.cuda.Stream(), normal and high priority), a ~30 ms spin kernel runs on stream A and a tiny
kernel + event on stream B; B's event completes before A's spin ends only if the two streams are
on different queues.  usage: python tools/micro/queue_probe.py [n]"""
import json
import sys
import time

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
x = torch.zeros(1, device=dev)
torch.cuda.synchronize()
# spin length: calibrate cycles for ~30 ms
CYC = 30_000_000 * 2  # ~2 GHz shader clock


def concurrent(a, b):
    """True when a tiny kernel on b finishes while a spin kernel on a is still running."""
    torch.cuda.synchronize()
    ea = torch.cuda.Event()
    eb = torch.cuda.Event()
    with torch.cuda.stream(a):
        torch.cuda._sleep(CYC)
        ea.record(a)
    with torch.cuda.stream(b):
        x.add_(1)
        eb.record(b)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.012:
        if eb.query():
            break
    res = eb.query() and not ea.query()
    torch.cuda.synchronize()
    return bool(res)


null = torch.cuda.current_stream(dev)
out = {"null_vs_pool_normal": [], "null_vs_pool_high": [], "consecutive_normal": []}
normal = [torch.cuda.Stream(device=dev) for _ in range(n)]
high = [torch.cuda.Stream(device=dev, priority=-1) for _ in range(n)]
for s in normal:
    out["null_vs_pool_normal"].append(concurrent(null, s))
for s in high:
    out["null_vs_pool_high"].append(concurrent(null, s))
for i in range(n - 1):
    out["consecutive_normal"].append(concurrent(normal[i], normal[i + 1]))
# every pair among the first 8 normal pool streams: False = same hardware queue
out["pairs_normal_first8"] = [[j for j in range(8) if j != i and not concurrent(normal[i], normal[j])]
                              for i in range(8)]
print(json.dumps(out), flush=True)
