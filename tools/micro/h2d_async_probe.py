"""Does a pinned host -> device copy_(non_blocking=True) return before the copy runs?  Host time of the call
(a) on an idle stream, (b) on a stream busy with ~10 ms of matmuls queued ahead of it, for one 25 MB batch
(32 x 65 536 x 3 float32, the SSG feed's batch), against the copy's own device time.
usage: python tools/micro/h2d_async_probe.py"""
import time

import torch

dev = torch.device("cuda:0")
nbytes = 32 * 65536 * 3 * 4
pin = torch.empty(nbytes // 4, dtype=torch.float32, pin_memory=True)
dst = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
a = torch.randn(8192, 8192, device=dev)
s = torch.cuda.Stream(device=dev)


def busy(ms_target):
    for _ in range(ms_target):
        a @ a  # ~1 ms each on the chip


with torch.cuda.stream(s):
    busy(2)
torch.cuda.synchronize()
t0 = time.perf_counter()
with torch.cuda.stream(s):
    busy(10)
torch.cuda.synchronize()
print(f"10 matmuls: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
for label, nbusy in (("idle stream", 0), ("busy stream", 10)):
    for rep in range(3):
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            busy(nbusy)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            t = time.perf_counter()
            dst.copy_(pin, non_blocking=True)
            call = time.perf_counter() - t
            e1.record(s)
        t = time.perf_counter()
        torch.cuda.synchronize()
        rest = time.perf_counter() - t
        print(f"{label}: copy_ call {call * 1e3:.3f} ms on the host, then {rest * 1e3:.3f} ms to drain; "
              f"copy on the device {e0.elapsed_time(e1):.3f} ms", flush=True)

# the feed's pattern: several streams, each busy, each with 4 copies (4 pinned buffers) queued behind its work
pins = [torch.empty(nbytes // 4, dtype=torch.float32, pin_memory=True) for _ in range(12)]
dsts = [torch.empty(nbytes // 4, dtype=torch.float32, device=dev) for _ in range(12)]
ss = [torch.cuda.Stream(device=dev) for _ in range(3)]
for rep in range(2):
    torch.cuda.synchronize()
    calls = []
    for si, st in enumerate(ss):
        with torch.cuda.stream(st):
            busy(3)
            for j in range(4):
                t = time.perf_counter()
                dsts[4 * si + j].copy_(pins[4 * si + j], non_blocking=True)
                calls.append(round((time.perf_counter() - t) * 1e3, 3))
    torch.cuda.synchronize()
    print("3 busy streams x 4 copies, host ms per copy_ call:", calls, flush=True)
# a copy whose destination a kernel on another stream reads later, with an event between (the feed's hand-off)
ev = torch.cuda.Event()
for rep in range(2):
    torch.cuda.synchronize()
    calls = []
    for si, st in enumerate(ss):
        with torch.cuda.stream(st):
            busy(3)
            for j in range(4):
                t = time.perf_counter()
                dsts[4 * si + j].copy_(pins[4 * si + j], non_blocking=True)
                ev.record(st)
                calls.append(round((time.perf_counter() - t) * 1e3, 3))
    torch.cuda.synchronize()
    print("... with an event recorded after each copy:", calls, flush=True)
# the feed's order on a side stream: wait for an event of ANOTHER (busy) stream, then the copies
other = torch.cuda.Stream(device=dev)
for rep in range(3):
    torch.cuda.synchronize()
    calls = []
    with torch.cuda.stream(other):
        busy(5)
        e_other = torch.cuda.Event()
        e_other.record(other)
    for si, st in enumerate(ss):
        with torch.cuda.stream(st):
            busy(2)
            st.wait_event(e_other)
            for j in range(4):
                t = time.perf_counter()
                dsts[4 * si + j].copy_(pins[4 * si + j], non_blocking=True)
                calls.append(round((time.perf_counter() - t) * 1e3, 3))
    t = time.perf_counter()
    torch.cuda.synchronize()
    print("after a wait on another busy stream's event, host ms per copy_ call:", calls,
          f"(drain {(time.perf_counter() - t) * 1e3:.1f} ms)", flush=True)
# many kernels and events queued on the stream (and on others) ahead of the copy: does the call then block?
small = torch.empty(1024, device=dev)
for nk, nev in ((50, 0), (200, 0), (20, 20), (50, 50), (200, 200)):
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        busy(10)
        for i in range(nk):
            small.add_(1.0)
            if i < nev:
                torch.cuda.Event().record(s)
        t = time.perf_counter()
        dst.copy_(pin, non_blocking=True)
        call = time.perf_counter() - t
    torch.cuda.synchronize()
    print(f"{nk} small kernels + {nev} events queued behind ~70 ms of matmuls: copy_ call {call * 1e3:.3f} ms", flush=True)
