// Shader-clock probe: one 64-thread workgroup spins ~spin_us of wall time and records the shader
// clock ticks (s_memtime) against the constant 100 MHz wall clock (s_memrealtime), so that a probe
// launched on a side stream while other kernels run reports the clock the chip is running at.
// Built by tools/micro/clock_probe.py into tools/micro/libclockprobe.so (not part of the product).
#include <hip/hip_runtime.h>

__global__ void probe(double *out, int slot, int spin_us)
{
    if (threadIdx.x != 0) return;
    const long long w0 = wall_clock64(), c0 = clock64();
    long long w = w0;
    while (w - w0 < (long long)spin_us * 100) w = wall_clock64();  // 100 MHz wall clock
    const long long c1 = clock64();
    out[2 * slot] = (double)(c1 - c0);
    out[2 * slot + 1] = (double)(w - w0);
}

extern "C" int clock_probe(double *out, int slot, int spin_us, void *stream)
{
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), out, slot, spin_us);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
