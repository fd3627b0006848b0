// Synthetic side loads for the main-chain contention question:
//   chase:  one wave per workgroup walks a random cyclic permutation of a large buffer (every load
//           depends on the previous one and misses the L2), like the FPS bucket loads but on ~no CU
//           resources;
//   occupy: 512-thread workgroups holding 64+ VGPRs per lane and 17 KiB of LDS that only sleep
//           and meet at barriers, like the FPS workgroups' CU footprint without their memory traffic.
// Both run until `us` microseconds of wall clock have passed.  Not part of the product.
#include <hip/hip_runtime.h>

__global__ void chase(const unsigned *next, unsigned start, int us, unsigned *sink)
{
    const long long w0 = wall_clock64();
    unsigned p = start + blockIdx.x * 7919u + threadIdx.x * 104729u;
    while (wall_clock64() - w0 < (long long)us * 100) {
#pragma unroll 1
        for (int k = 0; k < 64; ++k) p = next[p];
    }
    if (p == 0xffffffffu) sink[0] = p;
}

template <int NREG, int LDSF>
__global__ __launch_bounds__(512) void occupy(int us, float *sink)
{
    __shared__ float lds[LDSF > 0 ? LDSF : 1];
    const long long w0 = wall_clock64();
    float r[NREG > 0 ? NREG : 1];
#pragma unroll
    for (int i = 0; i < NREG; ++i) r[i] = (float)(threadIdx.x + i);
    for (int i = threadIdx.x; i < LDSF; i += 512) lds[i] = 0.0f;
    while (wall_clock64() - w0 < (long long)us * 100) {
        __builtin_amdgcn_s_sleep(8);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NREG; ++i) asm volatile("" : "+v"(r[i]));
    }
    float s = LDSF > 0 ? lds[threadIdx.x % (LDSF > 0 ? LDSF : 1)] : 0.0f;
#pragma unroll
    for (int i = 0; i < NREG; ++i) s += r[i];
    if (s == -1.0f) sink[0] = s;
}

// one-wave workgroups (the one-wave FPS's footprint): NREG VGPRs per lane, LDSF floats of LDS
template <int NREG, int LDSF>
__global__ __launch_bounds__(64) void occupy1(int us, float *sink)
{
    __shared__ float lds[LDSF > 0 ? LDSF : 1];
    const long long w0 = wall_clock64();
    float r[NREG > 0 ? NREG : 1];
#pragma unroll
    for (int i = 0; i < NREG; ++i) r[i] = (float)(threadIdx.x + i);
    for (int i = threadIdx.x; i < LDSF; i += 64) lds[i] = 0.0f;
    while (wall_clock64() - w0 < (long long)us * 100) {
        __builtin_amdgcn_s_sleep(8);
#pragma unroll
        for (int i = 0; i < NREG; ++i) asm volatile("" : "+v"(r[i]));
    }
    float s = LDSF > 0 ? lds[threadIdx.x % (LDSF > 0 ? LDSF : 1)] : 0.0f;
#pragma unroll
    for (int i = 0; i < NREG; ++i) s += r[i];
    if (s == -1.0f) sink[0] = s;
}

// coalesced traffic without CU footprint: one wave per workgroup reads DEPTH random 1-KiB chunks
// (16 B per lane, like an FPS bucket's float4 records) per round trip from a buffer far larger than
// the Infinity Cache, until `us` microseconds have passed
template <int DEPTH>
__global__ __launch_bounds__(64) void stream1k(const float4 *buf, unsigned nchunks, int us, float *sink,
                                               unsigned long long *rounds)
{
    const long long w0 = wall_clock64();
    unsigned r = 2654435761u * (blockIdx.x + 1);
    float acc = 0.0f;
    unsigned long long nr = 0;
    while (wall_clock64() - w0 < (long long)us * 100) {
        ++nr;
        float4 v[DEPTH];
#pragma unroll
        for (int k = 0; k < DEPTH; ++k) {
            r = r * 1664525u + 1013904223u;
            v[k] = buf[(size_t)(r % nchunks) * 64 + threadIdx.x];
        }
#pragma unroll
        for (int k = 0; k < DEPTH; ++k) acc += v[k].x;
    }
    if (acc == -1.0f) sink[0] = acc;
    if (threadIdx.x == 0) atomicAdd(rounds, nr);
}

extern "C" int contend_stream(const void *buf, unsigned nchunks, int blocks, int depth, int us, float *sink,
                              unsigned long long *rounds, void *stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    const float4 *b = static_cast<const float4 *>(buf);
    if (depth == 1) hipLaunchKernelGGL(stream1k<1>, dim3(blocks), dim3(64), 0, st, b, nchunks, us, sink, rounds);
    if (depth == 4) hipLaunchKernelGGL(stream1k<4>, dim3(blocks), dim3(64), 0, st, b, nchunks, us, sink, rounds);
    if (depth == 16) hipLaunchKernelGGL(stream1k<16>, dim3(blocks), dim3(64), 0, st, b, nchunks, us, sink, rounds);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int contend_chase(const unsigned *next, int blocks, int us, unsigned *sink, void *stream)
{
    hipLaunchKernelGGL(chase, dim3(blocks), dim3(64), 0, static_cast<hipStream_t>(stream), next, 12345u, us, sink);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int contend_occupy(int blocks, int us, float *sink, void *stream, int variant)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (variant == 0) hipLaunchKernelGGL((occupy<64, 17 * 256>), dim3(blocks), dim3(512), 0, st, us, sink);
    if (variant == 1) hipLaunchKernelGGL((occupy<0, 17 * 256>), dim3(blocks), dim3(512), 0, st, us, sink);
    if (variant == 2) hipLaunchKernelGGL((occupy<64, 0>), dim3(blocks), dim3(512), 0, st, us, sink);
    if (variant == 3) hipLaunchKernelGGL((occupy1<116, 22 * 256>), dim3(blocks), dim3(64), 0, st, us, sink);
    if (variant == 4) hipLaunchKernelGGL((occupy1<116, 0>), dim3(blocks), dim3(64), 0, st, us, sink);
    if (variant == 5) hipLaunchKernelGGL((occupy1<0, 22 * 256>), dim3(blocks), dim3(64), 0, st, us, sink);
    if (variant == 6) hipLaunchKernelGGL((occupy1<0, 11 * 256>), dim3(blocks), dim3(64), 0, st, us, sink);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
