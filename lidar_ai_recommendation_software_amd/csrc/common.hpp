// common.hpp — shared pieces of liblidar_amd.so: handle, errors, workspace, wave helpers.
// gfx950 only: 64-lane wavefronts, built with -ffp-contract=off (every float
// expression rounds once per operation, as the CPU path it must match bit for bit).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/lidar_amd.h"

#define LIDAR_EXPORT extern "C" __attribute__((visibility("default")))

struct lidar_handle {
    int device = 0;
    void *ws = nullptr;       // scratch workspace (device)
    uint64_t ws_bytes = 0;
    void *host_pinned = nullptr;  // small pinned host buffer for scalar read-backs
};

namespace lidar {

void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
// grow the handle's workspace to `bytes`; returns device pointer or nullptr
void *workspace(lidar_handle *h, uint64_t bytes);
inline uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// carve consecutive 256-B aligned regions out of one workspace allocation
struct Carver {
    uint64_t off = 0;
    template <class T> uint64_t take(uint64_t count) {
        uint64_t o = off;
        off = align_up(off + count * sizeof(T), 256);
        return o;
    }
};

}  // namespace lidar

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return lidar::fail(LIDAR_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define LAUNCH_CHECK()                                                                     \
    do {                                                                                   \
        hipError_t e_ = hipGetLastError();                                                 \
        if (e_ != hipSuccess)                                                              \
            return lidar::fail(LIDAR_EHIP, std::string("kernel launch: ") + hipGetErrorString(e_)); \
    } while (0)

#define REQUIRE(cond, msg)                                                                 \
    do {                                                                                   \
        if (!(cond)) return lidar::fail(LIDAR_EINVAL, msg);                                \
    } while (0)

// ----------------------------------------------------------------- device helpers
namespace lidar {

// (dx*dx + dy*dy) + dz*dz with one rounding per operation (the -ffp-contract=off
// build guarantees no FMA contraction)
__device__ __forceinline__ float dist2f(float ax, float ay, float az, float bx, float by, float bz)
{
    float dx = ax - bx, dy = ay - by, dz = az - bz;
    float d = __fmul_rn(dx, dx);
    d = __fadd_rn(d, __fmul_rn(dy, dy));
    return __fadd_rn(d, __fmul_rn(dz, dz));
}

__device__ __forceinline__ double dist2d(double ax, double ay, double az, double bx, double by,
                                         double bz)
{
    double dx = ax - bx, dy = ay - by, dz = az - bz;
    double d = __dmul_rn(dx, dx);
    d = __dadd_rn(d, __dmul_rn(dy, dy));
    return __dadd_rn(d, __dmul_rn(dz, dz));
}

// argmax key: larger distance first, then LOWER index (non-negative floats order as
// their bit patterns)
__device__ __forceinline__ uint64_t make_key(float d, uint32_t idx)
{
    return ((uint64_t)__float_as_uint(d) << 32) | (uint64_t)(~idx);
}
__device__ __forceinline__ uint32_t key_index(uint64_t k) { return ~(uint32_t)(k & 0xffffffffu); }
__device__ __forceinline__ float key_dist(uint64_t k) { return __uint_as_float((uint32_t)(k >> 32)); }

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        uint64_t o = __shfl_xor(v, m, 64);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ float wave_max_f(float v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
    return v;
}
__device__ __forceinline__ float wave_min_f(float v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fminf(v, __shfl_xor(v, m, 64));
    return v;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

}  // namespace lidar
