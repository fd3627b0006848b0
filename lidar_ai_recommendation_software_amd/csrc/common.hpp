// common.hpp — shared pieces of liblidar_amd.so: handle, errors, workspace, wave helpers.
// gfx950 only: 64-lane wavefronts, built with -ffp-contract=off (every float
// expression rounds once per operation, as the CPU path it must match bit for bit).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>

#include "../../include/lidar_amd.h"

#define LIDAR_EXPORT extern "C" __attribute__((visibility("default")))

namespace lidar {
// per-launch HIP events of a handle while lidar_profile is on (bench.py's in-window kernel times)
struct Prof {
    struct Rec {
        const char *name;
        hipEvent_t a, b;
    };
    std::vector<Rec> recs;
};
}  // namespace lidar

struct lidar_handle {
    int device = 0;
    void *ws = nullptr;       // scratch workspace (device)
    uint64_t ws_bytes = 0;
    // workspaces replaced by a larger one: queued kernels on any stream may still read them, so
    // they are freed only where the handle is known idle (lidar_destroy, lidar_trim), never by a
    // device-wide synchronisation in the middle of a pipeline
    std::vector<void *> retired;
    uint64_t retired_bytes = 0;
    void *host_pinned = nullptr;  // small pinned host buffer for scalar read-backs
    lidar::Prof *prof = nullptr;  // non-null while lidar_profile(h, 1) is on
    uint32_t epoch = 0;           // per-call tag of in-launch hand-offs (voxel_batch.hip's granules)
    // voxel_batch.hip's granules and meta words: their own block, written only by voxel calls (tags of
    // earlier calls, never the current one; zeroed when allocated and when the epoch wraps)
    void *vx_tags = nullptr;
    uint64_t vx_tags_bytes = 0;
};

namespace lidar {

void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

// Makes `device` current for the scope of one C-ABI call and restores the caller's device on
// return: the library never changes the calling thread's current device as a side effect.
struct DeviceScope {
    int prev = -1;
    hipError_t rc = hipSuccess;
    explicit DeviceScope(int device)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != device) rc = hipSetDevice(device);
    }
    ~DeviceScope()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// Brackets the launches issued in its scope with two HIP events on `s` when the handle is
// profiling (one record per span, read back by lidar_profile_read); free otherwise.
struct Span {
    Prof *p;
    const char *name;
    hipStream_t s;
    hipEvent_t a = nullptr;
    Span(lidar_handle *h, const char *n, hipStream_t st) : p(h ? h->prof : nullptr), name(n), s(st)
    {
        if (p && hipEventCreate(&a) == hipSuccess && hipEventRecord(a, s) != hipSuccess) {
            (void)hipEventDestroy(a);
            a = nullptr;
        }
    }
    ~Span()
    {
        if (!a) return;
        hipEvent_t b = nullptr;
        if (hipEventCreate(&b) == hipSuccess && hipEventRecord(b, s) == hipSuccess) {
            p->recs.push_back({name, a, b});
            return;
        }
        (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
    }
};
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

// the device of a C-ABI call for the rest of the enclosing scope (restored on return)
#define ON_DEVICE(dev)                                                                     \
    lidar::DeviceScope lidar_dev_scope_(dev);                                              \
    if (lidar_dev_scope_.rc != hipSuccess)                                                 \
    return lidar::fail(LIDAR_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(lidar_dev_scope_.rc))

// ----------------------------------------------------------------- device helpers
namespace lidar {

// (dx*dx + dy*dy) + dz*dz with one rounding per operation (the -ffp-contract=off
// build guarantees no FMA contraction)
// XCD-affine block order (LIDAR_XCD_MAP, default on): the hardware hands workgroup b of a launch to
// XCD b % 8, so consecutive blocks land on eight different L2s.  Blocks whose work gathers from the
// same per-frame data (all centres of a frame read that frame's rows) are renumbered so that XCD x
// runs the logical range [x G/8, (x+1) G/8) in order: a frame's gathers then hit one L2 instead of
// being fetched into all eight.  A bijection of [0, G) for any G; results do not depend on it.
#ifndef LIDAR_XCD_MAP
#define LIDAR_XCD_MAP 1
#endif
__device__ __forceinline__ int64_t xcd_block()
{
    const int64_t b = blockIdx.x;
    if (!LIDAR_XCD_MAP) return b;
    const int64_t G = gridDim.x, q = G / 8, r = G % 8, x = b % 8, i = b / 8;
    return x * q + (x < r ? x : r) + i;
}

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

// ----------------------------------------------------------------- DPP wave reductions
// gfx9 DPP controls: quad_perm [1,0,3,2] = 0xB1, [2,3,0,1] = 0x4E, row_half_mirror 0x141,
// row_mirror 0x140.  Four DPP steps reduce each 16-lane row; 4 readlanes finish the wave.
// Far cheaper than __shfl_xor (ds_bpermute, ~50+ cycles per hop).
namespace lidar {
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v)
{
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
// inclusive prefix sum inside each 16-lane row (row_shr 1, 2, 4, 8; lanes without a source add 0)
__device__ __forceinline__ int row_incl_scan_i32(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
    return v;
}
// inclusive prefix sum over the wave: the row scans above, then row_bcast 15 / 31 carry the rows' totals
__device__ __forceinline__ int wave_incl_scan_i32(int v)
{
    v = row_incl_scan_i32(v);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
    return v;
}
__device__ __forceinline__ float wave_max_dpp(float v)
{
    v = fmaxf(v, __int_as_float(dpp_i<0xB1>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_i<0x4E>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_i<0x141>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp_i<0x140>(__float_as_int(v))));
    const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return fmaxf(fmaxf(a, b), fmaxf(c, d));
}
__device__ __forceinline__ uint32_t wave_min_u32_dpp(uint32_t v)
{
    v = min(v, (uint32_t)dpp_i<0xB1>((int)v));
    v = min(v, (uint32_t)dpp_i<0x4E>((int)v));
    v = min(v, (uint32_t)dpp_i<0x141>((int)v));
    v = min(v, (uint32_t)dpp_i<0x140>((int)v));
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    return min(min(a, b), min(c, d));
}
// Distances in bit space: for IEEE floats that are >= +0 or the -1 sentinel, the signed
// int order of the bits IS the float order, and an int max/min needs no NaN canonicalisation,
// so LLVM fuses each DPP move into the max (1 VALU per step instead of 3).
__device__ __forceinline__ int wave_max_i32_dpp(int v)
{
    v = max(v, dpp_i<0xB1>(v));
    v = max(v, dpp_i<0x4E>(v));
    v = max(v, dpp_i<0x141>(v));
    v = max(v, dpp_i<0x140>(v));
    const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const int c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return max(max(a, b), max(c, d));
}
// wave argmax of (dbits, -idx) in bit space (see wave_max_i32_dpp); *dmax = the max bits
__device__ __forceinline__ int wave_argmax_lane_i32(int dbits, uint32_t idx, int *dmax)
{
    const int m = wave_max_i32_dpp(dbits);
    const uint64_t c = __ballot(dbits == m);
    *dmax = m;
    if (__popcll(c) == 1) return __ffsll((unsigned long long)c) - 1;
    const uint32_t mi = wave_min_u32_dpp(dbits == m ? idx : 0xffffffffu);
    return __ffsll((unsigned long long)__ballot(dbits == m && idx == mi)) - 1;
}
// lane holding the wave argmax of (d, -idx): max d, lowest idx among equal d.
// Inactive lanes pass d = -1.  Returns the lane; *dmax = the max.
__device__ __forceinline__ int wave_argmax_lane(float d, uint32_t idx, float *dmax)
{
    const float m = wave_max_dpp(d);
    const uint64_t c = __ballot(d == m);
    *dmax = m;
    if (__popcll(c) == 1) return __ffsll((unsigned long long)c) - 1;
    const uint32_t mi = wave_min_u32_dpp(d == m ? idx : 0xffffffffu);
    return __ffsll((unsigned long long)__ballot(d == m && idx == mi)) - 1;
}
}  // namespace lidar
