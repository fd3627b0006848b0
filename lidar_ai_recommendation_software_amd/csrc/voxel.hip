// voxel.hip — voxel downsampling on gfx950 (north_star "voxel hashing").
//
// Spec (oracle tier_n.voxel_downsample): v = floor((p - min(p)) / voxel)
// per axis in fp32 (one rounding per op), key = (vx*Dy + vy)*Dz + vz with D = max(v)+1,
// voxels in ascending key order, per-point voxel id = rank of its key, centroid =
// sequential fp32 sum of the voxel's points in point order / count.
//
// Pipeline (one frame): bbox -> keys -> stable LSD radix sort of (key, index) in one
// 1024-thread workgroup (8-bit digits; the stable in-wave rank comes from 8 ballots per
// digit: lanes with an equal digit, below me) -> run starts -> scan -> per-voxel
// sequential sums (one lane per voxel walks its run, which is in index order because
// the sort is stable).  HBM-bound integer work: no float reductions besides the
// centroid sums, whose order is part of the spec.
#include "common.hpp"

namespace {

constexpr int kT = 1024;
constexpr int kW = kT / 64;

__global__ __launch_bounds__(kT) void voxel_keys_kernel(const float *__restrict__ xyz, int64_t n, float voxel,
                                                        uint32_t *__restrict__ key, uint32_t *__restrict__ idx,
                                                        uint32_t *__restrict__ meta)
{
    __shared__ float red[3][kW];
    __shared__ int ired[3][kW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float lo[3] = {INFINITY, INFINITY, INFINITY};
    for (int64_t i = tid; i < n; i += kT)
        for (int a = 0; a < 3; ++a) lo[a] = fminf(lo[a], xyz[3 * i + a]);
    for (int a = 0; a < 3; ++a) {
        float v = lidar::wave_min_f(lo[a]);
        if (lane == 0) red[a][wave] = v;
    }
    __syncthreads();
    for (int a = 0; a < 3; ++a) {
        float v = red[a][0];
        for (int w = 1; w < kW; ++w) v = fminf(v, red[a][w]);
        lo[a] = v;
    }
    int hi[3] = {0, 0, 0};
    for (int64_t i = tid; i < n; i += kT)
        for (int a = 0; a < 3; ++a) {
            const float q = __fdiv_rn(__fsub_rn(xyz[3 * i + a], lo[a]), voxel);
            hi[a] = max(hi[a], (int)floorf(q));
        }
    for (int a = 0; a < 3; ++a) {
        int v = hi[a];
        for (int m = 32; m >= 1; m >>= 1) v = max(v, __shfl_xor(v, m, 64));
        if (lane == 0) ired[a][wave] = v;
    }
    __syncthreads();
    uint32_t dim[3];
    for (int a = 0; a < 3; ++a) {
        int v = ired[a][0];
        for (int w = 1; w < kW; ++w) v = max(v, ired[a][w]);
        dim[a] = (uint32_t)v + 1u;
    }
    for (int64_t i = tid; i < n; i += kT) {
        uint32_t c[3];
        for (int a = 0; a < 3; ++a)
            c[a] = (uint32_t)(int)floorf(__fdiv_rn(__fsub_rn(xyz[3 * i + a], lo[a]), voxel));
        key[i] = (c[0] * dim[1] + c[1]) * dim[2] + c[2];
        idx[i] = (uint32_t)i;
    }
    if (tid == 0) {
        const uint64_t tot = (uint64_t)dim[0] * dim[1] * dim[2];
        meta[0] = tot > 0xffffffffull ? 0xffffffffu : (uint32_t)tot;
        meta[1] = dim[0];
        meta[2] = dim[1];
        meta[3] = dim[2];
    }
}

// one stable 8-bit LSD pass: (kin, vin) -> (kout, vout) by digit (key >> shift) & 255
__global__ __launch_bounds__(kT) void radix_pass_kernel(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                        uint32_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                        int64_t n, int shift, const uint32_t *meta)
{
    __shared__ uint32_t cnt[256];          // total per digit, then running offsets
    __shared__ uint32_t wcnt[kW][256];     // per-wave per-digit counts of the current tile
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // skip passes above the key range (keys < meta[0])
    if (shift > 0 && ((uint64_t)meta[0] - 1) >> shift == 0) {
        for (int64_t i = tid; i < n; i += kT) {
            kout[i] = kin[i];
            vout[i] = vin[i];
        }
        return;
    }
    for (int d = tid; d < 256; d += kT) cnt[d] = 0;
    __syncthreads();
    for (int64_t i = tid; i < n; i += kT) atomicAdd(&cnt[(kin[i] >> shift) & 255u], 1u);
    __syncthreads();
    if (tid == 0) {
        uint32_t s = 0;
        for (int d = 0; d < 256; ++d) {
            const uint32_t c = cnt[d];
            cnt[d] = s;
            s += c;
        }
    }
    __syncthreads();
    const uint64_t below = (1ull << lane) - 1;
    for (int64_t b0 = 0; b0 < n; b0 += kT) {
        const int64_t i = b0 + tid;
        const bool valid = i < n;
        const uint32_t k = valid ? kin[i] : 0u;
        const uint32_t v = valid ? vin[i] : 0u;
        const uint32_t dig = (k >> shift) & 255u;
        // lanes of this wave holding the same digit
        uint64_t same = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const uint64_t bm = __ballot((dig >> bit) & 1u);
            same &= ((dig >> bit) & 1u) ? bm : ~bm;
        }
        const uint32_t rank_in_wave = (uint32_t)__popcll(same & below);
        for (int d = lane; d < 256; d += 64) wcnt[wave][d] = 0;
        __syncthreads();
        // the lowest lane of each digit group publishes the group's size
        if (valid && (same & below) == 0) wcnt[wave][dig] = (uint32_t)__popcll(same);
        __syncthreads();
        if (valid) {
            uint32_t off = cnt[dig] + rank_in_wave;
            for (int w = 0; w < wave; ++w) off += wcnt[w][dig];
            kout[off] = k;
            vout[off] = v;
        }
        __syncthreads();
        // advance the running digit offsets by this tile's counts
        for (int d = tid; d < 256; d += kT) {
            uint32_t s = 0;
            for (int w = 0; w < kW; ++w) s += wcnt[w][d];
            cnt[d] += s;
        }
        __syncthreads();
    }
}

// run starts over the sorted keys -> voxel ids per sorted position (inclusive scan - 1)
__global__ __launch_bounds__(kT) void voxel_runs_kernel(const uint32_t *__restrict__ skey, const uint32_t *__restrict__ sidx,
                                                        int64_t n, int32_t *__restrict__ vid, uint32_t *__restrict__ vstart,
                                                        uint32_t *__restrict__ meta)
{
    __shared__ uint32_t ws[kW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t base = 0;
    for (int64_t b0 = 0; b0 < n; b0 += kT) {
        const int64_t i = b0 + tid;
        const bool f = i < n && (i == 0 || skey[i] != skey[i - 1]);
        const uint64_t m = __ballot(f);
        const uint32_t inw = (uint32_t)__popcll(m & ((1ull << lane) - 1));
        if (lane == 0) ws[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t pre = 0, tot = 0;
        for (int w = 0; w < kW; ++w) {
            pre += w < wave ? ws[w] : 0;
            tot += ws[w];
        }
        if (i < n) {
            const uint32_t v = base + pre + inw + (f ? 1u : 0u) - 1u;  // id of my voxel
            vid[sidx[i]] = (int32_t)v;
            if (f) vstart[v] = (uint32_t)i;
        }
        base += tot;
        __syncthreads();
    }
    if (tid == 0) {
        meta[4] = base;
        vstart[base] = (uint32_t)n;
    }
}

__global__ void voxel_centroid_kernel(const float *__restrict__ xyz, const uint32_t *__restrict__ sidx,
                                      const uint32_t *__restrict__ vstart, const uint32_t *__restrict__ meta,
                                      float *__restrict__ cent, int32_t *__restrict__ counts)
{
    const uint32_t V = meta[4];
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < V; v += gridDim.x * blockDim.x) {
        const uint32_t a = vstart[v], b = vstart[v + 1];
        float s[3] = {0.f, 0.f, 0.f};
        for (uint32_t t = a; t < b; ++t) {
            const uint32_t i = sidx[t];
            for (int c = 0; c < 3; ++c) s[c] = __fadd_rn(s[c], xyz[3 * i + c]);
        }
        const float cnt = (float)(b - a);
        for (int c = 0; c < 3; ++c) cent[3 * v + c] = __fdiv_rn(s[c], cnt);
        counts[v] = (int32_t)(b - a);
    }
}

}  // namespace

LIDAR_EXPORT int lidar_voxel_downsample_f32(lidar_handle *h, const float *xyz, int64_t n, float voxel,
                                            int32_t *voxel_id, float *centroids, int32_t *counts,
                                            int64_t *nvox_host, void *stream)
{
    REQUIRE(h && xyz && voxel_id && centroids && counts && nvox_host, "lidar_voxel_downsample_f32: null pointer");
    REQUIRE(n >= 0 && n < 0x7fffffff, "lidar_voxel_downsample_f32: n out of range");
    REQUIRE(voxel > 0.0f, "lidar_voxel_downsample_f32: voxel size must be > 0");
    *nvox_host = 0;
    if (n == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    lidar::Carver cv;
    const uint64_t ok0 = cv.take<uint32_t>(n), ov0 = cv.take<uint32_t>(n);
    const uint64_t ok1 = cv.take<uint32_t>(n), ov1 = cv.take<uint32_t>(n);
    const uint64_t ost = cv.take<uint32_t>(n + 1), ometa = cv.take<uint32_t>(8);
    char *base = static_cast<char *>(lidar::workspace(h, cv.off));
    if (!base) return LIDAR_ENOMEM;
    auto U = [&](uint64_t o) { return reinterpret_cast<uint32_t *>(base + o); };
    uint32_t *meta = U(ometa);
    hipLaunchKernelGGL(voxel_keys_kernel, dim3(1), dim3(kT), 0, s, xyz, n, voxel, U(ok0), U(ov0), meta);
    uint32_t *kin = U(ok0), *vin = U(ov0), *kout = U(ok1), *vout = U(ov1);
    for (int shift = 0; shift < 32; shift += 8) {
        hipLaunchKernelGGL(radix_pass_kernel, dim3(1), dim3(kT), 0, s, kin, vin, kout, vout, n, shift, meta);
        std::swap(kin, kout);
        std::swap(vin, vout);
    }
    hipLaunchKernelGGL(voxel_runs_kernel, dim3(1), dim3(kT), 0, s, kin, vin, n, voxel_id, U(ost), meta);
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 2048));
    hipLaunchKernelGGL(voxel_centroid_kernel, dim3(g), dim3(256), 0, s, xyz, vin, U(ost), meta, centroids, counts);
    LAUNCH_CHECK();
    uint32_t *hm = static_cast<uint32_t *>(h->host_pinned);
    HIP_TRY(hipMemcpyAsync(hm, meta, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    REQUIRE(hm[0] != 0xffffffffu, "lidar_voxel_downsample_f32: voxel grid exceeds 2^32 keys (voxel too small)");
    *nvox_host = hm[4];
    return LIDAR_OK;
}
