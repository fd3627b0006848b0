// voxel.hip — voxel downsampling on gfx950 (north_star "voxel hashing").
//
// Spec (voxel_grid.hpp, oracle tier_n.voxel_downsample): per axis the bins of
// calculate_grid_density (utils/data_processing.py:305-319: np.arange edges over the frame's
// extent with the 2-cell margin, histogram2d's searchsorted-right rule, last edge closed), key =
// (bx*ny + by)*nz + bz, voxels in ascending key order, per-point voxel id = rank of its key (-1
// outside every bin), centroid = sequential fp32 sum of the voxel's points in point order / count.
//
// Pipeline (one frame): bbox -> keys -> stable LSD radix sort of (key, index) in one
// 1024-thread workgroup (8-bit digits; the stable in-wave rank comes from 8 ballots per
// digit: lanes with an equal digit, below me) -> run starts -> scan -> per-voxel
// sequential sums (one lane per voxel walks its run, which is in index order because
// the sort is stable).  HBM-bound integer work: no float reductions besides the
// centroid sums, whose order is part of the spec.
#include "common.hpp"
#include "voxel_grid.hpp"

namespace {

constexpr int kT = 1024;
constexpr int kW = kT / 64;

__global__ __launch_bounds__(kT) void voxel_keys_kernel(const float *__restrict__ xyz, int64_t n, double voxel,
                                                        uint32_t *__restrict__ key, uint32_t *__restrict__ idx,
                                                        uint32_t *__restrict__ meta)
{
    __shared__ float red[6][kW];
    __shared__ int anyout;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // the extent: numpy's min / max (a NaN anywhere makes it NaN: no finite grid)
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    bool nan = false;
    for (int64_t i = tid; i < n; i += kT)
        for (int a = 0; a < 3; ++a) {
            const float v = xyz[3 * i + a];
            nan |= v != v;
            lo[a] = fminf(lo[a], v);
            hi[a] = fmaxf(hi[a], v);
        }
    if (tid == 0) anyout = 0;
    for (int a = 0; a < 3; ++a) {
        const float v = lidar::wave_min_f(lo[a]), w = -lidar::wave_min_f(-hi[a]);
        if (lane == 0) {
            red[a][wave] = v;
            red[3 + a][wave] = w;
        }
    }
    if (__ballot(nan) && lane == 0) red[0][wave] = NAN;
    __syncthreads();
    double dlo[3], dhi[3];
    for (int a = 0; a < 3; ++a) {
        float v = red[a][0], w = red[3 + a][0];
        for (int q = 1; q < kW; ++q) {
            v = (v != v || red[a][q] != red[a][q]) ? NAN : fminf(v, red[a][q]);
            w = fmaxf(w, red[3 + a][q]);
        }
        dlo[a] = (double)v;
        dhi[a] = (double)w;
    }
    const lidar_vox::Grid g = lidar_vox::make_grid(dlo, dhi, voxel);
    if (!g.ok) {
        if (tid == 0) meta[0] = 0xffffffffu;
        return;
    }
    bool outside = false;
    for (int64_t i = tid; i < n; i += kT) {
        const uint32_t k = lidar_vox::key(g, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
        outside |= k == lidar_vox::kOutside;
        key[i] = k;
        idx[i] = (uint32_t)i;
    }
    if (__ballot(outside) && lane == 0) atomicOr(&anyout, 1);
    __syncthreads();
    if (tid == 0) {
        // keys span [0, g.keys) (plus kOutside): the radix passes above their bits are skipped
        meta[0] = anyout ? 0xfffffffeu : (uint32_t)g.keys;
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
    if (meta[0] == 0xffffffffu) return;  // no usable grid: nothing was keyed
    // skip passes above the key range (keys < meta[0]; 0xfffffffe: keys up to kOutside)
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
    __shared__ uint32_t end;  // end of the last voxel's run: n, or the first point outside every bin
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (meta[0] == 0xffffffffu) return;
    if (tid == 0) end = (uint32_t)n;
    uint32_t base = 0;
    for (int64_t b0 = 0; b0 < n; b0 += kT) {
        const int64_t i = b0 + tid;
        const bool in = i < n && skey[i] != lidar_vox::kOutside;
        const bool f = in && (i == 0 || skey[i] != skey[i - 1]);
        const uint64_t m = __ballot(f);
        const uint32_t inw = (uint32_t)__popcll(m & ((1ull << lane) - 1));
        if (lane == 0) ws[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t pre = 0, tot = 0;
        for (int w = 0; w < kW; ++w) {
            pre += w < wave ? ws[w] : 0;
            tot += ws[w];
        }
        if (in) {
            const uint32_t v = base + pre + inw + (f ? 1u : 0u) - 1u;  // id of my voxel
            vid[sidx[i]] = (int32_t)v;
            if (f) vstart[v] = (uint32_t)i;
        } else if (i < n) {
            vid[sidx[i]] = -1;  // outside every bin (sorted after the last voxel)
            if (i == 0 || skey[i - 1] != lidar_vox::kOutside) end = (uint32_t)i;
        }
        base += tot;
        __syncthreads();
    }
    __syncthreads();
    if (tid == 0) {
        meta[4] = base;
        vstart[base] = end;
    }
}

__global__ void voxel_centroid_kernel(const float *__restrict__ xyz, const uint32_t *__restrict__ sidx,
                                      const uint32_t *__restrict__ vstart, const uint32_t *__restrict__ meta,
                                      float *__restrict__ cent, int32_t *__restrict__ counts)
{
    if (meta[0] == 0xffffffffu) return;
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

LIDAR_EXPORT int lidar_voxel_downsample_f32(lidar_handle *h, const float *xyz, int64_t n, double voxel,
                                            int32_t *voxel_id, float *centroids, int32_t *counts,
                                            int64_t *nvox_host, void *stream)
{
    REQUIRE(h && xyz && voxel_id && centroids && counts && nvox_host, "lidar_voxel_downsample_f32: null pointer");
    REQUIRE(n >= 0 && n < 0x7fffffff, "lidar_voxel_downsample_f32: n out of range");
    REQUIRE(voxel > 0.0 && voxel < INFINITY, "lidar_voxel_downsample_f32: voxel size must be finite and > 0");
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
    REQUIRE(hm[0] != 0xffffffffu,
            "lidar_voxel_downsample_f32: the extent is not finite or the voxel grid has 2^32 keys or more");
    *nvox_host = hm[4];
    return LIDAR_OK;
}
