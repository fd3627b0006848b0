// voxel_batch.hip — voxel downsampling of a batch of frames over the whole chip.
//
// Spec (voxel_grid.hpp): the voxel key of a point is calculate_grid_density's grid
// hash (utils/data_processing.py:305-319: np.arange edges over the frame's extent with the 2-cell
// margin, histogram2d's searchsorted-right binning with the last edge closed) per axis, key =
// (bx*ny + by)*nz + bz; voxels in ascending key order, voxel id = rank of the key (-1 for a point
// outside every bin), centroid = sequential fp32 sum of the voxel's points in point order / count.
// voxel.hip runs one frame in one workgroup; here every pass is spread over (tiles x frames)
// workgroups:
//
//   bbox (min, max)                                       grid (chunks, frames), atomics per frame
//   keys (u32) + indices per 4096-element tile, with the tile's histogram of radix digit 0 (LDS)
//          -> hist[frame][digit][tile]; a point outside every bin takes the key nx ny nz (one past the
//          last voxel), so every frame's key bits follow from its grid alone
//   LSD radix sort, 8-bit digits, only the passes a frame's key range needs (per-frame parity):
//     hist    (passes after the first) per 4096-element tile, LDS histogram
//     scatter per tile, stable: the tile's base per digit from the frame's tile histograms (its own
//             scan of them, frames of <= 32 tiles; a separate scan launch above), then 1024-element
//             sub-tiles ranked by wave ballots (8 per digit) and per-wave prefix counts in LDS, running
//             per-digit offsets
//   runs      per tile: run starts counted, then written from the frame's earlier tiles' counts
//             -> voxel id per point, run offsets, voxel count
//   centroid  one thread per voxel walks its run (index order: the sort is stable)
// 6 + 2 passes launches (round 3: 6 + 3 passes: the first histogram and every scan were launches of their own).
// (Counting the next pass's histogram with global atomics inside the scatter, and the centroids inside the
// runs kernel, were measured slower: 499 vs 238 us per 32-frame call.)
//
// Memory-side bytes per point: xyz read 3x (36 B: bbox, keys, centroids) + keys/indices (8 B written) + per radix pass
// 24 B (two reads, one write of 8 B) + runs 12 B + centroid gathers 12 B; the algorithmic floor is
// 12 B in + 4 B voxel id out (+16 B per voxel).  No host synchronisation: nvox[f] lands on the
// device (-1: the frame's extent is not finite, or its grid has 2^32 keys or more).
#include <algorithm>

#include "common.hpp"
#include "voxel_grid.hpp"

namespace {

constexpr int VT = 256;      // threads of the streaming kernels
constexpr int TILE = 4096;   // radix tile (elements per scatter workgroup)
constexpr int ST = 1024;     // scatter / runs workgroup threads
constexpr int SW = ST / 64;  // waves per scatter workgroup

// per-frame meta words: [0..2] / [3..5] monotone bits of the min / max point, [6] key bits (of the
// outside key), [7] unusable grid, [8] voxel count, [10] end of the last voxel's run, [11] the outside key
constexpr int MW = 16;
constexpr int kFuseScanTiles = 32;  // frames of at most this many tiles: the scatter scans the histograms itself

__device__ __forceinline__ uint32_t ord(float f)  // monotone float -> u32
{
    const uint32_t u = __float_as_uint(f);
    return u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
}
__device__ __forceinline__ float unord(uint32_t u)
{
    return __uint_as_float(u ^ (((u >> 31) - 1u) | 0x80000000u));
}

__global__ void vb_init_kernel(uint32_t *meta, int batch)
{
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= batch) return;
    uint32_t *m = meta + (int64_t)f * MW;
    for (int a = 0; a < 3; ++a) {
        m[a] = 0xffffffffu;  // >= ord(any float)
        m[3 + a] = 0u;        // <= ord(any float)
    }
    m[6] = m[7] = m[8] = m[9] = 0u;
}

// per-frame bbox in one pass: min and max as monotone bit patterns (atomics per wave)
__global__ __launch_bounds__(VT) void vb_bbox_kernel(const float *__restrict__ xyz, int64_t n, uint32_t *meta)
{
    const int f = blockIdx.y;
    const float *p = xyz + (int64_t)f * n * 3;
    uint32_t lo[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, hi[3] = {0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * VT + threadIdx.x; i < n; i += (int64_t)gridDim.x * VT)
        for (int a = 0; a < 3; ++a) {
            const uint32_t o = ord(p[3 * i + a]);
            lo[a] = min(lo[a], o);
            hi[a] = max(hi[a], o);
        }
    for (int a = 0; a < 3; ++a) {
        uint32_t v = lo[a], w = hi[a];
        for (int m = 32; m >= 1; m >>= 1) {
            v = min(v, (uint32_t)__shfl_xor((int)v, m, 64));
            w = max(w, (uint32_t)__shfl_xor((int)w, m, 64));
        }
        if ((threadIdx.x & 63) == 0) {
            atomicMin(meta + (int64_t)f * MW + a, v);
            atomicMax(meta + (int64_t)f * MW + 3 + a, w);
        }
    }
}

__device__ __forceinline__ lidar_vox::Grid frame_grid(const uint32_t *m, double voxel)
{
    const double lo[3] = {unord(m[0]), unord(m[1]), unord(m[2])}, hi[3] = {unord(m[3]), unord(m[4]), unord(m[5])};
    return lidar_vox::make_grid(lo, hi, voxel);
}

// grid (ntiles, frames): keys and indices of one 4096-element tile and the tile's histogram of digit 0
__global__ __launch_bounds__(ST) void vb_keys_kernel(const float *__restrict__ xyz, int64_t n, double voxel,
                                                     uint32_t *meta, uint32_t *__restrict__ key,
                                                     uint32_t *__restrict__ idx, uint32_t *__restrict__ hist,
                                                     int ntiles)
{
    const int f = blockIdx.y, t = blockIdx.x;
    const float *p = xyz + (int64_t)f * n * 3;
    uint32_t *m = meta + (int64_t)f * MW;
    const lidar_vox::Grid g = frame_grid(m, voxel);
    const uint32_t okey = g.ok ? (uint32_t)g.keys : 0u;
    const int bits = g.ok ? 32 - __clz((int)okey) : 0;  // okey = nx ny nz >= 1
    if (t == 0 && threadIdx.x == 0) {
        m[7] = g.ok ? 0u : 1u;
        m[6] = (uint32_t)bits;
        m[11] = okey;
        m[10] = (uint32_t)n;  // end of the last voxel's run, unless points lie outside every bin (runs kernel)
    }
    if (!g.ok) return;
    __shared__ uint32_t h[256];
    if (threadIdx.x < 256) h[threadIdx.x] = 0;
    __syncthreads();
    uint32_t *k = key + (int64_t)f * n;
    uint32_t *v = idx + (int64_t)f * n;
    const int64_t i0 = (int64_t)t * TILE, i1 = min<int64_t>(n, i0 + TILE);
    for (int64_t i = i0 + threadIdx.x; i < i1; i += ST) {
        uint32_t kk = lidar_vox::key(g, p[3 * i], p[3 * i + 1], p[3 * i + 2]);
        kk = kk == lidar_vox::kOutside ? okey : kk;  // sorts after every voxel's key
        k[i] = kk;
        v[i] = (uint32_t)i;
        atomicAdd(&h[kk & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 256) hist[((int64_t)f * 256 + threadIdx.x) * ntiles + t] = h[threadIdx.x];
}

// key bits of frame f, read after vb_keys_kernel (0 when the grid overflowed: nothing is sorted,
// the runs kernel reports -1)
__device__ __forceinline__ int frame_bits(const uint32_t *meta, int f)
{
    const uint32_t *m = meta + (int64_t)f * MW;
    return m[7] ? 0 : (int)m[6];
}

__global__ __launch_bounds__(VT) void vb_hist_kernel(const uint32_t *__restrict__ kin, int64_t n, int shift,
                                                     int ntiles, const uint32_t *meta, uint32_t *__restrict__ hist)
{
    const int f = blockIdx.y, t = blockIdx.x;
    if (frame_bits(meta, f) <= shift) return;  // this frame needs no pass at this digit
    __shared__ uint32_t h[256];
    for (int d = threadIdx.x; d < 256; d += VT) h[d] = 0;
    __syncthreads();
    const uint32_t *k = kin + (int64_t)f * n;
    const int64_t i0 = (int64_t)t * TILE, i1 = min<int64_t>(n, i0 + TILE);
    for (int64_t i = i0 + threadIdx.x; i < i1; i += VT) atomicAdd(&h[(k[i] >> shift) & 255u], 1u);
    __syncthreads();
    uint32_t *hf = hist + (int64_t)f * 256 * ntiles;
    for (int d = threadIdx.x; d < 256; d += VT) hf[(int64_t)d * ntiles + t] = h[d];
}

// per frame: exclusive scan of hist[f] in (digit, tile) order
__global__ __launch_bounds__(ST) void vb_scan_kernel(uint32_t *__restrict__ hist, int ntiles, int shift,
                                                     const uint32_t *meta)
{
    const int f = blockIdx.x;
    if (frame_bits(meta, f) <= shift) return;
    __shared__ uint32_t wsum[SW];
    __shared__ uint32_t carry;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t *hf = hist + (int64_t)f * 256 * ntiles;
    const int64_t total = (int64_t)256 * ntiles;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int64_t b0 = 0; b0 < total; b0 += ST) {
        const int64_t i = b0 + threadIdx.x;
        const uint32_t v = i < total ? hf[i] : 0u;
        uint32_t inc = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = (uint32_t)__shfl_up((int)inc, o, 64);
            if (lane >= o) inc += u;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        uint32_t pre = carry, tot = 0;
        for (int w = 0; w < SW; ++w) {
            pre += w < wave ? wsum[w] : 0u;
            tot += wsum[w];
        }
        if (i < total) hf[i] = pre + inc - v;
        __syncthreads();
        if (threadIdx.x == 0) carry += tot;
        __syncthreads();
    }
}

// FUSED: the tile's base per digit from the frame's raw tile histograms (its own scan: the digit's
// count in the frame's earlier tiles plus every smaller digit's total); else hist holds vb_scan_kernel's
// exclusive offsets
template <bool FUSED>
__global__ __launch_bounds__(ST) void vb_scatter_kernel(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                        uint32_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                        int64_t n, int shift, int ntiles, const uint32_t *meta,
                                                        const uint32_t *__restrict__ hist)
{
    const int f = blockIdx.y, t = blockIdx.x;
    if (frame_bits(meta, f) <= shift) return;
    __shared__ uint32_t off[256];      // running global offset per digit
    __shared__ uint32_t wcnt[SW][256]; // per-wave digit counts of the current sub-tile
    __shared__ uint32_t wtot[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t *hf = hist + (int64_t)f * 256 * ntiles;
    if constexpr (FUSED) {
        uint32_t tot = 0, pre = 0;  // thread d < 256: digit d's frame total and its count before tile t
        if (tid < 256)
            for (int u = 0; u < ntiles; ++u) {
                const uint32_t c = hf[(int64_t)tid * ntiles + u];
                tot += c;
                pre += u < t ? c : 0u;
            }
        uint32_t inc = tot;  // exclusive scan of the totals over the 256 digits (waves 0-3)
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = (uint32_t)__shfl_up((int)inc, o, 64);
            if (lane >= o) inc += u;
        }
        if (tid < 256 && lane == 63) wtot[wave] = inc;
        __syncthreads();
        if (tid < 256) {
            uint32_t base = inc - tot;
            for (int w = 0; w < wave; ++w) base += wtot[w];
            off[tid] = base + pre;
        }
    } else {
        for (int d = tid; d < 256; d += ST) off[d] = hf[(int64_t)d * ntiles + t];
    }
    const uint32_t *k = kin + (int64_t)f * n;
    const uint32_t *v = vin + (int64_t)f * n;
    uint32_t *ko = kout + (int64_t)f * n;
    uint32_t *vo = vout + (int64_t)f * n;
    const uint64_t below = (1ull << lane) - 1;
    const int64_t i0 = (int64_t)t * TILE, i1 = min<int64_t>(n, i0 + TILE);
    for (int64_t b0 = i0; b0 < i1; b0 += ST) {
        const int64_t i = b0 + tid;
        const bool valid = i < i1;
        const uint32_t kk = valid ? k[i] : 0u, vv = valid ? v[i] : 0u;
        const uint32_t dig = (kk >> shift) & 255u;
        uint64_t same = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const uint64_t bm = __ballot((dig >> bit) & 1u);
            same &= ((dig >> bit) & 1u) ? bm : ~bm;
        }
        for (int d = lane; d < 256; d += 64) wcnt[wave][d] = 0;
        __syncthreads();  // (also: off[] initialised / advanced)
        if (valid && (same & below) == 0) wcnt[wave][dig] = (uint32_t)__popcll(same);
        __syncthreads();
        if (valid) {
            uint32_t o = off[dig] + (uint32_t)__popcll(same & below);
            for (int w = 0; w < wave; ++w) o += wcnt[w][dig];
            ko[o] = kk;
            vo[o] = vv;
        }
        __syncthreads();
        for (int d = tid; d < 256; d += ST) {
            uint32_t s = 0;
            for (int w = 0; w < SW; ++w) s += wcnt[w][d];
            off[d] += s;
        }
        __syncthreads();  // wcnt is reset by the next sub-tile
    }
}

// run starts of the sorted keys, per 4096-element tile (chip-wide): count, then write with the
// tile's base from the counts of the frame's earlier tiles (<= n / 4096 loads)
__device__ __forceinline__ void sorted_bufs(const uint32_t *m, int f, int64_t n, const uint32_t *k0,
                                            const uint32_t *v0, const uint32_t *k1, const uint32_t *v1,
                                            const uint32_t *&sk, const uint32_t *&si)
{
    const int passes = ((int)m[6] + 7) / 8;  // the sorted data sits in buffer (passes run) % 2
    sk = (passes & 1 ? k1 : k0) + (int64_t)f * n;
    si = (passes & 1 ? v1 : v0) + (int64_t)f * n;
}

__global__ __launch_bounds__(ST) void vb_runs_count_kernel(const uint32_t *__restrict__ k0, const uint32_t *__restrict__ v0,
                                                           const uint32_t *__restrict__ k1, const uint32_t *__restrict__ v1,
                                                           int64_t n, int ntiles, const uint32_t *meta,
                                                           uint32_t *__restrict__ tilecnt)
{
    const int f = blockIdx.y, t = blockIdx.x;
    const uint32_t *m = meta + (int64_t)f * MW;
    if (m[7]) return;
    const uint32_t *sk, *si;
    sorted_bufs(m, f, n, k0, v0, k1, v1, sk, si);
    __shared__ uint32_t ws[SW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t i0 = (int64_t)t * TILE, i1 = min<int64_t>(n, i0 + TILE);
    const uint32_t okey = m[11];
    uint32_t c = 0;
    for (int64_t i = i0 + tid; i < i1; i += ST)
        c += (sk[i] != okey && (i == 0 || sk[i] != sk[i - 1])) ? 1u : 0u;
    for (int o = 32; o >= 1; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o, 64);
    if (lane == 0) ws[wave] = c;
    __syncthreads();
    if (tid == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < SW; ++w) tot += ws[w];
        tilecnt[(int64_t)f * ntiles + t] = tot;
    }
}

__global__ __launch_bounds__(ST) void vb_runs_write_kernel(const uint32_t *__restrict__ k0, const uint32_t *__restrict__ v0,
                                                           const uint32_t *__restrict__ k1, const uint32_t *__restrict__ v1,
                                                           int64_t n, int ntiles, uint32_t *meta,
                                                           const uint32_t *__restrict__ tilecnt,
                                                           int32_t *__restrict__ vid, uint32_t *__restrict__ vstart,
                                                           int32_t *__restrict__ nvox)
{
    const int f = blockIdx.y, t = blockIdx.x;
    uint32_t *m = meta + (int64_t)f * MW;
    if (m[7]) {
        if (t == 0 && threadIdx.x == 0) nvox[f] = -1;
        return;
    }
    const uint32_t *sk, *si;
    sorted_bufs(m, f, n, k0, v0, k1, v1, sk, si);
    int32_t *vf = vid + (int64_t)f * n;
    uint32_t *vs = vstart + (int64_t)f * (n + 1);
    __shared__ uint32_t ws[SW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t okey = m[11];
    uint32_t base = 0;
    for (int u = 0; u < t; ++u) base += tilecnt[(int64_t)f * ntiles + u];
    const int64_t i0 = (int64_t)t * TILE, i1 = min<int64_t>(n, i0 + TILE);
    for (int64_t b0 = i0; b0 < i1; b0 += ST) {
        const int64_t i = b0 + tid;
        const bool in = i < i1 && sk[i] != okey;
        const bool st = in && (i == 0 || sk[i] != sk[i - 1]);
        const uint64_t mk = __ballot(st);
        const uint32_t inw = (uint32_t)__popcll(mk & ((1ull << lane) - 1));
        if (lane == 0) ws[wave] = (uint32_t)__popcll(mk);
        __syncthreads();
        uint32_t pre = 0, tot = 0;
        for (int w = 0; w < SW; ++w) {
            pre += w < wave ? ws[w] : 0u;
            tot += ws[w];
        }
        if (in) {
            const uint32_t r = base + pre + inw + (st ? 1u : 0u) - 1u;  // my voxel's rank
            vf[si[i]] = (int32_t)r;
            if (st) vs[r] = (uint32_t)i;
        } else if (i < i1) {
            vf[si[i]] = -1;  // outside every bin (sorted after the last voxel)
            if (i == 0 || sk[i - 1] != okey) m[10] = (uint32_t)i;  // the last run's end
        }
        base += tot;
        __syncthreads();
    }
    if (t == ntiles - 1 && tid == 0) {
        m[8] = base;
        nvox[f] = (int32_t)base;
    }
}

__global__ __launch_bounds__(VT) void vb_centroid_kernel(const float *__restrict__ xyz, int64_t n,
                                                         const uint32_t *__restrict__ v0, const uint32_t *__restrict__ v1,
                                                         const uint32_t *meta, const uint32_t *__restrict__ vstart,
                                                         float *__restrict__ cent, int32_t *__restrict__ counts)
{
    const int f = blockIdx.y;
    const uint32_t *m = meta + (int64_t)f * MW;
    if (m[7]) return;
    const int passes = ((int)m[6] + 7) / 8;  // the sorted indices sit in buffer (passes run) % 2
    const uint32_t *si = (passes & 1 ? v1 : v0) + (int64_t)f * n;
    const uint32_t *vs = vstart + (int64_t)f * (n + 1);
    const float *p = xyz + (int64_t)f * n * 3;
    const uint32_t V = m[8];
    for (uint32_t v = blockIdx.x * VT + threadIdx.x; v < V; v += gridDim.x * VT) {
        const uint32_t a = vs[v], b = v + 1 < V ? vs[v + 1] : m[10];
        float s[3] = {0.f, 0.f, 0.f};
        for (uint32_t t = a; t < b; ++t) {
            const uint32_t i = si[t];
            for (int c = 0; c < 3; ++c) s[c] = __fadd_rn(s[c], p[3 * i + c]);
        }
        const float cnt = (float)(b - a);
        float *o = cent + ((int64_t)f * n + v) * 3;
        for (int c = 0; c < 3; ++c) o[c] = __fdiv_rn(s[c], cnt);
        counts[(int64_t)f * n + v] = (int32_t)(b - a);
    }
}

}  // namespace

// workspace bytes of lidar_voxel_downsample_batch_f32 for (batch, n)
LIDAR_EXPORT uint64_t lidar_voxel_batch_workspace_bytes(int64_t batch, int64_t n)
{
    const int64_t ntiles = (n + TILE - 1) / TILE;
    return (uint64_t)batch * ((uint64_t)n * 16 + (uint64_t)(n + 1) * 4 + (uint64_t)257 * ntiles * 4 + MW * 4) + 2048;
}

// Voxel downsampling of `batch` frames of n points (xyz (batch, n, 3) fp32), all on the device:
// voxel_id (batch, n) int32, centroids (batch, n, 3) and counts (batch, n) with the first nvox[f]
// rows of frame f valid, nvox (batch,) int32 (-1: the frame's extent is not finite or its voxel grid
// has 2^32 keys or more; voxel_id -1: a point outside every bin).
// Same results as lidar_voxel_downsample_f32 per frame.
LIDAR_EXPORT int lidar_voxel_downsample_batch_f32(lidar_handle *h, const float *xyz, int64_t batch, int64_t n,
                                                  double voxel, int32_t *voxel_id, float *centroids, int32_t *counts,
                                                  int32_t *nvox, void *stream)
{
    REQUIRE(h && xyz && voxel_id && centroids && counts && nvox, "lidar_voxel_downsample_batch_f32: null pointer");
    REQUIRE(batch >= 0 && batch <= 65535 && n >= 1 && n < 0x7fffffff,
            "lidar_voxel_downsample_batch_f32: batch in [0, 65535], n >= 1");
    REQUIRE(voxel > 0.0 && voxel < INFINITY, "lidar_voxel_downsample_batch_f32: voxel size must be finite and > 0");
    if (batch == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int ntiles = (int)((n + TILE - 1) / TILE);
    lidar::Carver cv;
    const uint64_t ok0 = cv.take<uint32_t>(batch * n), ov0 = cv.take<uint32_t>(batch * n);
    const uint64_t ok1 = cv.take<uint32_t>(batch * n), ov1 = cv.take<uint32_t>(batch * n);
    const uint64_t ost = cv.take<uint32_t>(batch * (n + 1));
    const uint64_t oh = cv.take<uint32_t>(batch * 256 * (int64_t)ntiles);
    const uint64_t om = cv.take<uint32_t>(batch * MW);
    const uint64_t otc = cv.take<uint32_t>(batch * (int64_t)ntiles);
    char *base = static_cast<char *>(lidar::workspace(h, cv.off));
    if (!base) return LIDAR_ENOMEM;
    auto U = [&](uint64_t o) { return reinterpret_cast<uint32_t *>(base + o); };
    uint32_t *meta = U(om), *hist = U(oh);
    const unsigned chunks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + VT * 8 - 1) / (VT * 8), 256));
    const dim3 sg(chunks, (unsigned)batch);
    hipLaunchKernelGGL(vb_init_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, s, meta, (int)batch);
    hipLaunchKernelGGL(vb_bbox_kernel, sg, dim3(VT), 0, s, xyz, n, meta);
    const dim3 tg((unsigned)ntiles, (unsigned)batch);
    // keys + the histogram of digit 0
    hipLaunchKernelGGL(vb_keys_kernel, tg, dim3(ST), 0, s, xyz, n, voxel, meta, U(ok0), U(ov0), hist, ntiles);
    uint32_t *kin = U(ok0), *vin = U(ov0), *kout = U(ok1), *vout = U(ov1);
    const bool fused = ntiles <= kFuseScanTiles;
    for (int shift = 0; shift < 32; shift += 8) {  // frames past their key bits skip (per-frame parity)
        if (shift > 0) hipLaunchKernelGGL(vb_hist_kernel, tg, dim3(VT), 0, s, kin, n, shift, ntiles, meta, hist);
        if (fused) {
            hipLaunchKernelGGL(vb_scatter_kernel<true>, tg, dim3(ST), 0, s, kin, vin, kout, vout, n, shift, ntiles, meta,
                               hist);
        } else {
            hipLaunchKernelGGL(vb_scan_kernel, dim3((unsigned)batch), dim3(ST), 0, s, hist, ntiles, shift, meta);
            hipLaunchKernelGGL(vb_scatter_kernel<false>, tg, dim3(ST), 0, s, kin, vin, kout, vout, n, shift, ntiles,
                               meta, hist);
        }
        std::swap(kin, kout);
        std::swap(vin, vout);
    }
    hipLaunchKernelGGL(vb_runs_count_kernel, tg, dim3(ST), 0, s, U(ok0), U(ov0), U(ok1), U(ov1), n, ntiles, meta,
                       U(otc));
    hipLaunchKernelGGL(vb_runs_write_kernel, tg, dim3(ST), 0, s, U(ok0), U(ov0), U(ok1), U(ov1), n, ntiles, meta,
                       U(otc), voxel_id, U(ost), nvox);
    // one thread per (possible) voxel: the gathers of a voxel's points are a dependent chain
    const dim3 cg((unsigned)((n + VT - 1) / VT), (unsigned)batch);
    hipLaunchKernelGGL(vb_centroid_kernel, cg, dim3(VT), 0, s, xyz, n, U(ov0), U(ov1), meta, U(ost), centroids,
                       counts);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
