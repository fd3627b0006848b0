// voxel_batch.hip — voxel downsampling of a batch of frames over the whole chip.
//
// Spec (voxel_grid.hpp): the voxel key of a point is calculate_grid_density's grid
// hash (utils/data_processing.py:305-319: np.arange edges over the frame's extent with the 2-cell
// margin, histogram2d's searchsorted-right binning with the last edge closed) per axis, key =
// (bx*ny + by)*nz + bz; voxels in ascending key order, voxel id = rank of the key (-1 for a point
// outside every bin), centroid = sequential fp32 sum of the voxel's points in point order / count.
//
// Round 5: a two-level sort in two launches (round 4: an 8-bit LSD radix sort over global memory,
// 13 launches and ~284 B of memory traffic per point):
//
//   keys     grid (8192-point tiles, frames; a frame's tiles on one XCD, dispatched together): each
//            tile loads its points once, publishes its extent as self-tagged 8-byte granules and
//            polls its frame's other tiles' (an in-launch hand-off instead of a bbox launch), builds
//            the frame's grid (float64, every workgroup alike), bins every point in float against
//            per-axis LDS tables of the float64 edges' float thresholds (float64 beyond 8192 edges per
//            axis; a point outside every bin takes nx ny nz, one past the last voxel), and publishes
//            its histogram over 4096 coarse bins (key >> hs, the top 12 bits of the range) as tagged
//            granules too; then, from the frame's histograms (polled), the exclusive scan over the
//            coarse bins plus the counts of the tiles before it, and it scatters its (key, index)
//            pairs from registers to their coarse bins (LDS atomics: order inside a bin is free, the
//            buckets sort by (key, index) anyway); tile 0 also writes the bucket table (bucket b = the
//            coarse bins whose start s has min(s NB / n, NB - 1) = b, ~2 048 points uniform).
//            Frames of more than 16 tiles (more than an XCD co-schedules with margin) split this into
//            an extent launch, a keys launch that writes the keys, and a scatter launch.  The granules
//            live in the handle's tag block: every tag there is an earlier call's epoch (no memset).
//   bucket   grid (buckets, frames; 4 workgroups per CU, the bench shape's 1 024 buckets in one round):
//            each bucket loads its pairs and counting-sorts them in LDS over its own key range — one
//            counter per key, whose exclusive scan of (count | occupied << 16) also gives every key its
//            voxel rank; or, for a sparse grid (a range past 4096 keys), counters over the keys' high
//            bits with each run ordered by (key low bits, index) words and the voxel ranks from a scan
//            of first-point flags — equal-key runs ranked by index in parallel; runs past 128: bitonic
//            in LDS, or a stable LSD radix in global memory above 2048 pairs.  Its voxel count goes out
//            at once for the decoupled look-back (every wait is on a lower workgroup index, i.e. one
//            dispatched earlier), then every point's voxel id from registers and, one thread per voxel
//            summing its points' xyz (gathered) in index order, the centroids and counts.
//
// Memory-side bytes per point: xyz 12 (keys) + pair 8 + 8 + id 4 + the xyz gather 12
// (+16 per voxel out; 62.9 measured by PMC at the bench shape); no host synchronisation: nvox[f] lands on the device (-1: the frame's extent is
// not finite, or its grid has 2^32 - 1 keys or more).
#include <algorithm>

#include "common.hpp"
#include "voxel_grid.hpp"

namespace {

constexpr int KT = 1024;           // keys / scatter threads
constexpr int TILE = 8192;         // points per keys / scatter workgroup (one round of the chip at B = 32)
constexpr int PPT = TILE / KT;     // points per keys / scatter thread
constexpr int kFuseTiles = 16;     // frames of up to this many tiles take their extent inside the keys launch
constexpr int HB = 12;             // coarse-bin bits of the key range
constexpr int NBIN = 1 << HB;      // coarse bins per frame
constexpr int BPT = NBIN / KT;     // coarse bins per scatter thread (its scan)
constexpr int UT = 512;            // bucket threads
constexpr int CAP = 2560;          // pairs a bucket sorts in LDS
constexpr int BITONIC_P = 2048;    // the LDS bitonic fallback's array (a power of two; larger buckets
                                   // sort in global memory: at P = 4 096 the LDS network is the slower)
constexpr int KMAX = 4096;         // local key range of the LDS counting sort
constexpr int SEGMAX = 128;        // longest equal-key run the counting sort orders by index itself
constexpr int BUCKET = 2048;       // target points per bucket (32 x 65 536 points: 1 024 buckets, one round of
                                   // four workgroups per CU)
constexpr int MW = 8;              // meta words per frame: [0] grid ok, [1] outside key, [2] hs, [3] hung tag
                                   // (keys / scatter), [4] the bucket launch's failure tag, [5] its nvox code
static_assert(NBIN % KT == 0 && NBIN % UT == 0, "bins per thread");

__device__ __forceinline__ uint32_t ord(float f)  // monotone float -> u32
{
    const uint32_t u = __float_as_uint(f);
    return u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
}
__device__ __forceinline__ float unord(uint32_t u)
{
    return __uint_as_float(u ^ (((u >> 31) - 1u) | 0x80000000u));
}

struct Ws {  // per-batch workspace, every array frame-major
    unsigned long long *gran;  // [F][T][6] the tiles' extents: epoch << 32 | monotone bits (self-tagged granules)
    uint32_t *meta;    // [F][MW] ([3]: the call's epoch when a hand-off timed out)
    uint32_t *key;     // [F][n]
    unsigned long long *hgran;  // [F][T][NBIN / 2] tile histograms: epoch << 32 | count(2g + 1) << 16 | count(2g)
    uint32_t *bstart;  // [F][NB + 1] the buckets' first pairs (bstart[NB] = n)
    uint64_t *pairs;   // [F][n] (key << 32 | index), coarse-bin order
    uint64_t *scratch; // [F][n] the global sort's other buffer
    uint64_t *flags;   // [F][NB] look-back words: status << 32 | count
    float *cent_diag;  // VX_DIAG_KEYS builds only: the centroids output, whose tail rows take the stamps
};

__device__ __forceinline__ int64_t n_buckets(int64_t n) { return (n + BUCKET - 1) / BUCKET; }

// (frame, part) of a 1-D grid of `parts` workgroups per frame.  XCD-affine (batch >= 8): workgroup L
// runs on XCD L % 8, which takes frames L % 8, L % 8 + 8, ... and their parts in order, so a frame's
// scattered writes and gathers stay in one L2 and its part p - 1 is dispatched before part p (the
// bucket look-back waits only on that); fewer frames: plain frame-major order.  false: padding.
__device__ __forceinline__ bool frame_part(int64_t batch, int64_t parts, int64_t &f, int64_t &p)
{
    const int64_t L = blockIdx.x;
    if (batch >= 8) {
        const int64_t x = L & 7, j = L >> 3;
        f = x + 8 * (j / parts);
        p = j % parts;
    } else {
        f = L / parts;
        p = L % parts;
    }
    return f < batch;
}
__host__ __forceinline__ unsigned frame_grid(int64_t batch, int64_t parts)
{
    return (unsigned)(batch >= 8 ? 8 * ((batch + 7) / 8) * parts : batch * parts);
}

// block-wide exclusive scan of one value per thread (T threads); returns the exclusive prefix and
// the total through *tot.  Uses red[T / 64]; starts and ends with a barrier.
// wave64 inclusive prefix sum by DPP: row_shr 1, 2, 4, 8 inside each 16-lane row (lanes without a
// source add 0), then row_bcast 15 / 31 carry the rows' totals (no LDS traffic, unlike __shfl_up)
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return v;
}

template <int T>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *red, uint32_t *tot)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan_u32(v);
    __syncthreads();  // red[] free (a previous scan's readers are done)
    if (lane == 63) red[wave] = inc;
    __syncthreads();
    uint32_t pre = 0, all = 0;
#pragma unroll
    for (int w = 0; w < T / 64; ++w) {
        pre += w < wave ? red[w] : 0u;
        all += red[w];
    }
    *tot = all;
    return pre + inc - v;
}

// ------------------------------------------------------------------------------------- scatter
// tile t of frame f: sums the frame's tile histograms (polling their granules until every tag is this
// call's), the exclusive scan over the coarse bins plus the counts of the tiles before it, the bucket
// table (tile 0), then its (key, index) pairs to their coarse bins.  kv: the tile's keys (thread tid:
// points t TILE + j KT + tid); off: NBIN words of LDS; red: KT / 64 words.
#ifdef VX_DIAG_KEYS
#define VX_KSTAMP(k)                                                                  \
    do {                                                                              \
        uint64_t t_;                                                                  \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");  \
        kts[k] = t_;                                                                  \
    } while (0)
#else
#define VX_KSTAMP(k)
#endif
__device__ __forceinline__ void scatter_tile(const uint32_t (&kv)[PPT], int64_t f, int64_t t, int64_t n, int ntiles,
                                             int hs, uint32_t epoch, const Ws &w, uint32_t *off, uint32_t *red,
                                             int64_t batch, uint64_t *kts = nullptr)
{
    const int tid = threadIdx.x;
    // coarse bins BPT tid .. BPT tid + BPT - 1: frame totals and the counts of the tiles before this one
    uint32_t tot[BPT], pre[BPT], sum = 0;
#pragma unroll
    for (int j = 0; j < BPT; ++j) tot[j] = pre[j] = 0;
    const unsigned long long *hg = w.hgran + (int64_t)f * ntiles * (NBIN / 2) + (BPT / 2) * tid;
    bool hung = false;
    // four tiles' granules per pass, every load in flight together (one round trip per pass, not per tile)
    constexpr int UCH = 4;
    for (int u0 = 0; u0 < ntiles; u0 += UCH) {
        unsigned long long g2[UCH][BPT / 2];
        uint32_t spins = 0;
        while (true) {  // bounded: a tile that never publishes is a bug, reported as nvox -2
            bool ready = true;
#pragma unroll
            for (int uu = 0; uu < UCH; ++uu)
#pragma unroll
                for (int e = 0; e < BPT / 2; ++e) {
                    g2[uu][e] = u0 + uu < ntiles ? __hip_atomic_load(&hg[(int64_t)(u0 + uu) * (NBIN / 2) + e],
                                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                 : ((unsigned long long)epoch << 32);
                }
#pragma unroll
            for (int uu = 0; uu < UCH; ++uu)
#pragma unroll
                for (int e = 0; e < BPT / 2; ++e) ready = ready && (uint32_t)(g2[uu][e] >> 32) == epoch;
            if (ready) break;
            if (++spins == (1u << 22)) {
                hung = true;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
#pragma unroll
        for (int uu = 0; uu < UCH; ++uu)
#pragma unroll
            for (int j = 0; j < BPT; ++j) {
                const uint32_t c = (uint32_t)(g2[uu][j >> 1] >> (16 * (j & 1))) & 0xffffu;  // 0 past ntiles
                tot[j] += c;
                pre[j] += u0 + uu < t ? c : 0u;
            }
    }
    if (hung) w.meta[f * MW + 3] = epoch;
    VX_KSTAMP(6);
#pragma unroll
    for (int j = 0; j < BPT; ++j) sum += tot[j];
    uint32_t all;
    uint32_t ex = block_excl_scan<KT>(sum, red, &all);
    uint32_t bsv[BPT];  // the frame-level start of each of this thread's bins
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
        bsv[j] = ex;
        off[BPT * tid + j] = ex + pre[j];
        ex += tot[j];
    }
    __syncthreads();
    if (t == 0) {
        // the bucket table: bucket b = the bins whose start s has bk(s) = min(s nb / n, nb - 1) = b, so
        // its first pair is the start of the first bin with bk >= b; buckets past the last bin's bk start
        // at n (empty), and bstart[nb] = n.  The previous bin's start: off[] still holds the frame-level
        // starts in this workgroup (t = 0: no earlier tiles), read before the barrier below lets the
        // scatter's atomics move them.
        const int64_t nb = n_buckets(n);
        const float inv = (float)nb / (float)n;
        auto bk = [&](uint32_t st) { return min<int64_t>((int64_t)((float)st * inv), nb - 1); };
        uint32_t *bst = w.bstart + (int64_t)f * (nb + 1);
        int64_t prev = tid == 0 ? -1 : bk(off[BPT * tid - 1]);
#pragma unroll
        for (int j = 0; j < BPT; ++j) {
            const int64_t cur = bk(bsv[j]);
            for (int64_t q = prev + 1; q <= cur; ++q) bst[q] = bsv[j];
            prev = cur;
        }
        if (tid == KT - 1)
            for (int64_t q = prev + 1; q <= nb; ++q) bst[q] = (uint32_t)n;
        __syncthreads();  // (uniform: t is the workgroup's)
    }
    VX_KSTAMP(8);
    VX_KSTAMP(7);
    uint64_t *pr = w.pairs + (int64_t)f * n;
    (void)kts;
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const int64_t i = (int64_t)t * TILE + j * KT + tid;
        if (i < n) {
            const uint32_t pos = atomicAdd(&off[kv[j] >> hs], 1u);
            if (pos < (uint64_t)n) pr[pos] = ((uint64_t)kv[j] << 32) | (uint32_t)i;  // (hung: counts unknown)
        }
    }
}

// ---------------------------------------------------------------------------------------- keys
constexpr int ETAB = lidar_vox::kTabEdges;  // edges per axis of the keys launch's LDS tables

using lidar_vox::bin_of_c;
using lidar_vox::bin_tab_c;
using lidar_vox::bin_tab_search;
using lidar_vox::ru_float;

// the tile's extent (min / max of ord() over its points in q) as six {epoch, value} granules gr[t * 6 ..]
template <typename Q>
__device__ __forceinline__ void publish_extent(const Q &q, int64_t n, int64_t t, unsigned long long *gr,
                                               uint32_t epoch, uint32_t (*red6)[6])
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t lo3[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, hi3[3] = {0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < PPT; ++j)
        if ((int64_t)t * TILE + j * KT + tid < n)
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                lo3[a] = min(lo3[a], ord(q[j][a]));
                hi3[a] = max(hi3[a], ord(q[j][a]));
            }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        lo3[a] = lidar::wave_min_u32_dpp(lo3[a]);
        hi3[a] = ~lidar::wave_min_u32_dpp(~hi3[a]);
    }
    if (lane == 0)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            red6[wave][a] = lo3[a];
            red6[wave][3 + a] = hi3[a];
        }
    __syncthreads();
    if (tid < 6) {
        uint32_t v = red6[0][tid];
        for (int q2 = 1; q2 < KT / 64; ++q2) v = tid < 3 ? min(v, red6[q2][tid]) : max(v, red6[q2][tid]);
        __hip_atomic_store(&gr[t * 6 + tid], ((unsigned long long)epoch << 32) | v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
}

// the extents of frames with more tiles than an XCD holds workgroups (the keys launch's poll then finds
// every granule already written): one launch more and the points read twice
__global__ __launch_bounds__(KT) void vx_extent_kernel(const float *__restrict__ xyz, int64_t n, Ws w, int ntiles,
                                                       int64_t batch, uint32_t epoch)
{
    int64_t f, t;
    if (!frame_part(batch, ntiles, f, t)) return;
    __shared__ uint32_t red6[KT / 64][6];
    const float *p = xyz + (int64_t)f * n * 3;
    float q[PPT][3];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const int64_t i = (int64_t)t * TILE + j * KT + threadIdx.x;
#pragma unroll
        for (int a = 0; a < 3; ++a) q[j][a] = i < n ? p[3 * i + a] : 0.f;
    }
    publish_extent(q, n, t, w.gran + (int64_t)f * ntiles * 6, epoch, red6);
}


template <bool FUSED>
__global__ __launch_bounds__(KT) void vx_keys_kernel(const float *__restrict__ xyz, int64_t n, double voxel, Ws w,
                                                     int ntiles, int64_t batch, uint32_t epoch, int64_t nb)
{
    int64_t f, t;
    if (!frame_part(batch, ntiles, f, t)) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef VX_DIAG_KEYS
    uint64_t kts[12] = {};
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(kts[10])::"memory");
#else
    uint64_t *kts = nullptr;
#endif
    VX_KSTAMP(0);
    __shared__ uint32_t ext[6];
    __shared__ uint32_t red6[KT / 64][6];
    __shared__ uint32_t hist[NBIN];
    __shared__ float etab[3][ETAB + 2];  // -inf, the thresholds, +inf
    const float *p = xyz + (int64_t)f * n * 3;
    float q[PPT][3];  // the tile's points, loaded once: its extent, then its keys
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const int64_t i = (int64_t)t * TILE + j * KT + tid;
#pragma unroll
        for (int a = 0; a < 3; ++a) q[j][a] = i < n ? p[3 * i + a] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < BPT; ++j) hist[tid + j * KT] = 0;
    if (t == 0)  // the bucket launch's look-back words start at "nothing published"
        for (int64_t b = tid; b < nb; b += KT) w.flags[(int64_t)f * nb + b] = 0ull;
    {
        // the tile's extent (monotone bits: min / max of ord()), then the frame's from every tile's
        // granules: {epoch, value} in one 8-byte agent-scope store each, polled until every tag is this
        // call's (self-contained: no fence; MI355X_MICROARCH.md R2).  A tile waits only on tiles of its
        // frame, which frame_part dispatches together, at most kFuseTiles of them (an XCD holds 32
        // workgroups of this launch; larger frames run vx_extent_kernel first); the spin is bounded (a
        // frame whose tiles never all arrive sets the hung tag meta[3]: nvox -2).
        unsigned long long *gr = w.gran + (int64_t)f * ntiles * 6;
        publish_extent(q, n, t, gr, epoch, red6);
        VX_KSTAMP(1);
        if (wave == 0) {
            uint32_t m[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
            bool ok = true;
            for (int64_t c0 = 0; c0 < (int64_t)ntiles * 6; c0 += 60) {  // 10 tiles per pass, lane l: word l % 6
                const int64_t c = c0 + lane;
                const bool mine = lane < 60 && c < (int64_t)ntiles * 6;
                unsigned long long v = 0;
                uint32_t spins = 0;
                while (true) {
                    v = mine ? __hip_atomic_load(&gr[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                    const bool ready = !mine || (uint32_t)(v >> 32) == epoch;
                    if (__ballot(!ready) == 0) break;
                    if (++spins == (1u << 22)) {
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                const int k = lane % 6;
                const uint32_t x = (uint32_t)v;
#pragma unroll
                for (int kk = 0; kk < 6; ++kk) {  // fold word kk over the lanes that hold it
                    uint32_t y = mine && k == kk ? x : (kk < 3 ? 0xffffffffu : 0u);
                    y = kk < 3 ? lidar::wave_min_u32_dpp(y) : ~lidar::wave_min_u32_dpp(~y);
                    m[kk] = kk < 3 ? min(m[kk], y) : max(m[kk], y);
                }
            }
#pragma unroll
            for (int kk = 0; kk < 6; ++kk)  // hung: NaN extent, the grid fails
                if (lane == kk) ext[kk] = ok ? m[kk] : ord(__builtin_nanf(""));
            if (!ok && lane == 0) w.meta[f * MW + 3] = epoch;  // reported as nvox -2
        }
    }
    __syncthreads();
    const double lo[3] = {unord(ext[0]), unord(ext[1]), unord(ext[2])};
    const double hi[3] = {unord(ext[3]), unord(ext[4]), unord(ext[5])};
    const lidar_vox::Grid g = lidar_vox::make_grid(lo, hi, voxel);
    uint32_t *m = w.meta + (int64_t)f * MW;
    const uint32_t okey = g.ok ? (uint32_t)g.keys : 0u;  // nx ny nz >= 1: one past the last voxel
    const int bits = g.ok ? 32 - __clz((int)okey) : 0;
    const int hs = max(0, bits - HB);
    if (t == 0 && tid == 0) {
        m[0] = g.ok ? 1u : 0u;
        m[1] = okey;
        m[2] = (uint32_t)hs;  // (m[3]: the hung tag, this call's epoch only when set by this call)
    }
    if (!g.ok) return;  // whole workgroup (uniform)
    // the float thresholds of every axis' edges in LDS when each axis has <= ETAB edges and the grid's
    // span is a float range (uniform); else every point runs lidar_vox::key in float64
    bool tab = true;
    int L[3];
    float s0[3], inv[3], lastf[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const lidar_vox::FAxis fa = lidar_vox::faxis(g.ax[a], ETAB);
        tab = tab && fa.ok;
        L[a] = fa.L;
        s0[a] = fa.s0;
        inv[a] = fa.inv;
        lastf[a] = fa.lastf;
    }
    VX_KSTAMP(2);
    if (tab) {
#pragma unroll
        for (int a = 0; a < 3; ++a)
            for (int i = tid; i < L[a] + 2; i += KT)
                etab[a][i] = i == 0 ? -INFINITY : i > L[a] ? INFINITY : ru_float(lidar_vox::edge(g.ax[a], i - 1));
        __syncthreads();
    }
    VX_KSTAMP(3);
    const uint32_t ny = (uint32_t)g.ax[1].nb, nz = (uint32_t)g.ax[2].nb;
    uint32_t kv[PPT];
    if (tab) {
        // the table lookups of half the tile's points in flight together (branch-free), the rare guess
        // off by more than a bin fixed afterwards
        constexpr int H = PPT / 2;
#pragma unroll
        for (int h0 = 0; h0 < PPT; h0 += H) {
            int c[H][3];
            bool miss = false;
#pragma unroll
            for (int j = 0; j < H; ++j)
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    c[j][a] = bin_tab_c(etab[a] + 1, L[a], q[h0 + j][a], s0[a], inv[a]);
                    miss = miss || c[j][a] < 0;
                }
            if (miss)
#pragma unroll
                for (int j = 0; j < H; ++j)
#pragma unroll
                    for (int a = 0; a < 3; ++a)
                        if (c[j][a] < 0) c[j][a] = bin_tab_search(etab[a] + 1, L[a], q[h0 + j][a]);
#pragma unroll
            for (int j = 0; j < H; ++j) {
                const uint32_t bx = bin_of_c(c[j][0], q[h0 + j][0], lastf[0], L[0]);
                const uint32_t by = bin_of_c(c[j][1], q[h0 + j][1], lastf[1], L[1]);
                const uint32_t bz = bin_of_c(c[j][2], q[h0 + j][2], lastf[2], L[2]);
                // (bx ny + by) nz + bz < nx ny nz < 2^32: exact in 32 bits
                const bool out = bx == lidar_vox::kOutside || by == lidar_vox::kOutside || bz == lidar_vox::kOutside;
                kv[h0 + j] = out ? okey : (bx * ny + by) * nz + bz;
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const uint32_t kk = lidar_vox::key(g, q[j][0], q[j][1], q[j][2]);
            kv[j] = kk == lidar_vox::kOutside ? okey : kk;  // sorts after every voxel's key
        }
    }
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const int64_t i = (int64_t)t * TILE + j * KT + tid;
        if (i < n) atomicAdd(&hist[kv[j] >> hs], 1u);
        else kv[j] = 0u;
    }
    __syncthreads();
    VX_KSTAMP(4);
    // the tile's histogram as self-tagged granules (bins 2g, 2g + 1 in granule g; thread tid publishes
    // the granules of its own scatter bins BPT tid .. BPT tid + 3)
    unsigned long long *hg = w.hgran + ((int64_t)f * ntiles + t) * (NBIN / 2);
#pragma unroll
    for (int e = 0; e < BPT / 2; ++e) {
        const int gi = (BPT / 2) * tid + e;
        const unsigned long long v = ((unsigned long long)epoch << 32) | (hist[2 * gi + 1] << 16) | hist[2 * gi];
        __hip_atomic_store(&hg[gi], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (!FUSED) {  // the scatter launch follows
        uint32_t *k = w.key + (int64_t)f * n;
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const int64_t i = (int64_t)t * TILE + j * KT + tid;
            if (i < n) k[i] = kv[j];
        }
    } else {
        // every tile of the frame is resident (<= kFuseTiles, one XCD): scatter straight from registers
        __syncthreads();  // hist[] becomes the scatter's offsets
        VX_KSTAMP(5);
        scatter_tile(kv, f, t, n, ntiles, hs, epoch, w, hist, &red6[0][0], batch, kts);
    }
#ifdef VX_DIAG_KEYS
    VX_KSTAMP(9);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(kts[11])::"memory");
    if (tid == 0) {  // diagnostic build only: stamps into the tail rows of the frame's centroids
        uint64_t *d = reinterpret_cast<uint64_t *>(w.cent_diag + (f + 1) * n * 3) - 12 * (t + 1);
        for (int k = 0; k < 12; ++k) d[k] = kts[k];
    }
#endif
}

// ------------------------------------------------------------------------------------- scatter
// the scatter of frames above kFuseTiles tiles (the keys launch wrote the keys)
__global__ __launch_bounds__(KT) void vx_scatter_kernel(int64_t n, Ws w, int ntiles, int64_t batch, uint32_t epoch)
{
    int64_t f, t;
    if (!frame_part(batch, ntiles, f, t)) return;
    const int tid = threadIdx.x;
    const uint32_t *m = w.meta + (int64_t)f * MW;
    if (!m[0]) return;
    const int hs = (int)m[2];
    __shared__ uint32_t off[NBIN];
    __shared__ uint32_t red[KT / 64];
    const uint32_t *k = w.key + (int64_t)f * n;
    uint32_t kv[PPT];
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
        const int64_t i = (int64_t)t * TILE + j * KT + tid;
        kv[j] = i < n ? k[i] : 0u;
    }
    scatter_tile(kv, f, t, n, ntiles, hs, epoch, w, off, red, batch);
}

// ------------------------------------------------------------------------------------- buckets
// stable LSD radix sort of m pairs in global memory by one workgroup (a bucket above CAP), over the
// 8-bit digits whose bits vary across the bucket; returns the buffer holding the result
__device__ uint64_t *bucket_radix(uint64_t *a, uint64_t *b, int64_t m, uint32_t *cnt, uint32_t (*wc)[256],
                                  uint32_t *red, unsigned long long *vary)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) *vary = 0ull;
    __syncthreads();
    const uint64_t v0 = a[0];
    uint64_t x = 0;
    for (int64_t i = tid; i < m; i += UT) x |= a[i] ^ v0;
    for (int o = 32; o >= 1; o >>= 1) x |= (uint64_t)__shfl_xor((long long)x, o, 64);
    if (lane == 0) atomicOr(vary, (unsigned long long)x);
    __syncthreads();
    const uint64_t vb = *vary;
    for (int shift = 0; shift < 64; shift += 8) {
        if (((vb >> shift) & 0xffull) == 0) continue;  // uniform: this digit is constant
        if (tid < 256) cnt[tid] = 0;
        __syncthreads();
        for (int64_t i = tid; i < m; i += UT) atomicAdd(&cnt[(a[i] >> shift) & 255u], 1u);
        __syncthreads();
        uint32_t all;
        const uint32_t ex = block_excl_scan<UT>(tid < 256 ? cnt[tid] : 0u, red, &all);
        __syncthreads();
        if (tid < 256) cnt[tid] = ex;  // running offset per digit
        const uint64_t below = (1ull << lane) - 1;
        for (int64_t c0 = 0; c0 < m; c0 += UT) {
            const int64_t i = c0 + tid;
            const bool valid = i < m;
            const uint64_t v = valid ? a[i] : 0ull;
            const uint32_t dig = (uint32_t)(v >> shift) & 255u;
            uint64_t same = __ballot(valid);
#pragma unroll
            for (int bit = 0; bit < 8; ++bit) {
                const uint64_t bm = __ballot((dig >> bit) & 1u);
                same &= ((dig >> bit) & 1u) ? bm : ~bm;
            }
            for (int d = lane; d < 256; d += 64) wc[wave][d] = 0;
            __syncthreads();  // (also: cnt advanced by the previous chunk)
            if (valid && (same & below) == 0) wc[wave][dig] = (uint32_t)__popcll(same);
            __syncthreads();
            if (valid) {
                uint32_t o = cnt[dig] + (uint32_t)__popcll(same & below);
                for (int q = 0; q < wave; ++q) o += wc[q][dig];
                b[o] = v;
            }
            __syncthreads();
            if (tid < 256) {
                uint32_t s = 0;
                for (int q = 0; q < UT / 64; ++q) s += wc[q][tid];
                cnt[tid] += s;
            }
        }
        __syncthreads();
        uint64_t *tmp = a;
        a = b;
        b = tmp;
    }
    return a;
}

// the bucket's voxel offset: the sum of the earlier buckets' voxel counts, by a decoupled look-back
// over 64 predecessors at a time (one wave; each lane one look-back word).  Publishes the bucket's
// own count first, its inclusive prefix last.  Waits only on lower part indices of the same frame,
// i.e. on workgroups dispatched before this one; every spin is bounded (*hung: a bug, not a hang).
// A look-back word is its own payload (status << 32 | count, one 8-byte sc1 store, read by sc1 loads
// that bypass the L1): relaxed agent-scope atomics, no fences (an acquire would invalidate the CU's
// L1 per poll and a release write back the XCD's L2 per store: MI355X_MICROARCH.md, ~1.7 us each).
// (published: the count went out earlier, by look_back_publish.)
__device__ __forceinline__ void look_back_publish(unsigned long long *fl, int64_t b, uint32_t nv)
{
    __hip_atomic_store(&fl[b], ((b == 0 ? 2ull : 1ull) << 32) | nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// (first: the words of the first window, loaded earlier by look_back_first, or null.)
__device__ __forceinline__ unsigned long long look_back_first(const unsigned long long *fl, int64_t b)
{
    const int64_t q = b - 1 - (threadIdx.x & 63);
    return q >= 0 ? __hip_atomic_load(&fl[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (2ull << 32);
}
__device__ uint64_t look_back(unsigned long long *fl, int64_t b, uint32_t nv, bool *hung, uint32_t *nspins = nullptr,
                              bool published = false, const unsigned long long *first = nullptr)
{
    const int lane = threadIdx.x & 63;
    if (lane == 0 && !published) look_back_publish(fl, b, nv);
    uint64_t pre = 0;
    *hung = false;
    int64_t top = b - 1;
    uint32_t spins = 0;
    while (top >= 0) {
        const int64_t q = top - lane;
        const unsigned long long v = first && top == b - 1 && spins == 0 ? *first
                                     : q >= 0 ? __hip_atomic_load(&fl[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                              : (2ull << 32);
        const uint32_t st = (uint32_t)(v >> 32);
        const uint64_t incl = __ballot(st == 2);
        const int k = incl ? __ffsll((unsigned long long)incl) - 1 : 63;
        const uint64_t upto = k == 63 ? ~0ull : ((2ull << k) - 1);
        if (__ballot(st == 0) & upto) {  // a predecessor before the first inclusive one has not published
            __builtin_amdgcn_s_sleep(2);
            if (++spins == (1u << 24)) {
                *hung = true;
                break;
            }
            continue;
        }
        uint64_t s = lane <= k ? (v & 0xffffffffull) : 0ull;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += (uint64_t)__shfl_xor((long long)s, o, 64);
        pre += s;
        if (incl) break;
        top -= 64;
    }
    if (nspins) *nspins = spins;
    if (lane == 0 && b > 0)
        __hip_atomic_store(&fl[b], (2ull << 32) | (pre + nv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return pre;
}

#ifdef LIDAR_DIAG
__device__ int64_t g_vx_inject_bad = -1;  // the diagnostic library's failure injection (a bucket index)
#endif

// A bucket's outcome for nvox[f] (lane 0 of wave 0).  A failure — a look-back wait that timed out (hung:
// nvox -2) or a bucket table that is not a partition of [0, n) (bad: nvox -3), both bugs upstream, never
// expected — tags the frame's meta[4] with this call's epoch before it stores its code, and the frame's
// last bucket reads that tag after its own look-back has completed.  A failed bucket ends its wait before
// the predecessor it waited for publishes, and the last bucket's look-back needs that publication, so the
// tag is set before the last bucket reads it: a failure always wins over the frame's voxel count (the
// count alone, written by the last bucket, would look valid with ids and centroids at wrong offsets).
__device__ __forceinline__ void bucket_report(int32_t *nvox, uint32_t *m, int64_t f, int64_t b, int64_t nb,
                                              uint64_t total, bool hung, bool bad, uint32_t epoch)
{
    if (hung || bad) {
        const uint32_t code = bad ? 3u : 2u;
        __hip_atomic_store(&m[5], code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&m[4], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        nvox[f] = -(int32_t)code;
    } else if (b == nb - 1) {
        nvox[f] = __hip_atomic_load(&m[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch
                      ? -(int32_t)__hip_atomic_load(&m[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : (int32_t)total;
    }
}

// 34 KiB: four 512-thread workgroups per CU (at <= 64 VGPRs)
struct BucketLds {
    union {
        struct {
            uint32_t s[CAP];   // the counting sort's unordered runs: point indices (a run is one key)
            union {
                uint32_t cnt[KMAX];  // counting-sort counters, then per key its first sorted position | its
                                     // voxel's rank in the bucket << 16 (the radix path: its digit tables)
                struct {
                    uint32_t idx[CAP];     // the point indices in sorted order (written once cnt is dead;
                                           // the shifted sort: bit 31 marks a voxel's first point)
                    uint16_t vpos[CAP];    // the shifted sort: voxels up to each sorted position
                };
            };
        };
        uint64_t a[BITONIC_P];  // the bitonic path's pairs (over the above)
    };
    uint16_t vstart[CAP + 1];  // voxel v's first sorted position, then the voxels' end
    uint8_t rank[CAP];         // the dense sort: each pair's rank inside its key (load order)
};
static_assert(CAP < 65536, "packed first position | voxel rank");

__global__ __launch_bounds__(UT, 8) void vx_bucket_kernel(const float *__restrict__ xyz, int64_t n, Ws w,
                                                       int32_t *__restrict__ vid, float *__restrict__ cent,
                                                       int32_t *__restrict__ counts, int32_t *__restrict__ nvox,
                                                       int64_t batch, uint32_t epoch)
{
    const int64_t nb = n_buckets(n);
    int64_t f, b;
    if (!frame_part(batch, nb, f, b)) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef VX_DIAG_PHASES
    uint64_t ts[8] = {}, rt[8] = {};
    auto stamp = [&](int k) {
        uint64_t t, r;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r)::"memory");
        ts[k] = t;
        rt[k] = r;
    };
#define VX_STAMP(k) stamp(k)
#else
#define VX_STAMP(k)
#endif
    VX_STAMP(0);
    // the bucket's pairs [bstart[b], bstart[b + 1]) (the scatter launch's bucket table), loaded beside the
    // frame's meta words
    const uint32_t bs = tid < 2 ? w.bstart[(int64_t)f * (nb + 1) + b + tid] : 0u;
    uint32_t *m = w.meta + (int64_t)f * MW;
    if (!m[0] || m[3] == epoch) {
        if (b == 0 && tid == 0) nvox[f] = m[3] == epoch ? -2 : -1;
        return;  // every bucket of the frame returns: nothing waits on this frame's look-back words
    }
    const uint32_t okey = m[1];
    __shared__ __attribute__((aligned(16))) BucketLds L;
    __shared__ uint32_t rng[4];
    __shared__ uint32_t red[UT / 64];
    __shared__ uint32_t flag;
    __shared__ unsigned long long prefix, vary;
#ifdef VX_DIAG_PHASES
    __shared__ uint32_t spins_dbg;
    if (tid == 0) spins_dbg = 0;
#endif
    if (tid < 2) rng[tid] = bs;
    if (tid == 2) rng[2] = 0xffffffffu;  // [2], [3]: key min / max
    if (tid == 3) rng[3] = 0u;
    if (tid == 0) flag = 0;
    __syncthreads();
    VX_STAMP(1);
    // a bucket table that is not a partition of [0, n) is a bug upstream: the bucket sorts nothing (its
    // count 0 still goes out, so the frame's later buckets do not wait on it) and reports nvox -3
    bool bad = rng[0] > rng[1] || (int64_t)rng[1] > n;  // (uniform)
#ifdef LIDAR_DIAG
    bad = bad || b == g_vx_inject_bad;  // testing aid (lidar_debug_voxel_inject): this bucket's table is "bad"
#endif
    const int64_t p0 = bad ? 0 : rng[0], size = bad ? 0 : (int64_t)rng[1] - rng[0];
    const uint64_t *gp = w.pairs + (int64_t)f * n + p0;
    const float *p = xyz + (int64_t)f * n * 3;
    unsigned long long *fl = reinterpret_cast<unsigned long long *>(w.flags + (int64_t)f * nb);
    int32_t *vf = vid + (int64_t)f * n;
    float *cf = cent + (int64_t)f * n * 3;
    int32_t *nf = counts + (int64_t)f * n;
    const uint64_t *seq = nullptr;  // the slow paths: the bucket sorted by (key, index), LDS or global
    bool radix = false;
    if (size <= CAP) {
        // the pairs, and the range of the keys they hold (not of their coarse bins: the first and last
        // buckets' bins reach over the grid's empty margins, past the counting sort's range)
        static_assert(CAP % UT == 0, "pairs per thread");
        uint32_t kk[CAP / UT], id[CAP / UT];  // the pairs' keys and point indices
        {
            uint32_t kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
            for (int j = 0; j < CAP / UT; ++j) {
                const uint64_t x = tid + j * UT < size ? gp[tid + j * UT] : 0ull;
                kk[j] = (uint32_t)(x >> 32);
                id[j] = (uint32_t)x;
            }
#pragma unroll
            for (int j = 0; j < CAP / UT; ++j)
                if (tid + j * UT < size) {
                    kmin = min(kmin, kk[j]);
                    kmax = max(kmax, kk[j]);
                }
            kmin = lidar::wave_min_u32_dpp(kmin);
            kmax = ~lidar::wave_min_u32_dpp(~kmax);
            if (lane == 0) {
                atomicMin(&rng[2], kmin);
                atomicMax(&rng[3], kmax);
            }
        }
        __syncthreads();
        const uint64_t k0 = rng[2], krange = size ? (uint64_t)rng[3] - rng[2] + 1 : 0;
        // local keys: (key - k0) >> sh, below KMAX.  sh = 0: one counter per key; sh > 0 (a sparse grid):
        // runs of a counter hold several keys, ordered by (key, index) as one 32-bit word (key's low sh
        // bits << ib | index) when that fits
        static_assert(KMAX == 4096, "12-bit local keys");
        const int kb = krange > 1 ? 64 - __clzll((unsigned long long)(krange - 1)) : 0;
        const int sh = max(0, kb - 12);
        const int ib = 32 - __clz((uint32_t)max<int64_t>(n - 1, 1));
        const bool counting = sh == 0 || sh + ib <= 32;
        const uint32_t nbin = counting && krange ? (uint32_t)((krange - 1) >> sh) + 1u : 0u;
        for (int64_t c = tid; c < (int64_t)nbin; c += UT) L.cnt[c] = 0;
        __syncthreads();
        auto lkey = [&](uint32_t key) { return (key - (uint32_t)k0) >> sh; };
        if (counting) {
            // counting sort by local key: a rank inside the local key from an LDS atomic (a run past
            // SEGMAX: the bitonic path instead)
            static_assert(SEGMAX < 256, "8-bit ranks");
#pragma unroll
            for (int j = 0; j < CAP / UT; ++j)
                if (tid + j * UT < size) {
                    const uint32_t r = atomicAdd(&L.cnt[lkey(kk[j])], 1u);
                    L.rank[tid + j * UT] = (uint8_t)r;
                    if (r == SEGMAX) flag = 1;
                }
            __syncthreads();
        }
        VX_STAMP(2);
        if (counting && !flag) {  // (uniform)
            uint32_t nvl;
            uint32_t sv[CAP / UT];  // finally: the point's voxel rank in the bucket (nvl: outside every bin)
            unsigned long long lb0 = 0;
            constexpr int PT = KMAX / UT;
            static_assert(CAP < 4096 && SEGMAX < 256, "packed run fields");
            if (sh == 0) {
                // one exclusive scan of (count | occupied << 16) over the keys gives every key its first
                // sorted position and its voxel's rank in the bucket (the outside key occupies no voxel),
                // and the bucket's voxel count, published at once for the later buckets' look-back
                uint32_t cv[PT], sum = 0;
#pragma unroll
                for (int j = 0; j < PT; ++j) {
                    const int64_t c = PT * tid + j;
                    const uint32_t x = c < (int64_t)nbin ? L.cnt[c] : 0u;
                    cv[j] = x + (x != 0u && (uint32_t)(k0 + c) != okey ? 0x10000u : 0u);
                    sum += cv[j];
                }
                uint32_t all;
                uint32_t ex = block_excl_scan<UT>(sum, red, &all);
#pragma unroll
                for (int j = 0; j < PT; ++j) {
                    const int64_t c = PT * tid + j;
                    if (c < (int64_t)nbin) L.cnt[c] = ex;
                    if (cv[j]) L.vstart[ex >> 16] = (uint16_t)ex;  // a voxel's first position (the outside
                    ex += cv[j];                                    // key's run, the last: vstart[nvl])
                }
                nvl = all >> 16;
                if (tid == 0) look_back_publish(fl, b, nvl);
                if (tid == 0 && rng[3] != okey) L.vstart[nvl] = (uint16_t)size;
                __syncthreads();
                VX_STAMP(3);
                // each key's run, unordered (sv: the point's voxel rank; the run: vstart[vp] ..
                // vstart[vp + 1], or the bucket's end for the outside key's run)
#pragma unroll
                for (int j = 0; j < CAP / UT; ++j)
                    if (tid + j * UT < size) {
                        const uint32_t e = L.cnt[lkey(kk[j])];
                        L.s[(e & 0xffffu) + L.rank[tid + j * UT]] = id[j];
                        sv[j] = e >> 16;
                    }
                __syncthreads();
                // wave 0: the look-back's first window in flight during the placement below (the
                // earlier buckets publish their counts at the same point of their lives)
                if (wave == 0) lb0 = look_back_first(fl, b);
                // index order inside a run (< SEGMAX long): every element counts the smaller indices of
                // its run; its index lands at its sorted position
#pragma unroll
                for (int j = 0; j < CAP / UT; ++j) {
                    const int64_t i = tid + j * UT;
                    if (i < size) {
                        const uint32_t vp = sv[j], st = L.vstart[vp];
                        const uint32_t en = vp == nvl ? (uint32_t)size : L.vstart[vp + 1];
                        uint32_t r = 0;
                        for (uint32_t x = st; x < en; ++x) r += L.s[x] < id[j] ? 1u : 0u;
                        L.idx[st + r] = id[j];
                    }
                }
            } else {
                // the shifted sort: starts of the local keys' runs by an exclusive scan of the counts
                uint32_t cv[PT], sum = 0;
#pragma unroll
                for (int j = 0; j < PT; ++j) {
                    const int64_t c = PT * tid + j;
                    cv[j] = c < (int64_t)nbin ? L.cnt[c] : 0u;
                    sum += cv[j];
                }
                uint32_t all;
                uint32_t ex = block_excl_scan<UT>(sum, red, &all);
#pragma unroll
                for (int j = 0; j < PT; ++j) {
                    const int64_t c = PT * tid + j;
                    if (c < (int64_t)nbin) L.cnt[c] = ex;
                    ex += cv[j];
                }
                __syncthreads();
                VX_STAMP(3);
                const uint32_t kmask = (1u << sh) - 1u;
                // each run, unordered (sv: its first position | its length << 12 | outside << 20; then a
                // slot from the local key's cursor for the point's word — (key's low sh bits, index) in
                // order — which replaces its key in kk)
#pragma unroll
                for (int j = 0; j < CAP / UT; ++j)
                    if (tid + j * UT < size) {
                        const uint32_t lk = lkey(kk[j]), st = L.cnt[lk];
                        const uint32_t en = lk + 1 < nbin ? L.cnt[lk + 1] : (uint32_t)size;
                        sv[j] = st | (en - st) << 12 | (kk[j] == okey ? 1u << 20 : 0u);
                    }
                __syncthreads();
#pragma unroll
                for (int j = 0; j < CAP / UT; ++j)
                    if (tid + j * UT < size) {
                        const uint32_t lk = lkey(kk[j]);
                        kk[j] = ((kk[j] - (uint32_t)k0) & kmask) << ib | id[j];
                        L.s[atomicAdd(&L.cnt[lk], 1u)] = kk[j];
                    }
                __syncthreads();
                // (key, index) order inside a run: every element counts the smaller words of its run, and
                // whether one of them holds its key (else it is its voxel's first point; the outside key
                // is no voxel)
#pragma unroll
                for (int j = 0; j < CAP / UT; ++j) {
                    const int64_t i = tid + j * UT;
                    if (i < size) {
                        const uint32_t st = sv[j] & 0xfffu, en = st + ((sv[j] >> 12) & 0xffu), wd = kk[j];
                        const uint32_t hi = ib == 32 ? 0u : wd >> ib;
                        uint32_t r = 0;
                        bool dup = false;
                        for (uint32_t x = st; x < en; ++x) {
                            const uint32_t w2 = L.s[x];
                            r += w2 < wd ? 1u : 0u;
                            dup = dup || (w2 < wd && (ib == 32 ? 0u : w2 >> ib) == hi);
                        }
                        const bool out = (sv[j] >> 20) & 1u;
                        L.idx[st + r] = id[j] | (!dup && !out ? 0x80000000u : 0u);
                        sv[j] = (st + r) | (!dup ? 1u << 16 : 0u) | (out ? 1u << 17 : 0u);
                    }
                }
                __syncthreads();
                // voxel ranks: the voxels' first points up to each sorted position (CAP / UT consecutive
                // positions per thread), the bucket's count published at once
                constexpr int CH = CAP / UT;
                uint32_t bits = 0, fc = 0;
#pragma unroll
                for (int k = 0; k < CH; ++k) {
                    const int64_t o = CH * tid + k;
                    const uint32_t fb = o < size ? L.idx[o] >> 31 : 0u;
                    bits |= fb << k;
                    fc += fb;
                }
                uint32_t allv;
                uint32_t inc = block_excl_scan<UT>(fc, red, &allv);
#pragma unroll
                for (int k = 0; k < CH; ++k) {
                    const int64_t o = CH * tid + k;
                    inc += (bits >> k) & 1u;
                    if (o < size) L.vpos[o] = (uint16_t)inc;
                }
                nvl = allv;
                if (tid == 0) look_back_publish(fl, b, nvl);
                __syncthreads();
                if (wave == 0) lb0 = look_back_first(fl, b);
#pragma unroll
                for (int j = 0; j < CAP / UT; ++j) {
                    const int64_t i = tid + j * UT;
                    if (i < size) {
                        const uint32_t o = sv[j] & 0xffffu;
                        const bool first = (sv[j] >> 16) & 1u, out = (sv[j] >> 17) & 1u;
                        const uint32_t vp = out ? nvl : (uint32_t)L.vpos[o] - 1u;
                        if (first) L.vstart[vp] = (uint16_t)o;  // the outside key's first point ends the last voxel
                        sv[j] = vp;
                    }
                }
                if (tid == 0 && rng[3] != okey) L.vstart[nvl] = (uint16_t)size;
            }
            VX_STAMP(4);
            if (wave == 0) {  // the earlier buckets have published their counts by now (one pass, no wait)
                bool hung;
                uint32_t nsp = 0;
                const uint64_t pre = look_back(fl, b, nvl, &hung, &nsp, true, &lb0);
#ifdef VX_DIAG_PHASES
                if (lane == 0) spins_dbg = nsp;
#endif
                if (lane == 0) {
                    prefix = pre;
                    bucket_report(nvox, m, f, b, nb, pre + nvl, hung, bad, epoch);
                }
            }
            __syncthreads();
            VX_STAMP(5);
            const uint32_t O = (uint32_t)prefix;
            // the points' voxel ids (from registers)
#pragma unroll
            for (int j = 0; j < CAP / UT; ++j)
                if (tid + j * UT < size)
                    vf[id[j]] = sv[j] == nvl ? -1 : (int32_t)(O + sv[j]);  // nvl: outside
            VX_STAMP(6);
            // one thread per voxel: the sequential fp32 sums over its points in index order, their xyz
            // gathered GB at a time (the frame's points are L2-resident since the keys launch), the
            // centroid and count (consecutive threads: consecutive voxels)
            for (uint32_t vv = tid; vv < nvl; vv += UT) {
                const int i0 = L.vstart[vv], i1 = L.vstart[vv + 1];
                float sx = 0.f, sy = 0.f, sz = 0.f;
                constexpr int GB = 8;  // one round trip for most voxels
                for (int e0 = i0; e0 < i1; e0 += GB) {
                    float q[GB][3];
#pragma unroll
                    for (int k = 0; k < GB; ++k) {
                        const int64_t id = (e0 + k < i1 ? L.idx[e0 + k] : L.idx[i0]) & 0x7fffffffu;
#pragma unroll
                        for (int c = 0; c < 3; ++c) q[k][c] = p[3 * id + c];
                    }
#pragma unroll
                    for (int k = 0; k < GB; ++k)
                        if (e0 + k < i1) {
                            sx = __fadd_rn(sx, q[k][0]);
                            sy = __fadd_rn(sy, q[k][1]);
                            sz = __fadd_rn(sz, q[k][2]);
                        }
                }
                const int64_t o = (int64_t)O + vv;
                const float c = (float)(i1 - i0);
                cf[3 * o] = __fdiv_rn(sx, c);
                cf[3 * o + 1] = __fdiv_rn(sy, c);
                cf[3 * o + 2] = __fdiv_rn(sz, c);
                nf[o] = i1 - i0;
            }
        } else if (size <= BITONIC_P) {
            // bitonic sort of the pairs in LDS (a key range past the counting sort, or a long run)
            __syncthreads();  // (the counting attempt's cnt reads are done: a overlays it)
            int64_t P = 1;
            while (P < size) P <<= 1;
            for (int64_t i = tid; i < P; i += UT) L.a[i] = i < size ? gp[i] : ~0ull;  // (reloaded; pads last)
            __syncthreads();
            for (int64_t k2 = 2; k2 <= P; k2 <<= 1)
                for (int64_t j = k2 >> 1; j > 0; j >>= 1) {
#pragma unroll 1
                    for (int64_t i = tid; i < P; i += UT) {
                        const int64_t l = i ^ j;
                        if (l > i) {
                            const uint64_t x = L.a[i], y = L.a[l];
                            if ((x > y) == ((i & k2) == 0)) {
                                L.a[i] = y;
                                L.a[l] = x;
                            }
                        }
                    }
                    __syncthreads();
                }
            seq = L.a;
        } else {
            radix = true;
        }
    } else {
        radix = true;
    }
    if (radix) {  // (uniform) a bucket past the LDS sorts: LSD radix sort in global memory
        __syncthreads();
        seq = bucket_radix(const_cast<uint64_t *>(gp), w.scratch + (int64_t)f * n + p0, size, L.cnt,
                           reinterpret_cast<uint32_t(*)[256]>(L.cnt + 256), red, &vary);
    }
    if (seq) {
        // the slow paths: voxel starts over the sorted sequence, the look-back, then ids and sums
        __syncthreads();
        constexpr int CH = 4;  // this thread's elements are CH consecutive ones per chunk of CH UT
        auto key_at = [&](int64_t i) { return (uint32_t)(seq[i] >> 32); };
        auto start_at = [&](int64_t i) {
            const uint32_t kk = key_at(i);
            return kk != okey && (i == 0 || kk != key_at(i - 1));
        };
        uint32_t nvl = 0;
        for (int64_t c0 = 0; c0 < size; c0 += CH * UT) {
            uint32_t s = 0;
#pragma unroll
            for (int j = 0; j < CH; ++j) {
                const int64_t i = c0 + CH * tid + j;
                if (i < size) s += start_at(i) ? 1u : 0u;
            }
            uint32_t all;
            block_excl_scan<UT>(s, red, &all);
            nvl += all;
        }
        if (wave == 0) {
            bool hung;
            const uint64_t pre = look_back(fl, b, nvl, &hung);
            if (lane == 0) {
                prefix = pre;
                bucket_report(nvox, m, f, b, nb, pre + nvl, hung, bad, epoch);
            }
        }
        __syncthreads();
        const uint32_t O = (uint32_t)prefix;
        uint32_t carry = 0;
        for (int64_t c0 = 0; c0 < size; c0 += CH * UT) {
            bool st[CH];
            uint32_t s = 0;
#pragma unroll
            for (int j = 0; j < CH; ++j) {
                const int64_t i = c0 + CH * tid + j;
                st[j] = i < size && start_at(i);
                s += st[j] ? 1u : 0u;
            }
            uint32_t all;
            uint32_t r = O + carry + block_excl_scan<UT>(s, red, &all);  // voxels before this thread's elements
#pragma unroll
            for (int j = 0; j < CH; ++j) {
                const int64_t i = c0 + CH * tid + j;
                if (i >= size) break;
                const uint64_t v = seq[i];
                const uint32_t kk = (uint32_t)(v >> 32);
                r += st[j] ? 1u : 0u;
                vf[(uint32_t)v] = kk == okey ? -1 : (int32_t)(r - 1);
                if (st[j]) {  // this voxel's points in index order: the sequential fp32 sums
                    float sx = 0.f, sy = 0.f, sz = 0.f;
                    int64_t e = i;
                    for (; e < size && key_at(e) == kk; ++e) {
                        const int64_t idx = (uint32_t)seq[e];
                        sx = __fadd_rn(sx, p[3 * idx]);
                        sy = __fadd_rn(sy, p[3 * idx + 1]);
                        sz = __fadd_rn(sz, p[3 * idx + 2]);
                    }
                    const int64_t o = r - 1;
                    const float c = (float)(e - i);
                    cf[3 * o] = __fdiv_rn(sx, c);
                    cf[3 * o + 1] = __fdiv_rn(sy, c);
                    cf[3 * o + 2] = __fdiv_rn(sz, c);
                    nf[o] = (int32_t)(e - i);
                }
            }
            carry += all;
        }
    }
#ifdef VX_DIAG_PHASES
    VX_STAMP(7);
    if (tid == 0)  // diagnostic build only: phase cycles into the scratch tail of the counts output
    {
        int32_t *d = nf + n - 16 * (b + 1);
        for (int k = 0; k < 7; ++k) d[k] = (int32_t)(ts[k + 1] - ts[k]);
        d[7] = (int32_t)spins_dbg;
        for (int k = 0; k < 8; ++k) d[8 + k] = (int32_t)(rt[k] & 0x7fffffff);  // 100 MHz, chip-wide
    }
#endif
#undef VX_STAMP
}

}  // namespace

#ifdef LIDAR_DIAG
// testing aid (the diagnostic library only): the bucket launches that follow treat bucket `bucket` of every
// frame as having an inconsistent bucket table (-1: none), so the sticky failure report can be tested
LIDAR_EXPORT int lidar_debug_voxel_inject(int64_t bucket)
{
    const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_vx_inject_bad), &bucket, sizeof(bucket));
    return e == hipSuccess ? LIDAR_OK : lidar::fail(LIDAR_EHIP, "lidar_debug_voxel_inject: hipMemcpyToSymbol");
}
#endif

// workspace bytes of lidar_voxel_downsample_batch_f32 for (batch, n) (the granules and meta words live in
// the handle's own tag block, beside it)
LIDAR_EXPORT uint64_t lidar_voxel_batch_workspace_bytes(int64_t batch, int64_t n)
{
    const int64_t nb = (n + BUCKET - 1) / BUCKET;
    lidar::Carver cv;
    cv.take<uint32_t>(batch * n);
    cv.take<uint32_t>(batch * (nb + 1));
    cv.take<uint64_t>(batch * n);
    cv.take<uint64_t>(batch * n);
    cv.take<uint64_t>(batch * nb);
    return cv.off;
}

namespace {
// the handle's tag block of at least `bytes` (granules + meta words), and this call's epoch.  The block
// is written by voxel calls only, so every tag in it is an earlier call's epoch or 0: no per-call reset.
// A larger block replaces a smaller one (the old one retired like a workspace: queued calls may still
// use it) and starts zeroed; so does the block when the epoch wraps.
void *vx_tags(lidar_handle *h, uint64_t bytes, hipStream_t s, uint32_t *epoch)
{
    if (bytes > h->vx_tags_bytes) {
        const uint64_t want = lidar::align_up(std::max(bytes + bytes / 4, 2 * h->vx_tags_bytes), 1 << 16);
        void *fresh = nullptr;
        const hipError_t e = hipMalloc(&fresh, want);
        if (e != hipSuccess) {
            lidar::set_error(std::string("voxel tag block hipMalloc(") + std::to_string(want) + "): " +
                             hipGetErrorString(e));
            return nullptr;
        }
        if (hipMemsetAsync(fresh, 0, want, s) != hipSuccess) {
            (void)hipFree(fresh);
            lidar::set_error("voxel tag block: hipMemsetAsync failed");
            return nullptr;
        }
        if (h->vx_tags) {
            h->retired.push_back(h->vx_tags);
            h->retired_bytes += h->vx_tags_bytes;
        }
        h->vx_tags = fresh;
        h->vx_tags_bytes = want;
    }
    if (++h->epoch == 0) {  // wrapped: no tag may equal a new epoch
        if (hipMemsetAsync(h->vx_tags, 0, h->vx_tags_bytes, s) != hipSuccess) {
            lidar::set_error("voxel tag block: hipMemsetAsync failed");
            return nullptr;
        }
        h->epoch = 1;
    }
    *epoch = h->epoch;
    return h->vx_tags;
}
}  // namespace

// Voxel downsampling of `batch` frames of n points (xyz (batch, n, 3) fp32), all on the device:
// voxel_id (batch, n) int32, centroids (batch, n, 3) and counts (batch, n) with the first nvox[f]
// rows of frame f valid, nvox (batch,) int32 (-1: the frame's extent is not finite or its voxel grid
// has 2^32 - 1 keys or more; voxel_id -1: a point outside every bin).
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
    const int64_t nb = (n + BUCKET - 1) / BUCKET;
    REQUIRE((int64_t)frame_grid(batch, std::max<int64_t>(ntiles, nb)) < 0x7fffffff,
            "lidar_voxel_downsample_batch_f32: batch * n too large");
    // the in-launch hand-offs' granules (extents, then histograms) and the meta words: the tag block
    lidar::Carver ct;
    const uint64_t ogran = ct.take<unsigned long long>(batch * ntiles * (6 + NBIN / 2));
    const uint64_t ometa = ct.take<uint32_t>(batch * MW);
    uint32_t epoch = 0;
    char *tags = static_cast<char *>(vx_tags(h, ct.off, s, &epoch));
    if (!tags) return LIDAR_ENOMEM;
    lidar::Carver cv;
    const uint64_t okey = cv.take<uint32_t>(batch * n);
    const uint64_t obst = cv.take<uint32_t>(batch * (nb + 1));
    const uint64_t opairs = cv.take<uint64_t>(batch * n), oscr = cv.take<uint64_t>(batch * n);
    const uint64_t oflags = cv.take<uint64_t>(batch * nb);
    char *base = static_cast<char *>(lidar::workspace(h, cv.off));
    if (!base) return LIDAR_ENOMEM;
    Ws w;
    w.gran = reinterpret_cast<unsigned long long *>(tags + ogran);
    w.meta = reinterpret_cast<uint32_t *>(tags + ometa);
    w.key = reinterpret_cast<uint32_t *>(base + okey);
    w.hgran = w.gran + batch * ntiles * 6;
    w.bstart = reinterpret_cast<uint32_t *>(base + obst);
    w.pairs = reinterpret_cast<uint64_t *>(base + opairs);
    w.scratch = reinterpret_cast<uint64_t *>(base + oscr);
    w.flags = reinterpret_cast<uint64_t *>(base + oflags);
    w.cent_diag = centroids;
    if (ntiles > kFuseTiles)
        hipLaunchKernelGGL(vx_extent_kernel, dim3(frame_grid(batch, ntiles)), dim3(KT), 0, s, xyz, n, w, ntiles, batch,
                           epoch);
    if (ntiles <= kFuseTiles) {  // keys + scatter in one launch (a frame's tiles all resident)
        hipLaunchKernelGGL(vx_keys_kernel<true>, dim3(frame_grid(batch, ntiles)), dim3(KT), 0, s, xyz, n, voxel, w,
                           ntiles, batch, epoch, nb);
    } else {
        hipLaunchKernelGGL(vx_keys_kernel<false>, dim3(frame_grid(batch, ntiles)), dim3(KT), 0, s, xyz, n, voxel, w,
                           ntiles, batch, epoch, nb);
        hipLaunchKernelGGL(vx_scatter_kernel, dim3(frame_grid(batch, ntiles)), dim3(KT), 0, s, n, w, ntiles, batch,
                           epoch);
    }
    hipLaunchKernelGGL(vx_bucket_kernel, dim3(frame_grid(batch, nb)), dim3(UT), 0, s, xyz, n, w, voxel_id, centroids,
                       counts, nvox, batch, epoch);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
