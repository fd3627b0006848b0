// ball_query.hip — first-nsample ball query on gfx950 (exact, index order).
//
// Spec (oracle orc_ball_query): for every centre, the first `nsample`
// point indices in ascending order with d < r*r (fp32, d = (dx*dx+dy*dy)+dz*dz, one
// rounding per op), unused slots repeat the first hit, no hit -> 0.
//
// Two kernels implement it:
//
// * Grid (default for n >= kGridMinN).  `bq_bin_kernel` (one workgroup per frame) bins
//   the frame by (index window, cell): windows are 2^w consecutive point indices, cells
//   a uniform grid of side s >= r * (1 + 2^-8) over the frame's finite bbox, so every hit
//   of a centre lies in the 3x3x3 cells around the centre's cell (the 2^-8 margin covers
//   fp32 rounding of the cell coordinates, see bin_params).  A counting sort in LDS gives
//   per (window, cell) slot a contiguous range of (x, y, z, index) float4s.
//   `bq_grid_kernel` (one wavefront per centre) walks the windows in order: for each it
//   gathers the <= 9 z-runs of candidate cells (contiguous slots), tests the candidates,
//   collects the hits in LDS and ranks them by index (hits of window w all precede those
//   of window w+1), and stops after the window where nsample hits are reached.  For a
//   uniform 65 536-point frame at r = 0.2 that is ~3 windows of ~110 candidates instead of
//   the ~8 000 points the index-order scan touches.  A window with more than kCap
//   candidates is scanned in index order (the brute loop below) instead.
// * Brute (small frames): one wavefront serves 8 centres and scans the frame in index
//   order, 128 points per step (two coalesced 64-point chunks, the next pair prefetched),
//   __ballot collects hits, popcount ranks them, and the scan stops once every centre has
//   nsample hits.
#include <cstdlib>

#include "bq_grid.hpp"

// windows per frame ~ LIDAR_BQ_WIN x (expected hits per centre) / nsample: ~nsample expected hits per
// window (1.0, measured: 1 234-1 254 vs 1 222-1 228 M pts/s for nsample / 2, 1 194-1 225 for 2 nsample)
#ifndef LIDAR_BQ_WIN
#define LIDAR_BQ_WIN 1.0
#endif
// the same for queries of ns >= 64, whose windows are ranked by the bitmap (bq_grid.hpp)
#ifndef LIDAR_BQ_WIN_BIG
#define LIDAR_BQ_WIN_BIG 1.0
#endif

namespace {

constexpr int kC = 8;  // centres per wavefront: every loaded 64-point chunk is tested against all

__global__ __launch_bounds__(256) void ball_query_kernel(const float *__restrict__ xyz,
                                                         const float *__restrict__ centres,
                                                         int n, int m, int64_t groups_per_frame,
                                                         int64_t total_groups, float r2, int ns,
                                                         int32_t *__restrict__ out)
{
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gw >= total_groups) return;  // wave-uniform
    const int64_t b = gw / groups_per_frame;
    const int c0 = (int)(gw % groups_per_frame) * kC;
    const int nc = min(kC, m - c0);
    const float *p = xyz + b * (int64_t)n * 3;
    float cx[kC], cy[kC], cz[kC];
    int cnt[kC], first[kC];
#pragma unroll
    for (int j = 0; j < kC; ++j) {
        const int64_t c = b * m + c0 + (j < nc ? j : 0);
        cx[j] = centres[3 * c];
        cy[j] = centres[3 * c + 1];
        cz[j] = centres[3 * c + 2];
        cnt[j] = j < nc ? 0 : ns;  // padding centres start "done"
        first[j] = -1;
    }
    const uint64_t below = (1ull << lane) - 1;
    // the scan is load-latency bound (a wave waits on its chunk ~half the time): the next
    // chunk's 12-byte point is in flight while the current one is tested
    struct P3 {
        float x, y, z;
    };
    const P3 *pp = reinterpret_cast<const P3 *>(p);
    const P3 zero{0.f, 0.f, 0.f};
    // two 64-point chunks per iteration (each lane tests two points against the 8 centres:
    // independent work in flight), the next pair prefetched.  Hand-unrolled: a generic
    // k-chunk loop measured slower (0.96 / 0.93 ms for 2 / 4 chunks vs 0.86, B=32 SA1).
    P3 c0p = lane < n ? pp[lane] : zero, c1p = lane + 64 < n ? pp[lane + 64] : zero;
    for (int base = 0; base < n; base += 128) {
        bool open = false;
#pragma unroll
        for (int j = 0; j < kC; ++j) open |= cnt[j] < ns;
        if (!open) break;  // wave-uniform
        const int k0 = base + lane, k1 = k0 + 64;
        const P3 n0 = k0 + 128 < n ? pp[k0 + 128] : zero, n1 = k1 + 128 < n ? pp[k1 + 128] : zero;
        const P3 a0 = c0p, a1 = c1p;
        c0p = n0;
        c1p = n1;
#pragma unroll
        for (int j = 0; j < kC; ++j) {
            if (cnt[j] >= ns) continue;  // wave-uniform
            const bool h0 = k0 < n && lidar::dist2f(a0.x, a0.y, a0.z, cx[j], cy[j], cz[j]) < r2;
            const bool h1 = k1 < n && lidar::dist2f(a1.x, a1.y, a1.z, cx[j], cy[j], cz[j]) < r2;
            const uint64_t m0 = __ballot(h0), m1 = __ballot(h1);
            if (m0 | m1) {
                int32_t *o = out + (b * m + c0 + j) * (int64_t)ns;
                if (first[j] < 0)
                    first[j] = m0 ? base + __ffsll((unsigned long long)m0) - 1
                                  : base + 64 + __ffsll((unsigned long long)m1) - 1;
                const int r0 = cnt[j] + __popcll(m0 & below);
                const int r1 = cnt[j] + __popcll(m0) + __popcll(m1 & below);  // chunk 1 after chunk 0
                if (h0 && r0 < ns) o[r0] = k0;
                if (h1 && r1 < ns) o[r1] = k1;
                cnt[j] += __popcll(m0) + __popcll(m1);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kC; ++j) {
        if (j >= nc) break;
        int32_t *o = out + (b * m + c0 + j) * (int64_t)ns;
        const int fill = first[j] < 0 ? 0 : first[j];
        for (int s2 = min(cnt[j], ns) + lane; s2 < ns; s2 += 64) o[s2] = fill;
    }
}


// ------------------------------------------------------------------ grid ball query
using namespace lidar_bq;

// Grid parameters of one frame (thread 0 of bq_bin_kernel).
//  * bbox over finite coordinates only: a point with an inf/NaN coordinate is never a hit
//    (its distance is inf or NaN), so where it is binned does not matter.
//  * s >= r (1 + 2^-8): a hit has |p - c| < r (1 + 2^-23) per axis (d < r2 in rounded
//    arithmetic), so |u_p - u_c| < (1 - 2^-8) + the rounding of u = (v - lo) * inv_s,
//    <= 3 * 2^-24 * 1024 (at most 1024 cells per axis): the cells differ by at most 1.
//  * windows: about ns expected hits per window for a uniform frame (LIDAR_BQ_WIN), <= 64 windows.
__device__ BqGrid bin_params(const float mn[3], const float mx[3], int n, float r, int ns)
{
    BqGrid g;
    float ext[3];
    for (int a = 0; a < 3; ++a) {
        const bool none = !(mn[a] <= mx[a]);
        const float lo = none ? 0.f : mn[a];
        float e = none ? 0.f : __fsub_rn(mx[a], lo);
        if (!(e <= 3.0e38f)) e = 3.0e38f;  // overflowed extent
        (&g.minx)[a] = lo;
        ext[a] = e;
    }
    const float emax = fmaxf(ext[0], fmaxf(ext[1], ext[2]));
    const double rr = (r > 0.f && r < 1e30f) ? (double)r : 0.0;
    double vol = 1.0;
    for (int a = 0; a < 3; ++a) vol *= fmax((double)ext[a], 2.0 * rr);
    const double hits = vol > 0.0 ? n * (4.18879020478639 * rr * rr * rr) / vol : (double)n;
    const double wf = ns >= 64 ? LIDAR_BQ_WIN_BIG : LIDAR_BQ_WIN;
    const double want = fmin(64.0, fmax(1.0, wf * hits / (double)max(ns, 1)));
    int shift = 6;
    while (shift < 30 && ((int64_t)n >> shift) > 64) ++shift;                      // <= 64 windows
    while (shift < 30 && (double)(1ll << shift) * want < (double)n) ++shift;       // ~want windows
    g.win_shift = shift;
    g.nwin = (int)(((int64_t)n + (1ll << shift) - 1) >> shift);
    const int cap = kTab / g.nwin;
    float s = fmaxf(fmaxf(__fmul_rn(r, 1.0f + 1.0f / 256.0f), emax / 1023.0f), 1e-30f);
    if (!(s <= 3.0e38f)) s = 3.0e38f;
    int d[3];
    for (int it = 0; it < 200; ++it) {
        const float inv = 1.0f / s;
        int64_t prod = 1;
        for (int a = 0; a < 3; ++a) {
            d[a] = min(1024, (int)floorf(__fmul_rn(ext[a], inv)) + 1);
            prod *= d[a];
        }
        if (prod <= cap) {
            g.inv_s = inv;
            break;
        }
        s = __fmul_rn(s, 1.25f);
    }
    g.dx = d[0];
    g.dy = d[1];
    g.dz = d[2];
    g.ncell = d[0] * d[1] * d[2];
    g.pad[0] = g.pad[1] = 0;
    return g;
}

// one 1024-thread workgroup per frame: finite bbox -> grid -> counting sort by
// (window, cell) into (x, y, z, index) float4s; tab[slot] = first position of the slot
__global__ __launch_bounds__(1024) void bq_bin_kernel(const float *__restrict__ xyz, int n, float r,
                                                      int ns, char *__restrict__ grid_ws)
{
    __shared__ int cnt[kTab];
    __shared__ float red[6][16];
    __shared__ int wsum[16];
    __shared__ BqGrid gs;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t b = blockIdx.x;
    const float *p = xyz + b * (int64_t)n * 3;
    char *fw = grid_ws + b * grid_frame_bytes(n);
    BqGrid *gout = reinterpret_cast<BqGrid *>(fw);
    int *tab = reinterpret_cast<int *>(fw + 64);
    float4 *sorted = reinterpret_cast<float4 *>(fw + 64 + (kTab + 64) * 4);

    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = tid; k < n; k += 1024) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float v = p[3 * (int64_t)k + a];
            if (fabsf(v) <= 3.4e38f) {  // finite
                mn[a] = fminf(mn[a], v);
                mx[a] = fmaxf(mx[a], v);
            }
        }
    }
    for (int i = tid; i < kTab; i += 1024) cnt[i] = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        mn[a] = lidar::wave_min_f(mn[a]);
        mx[a] = lidar::wave_max_f(mx[a]);
    }
    if (lane == 0)
        for (int a = 0; a < 3; ++a) {
            red[a][wid] = mn[a];
            red[3 + a][wid] = mx[a];
        }
    __syncthreads();
    if (tid == 0) {
        float a_mn[3], a_mx[3];
        for (int a = 0; a < 3; ++a) {
            a_mn[a] = red[a][0];
            a_mx[a] = red[3 + a][0];
            for (int w = 1; w < 16; ++w) {
                a_mn[a] = fminf(a_mn[a], red[a][w]);
                a_mx[a] = fmaxf(a_mx[a], red[3 + a][w]);
            }
        }
        gs = bin_params(a_mn, a_mx, n, r, ns);
        *gout = gs;
    }
    __syncthreads();
    const BqGrid g = gs;
    for (int k = tid; k < n; k += 1024) {
        const float *q = p + 3 * (int64_t)k;
        atomicAdd(&cnt[point_slot(q[0], q[1], q[2], k, g)], 1);
    }
    __syncthreads();
    // exclusive scan of the kTab counters: 16 per thread
    int loc[16], sum = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        loc[j] = cnt[tid * 16 + j];
        sum += loc[j];
    }
    int incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d, 64);
        if (lane >= d) incl += v;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int base = incl - sum;
    for (int w = 0; w < wid; ++w) base += wsum[w];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int slot = tid * 16 + j;
        cnt[slot] = base;
        tab[slot] = base;
        base += loc[j];
    }
    if (tid == 1023) tab[kTab] = base;  // == n
    __syncthreads();
    for (int k = tid; k < n; k += 1024) {
        const float *q = p + 3 * (int64_t)k;
        const float x = q[0], y = q[1], z = q[2];
        const int pos = atomicAdd(&cnt[point_slot(x, y, z, k, g)], 1);
        sorted[pos] = make_float4(x, y, z, __int_as_float(k));
    }
}

// one wavefront per centre; blocks are laid out so that the blocks of a contiguous range of
// frames share an XCD (block b and b + 8 share one): a frame's grid stays in one L2
__global__ __launch_bounds__(256) void bq_grid_kernel(const float *__restrict__ xyz,
                                                      const char *__restrict__ grid_ws,
                                                      const float *__restrict__ centres, int n, int m,
                                                      int64_t total, int64_t per_xcd, float r, float r2, int ns,
                                                      int32_t *__restrict__ out)
{
    __shared__ __attribute__((aligned(8))) int hits[4][kCap + 4];  // per wave: a window's hits / bitmap
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t L = blockIdx.x;
    const int64_t w = ((L & 7) * per_xcd + (L >> 3)) * 4 + wid;
    if (w >= total) return;  // wave-uniform
    const int64_t b = w / m;
    const char *fw = grid_ws + b * grid_frame_bytes(n);
    const float *p = xyz + b * (int64_t)n * 3;
    const float cx = centres[3 * w], cy = centres[3 * w + 1], cz = centres[3 * w + 2];
    grid_query_wave<kCap>(p, fw, n, cx, cy, cz, r, r2, ns, lane, hits[wid], out + w * (int64_t)ns);
}

}  // namespace

static int launch_bin(const float *xyz, int64_t batch, int64_t n, float radius, int32_t nsample,
                      char *grid, hipStream_t st)
{
    hipLaunchKernelGGL(bq_bin_kernel, dim3((unsigned)batch), dim3(1024), 0, st, xyz, (int)n, radius,
                       (int)nsample, grid);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

static int launch_grid_query(const float *xyz, const char *grid, const float *centres,
                             int64_t batch, int64_t n, int64_t m, float radius, int32_t nsample, int32_t *idx,
                             hipStream_t st)
{
    const int64_t total = batch * m, blocks = (total + 3) / 4, per_xcd = (blocks + 7) / 8;
    REQUIRE(per_xcd * 8 <= 0x7fffffff, "ball query: too many centres");
    hipLaunchKernelGGL(bq_grid_kernel, dim3((unsigned)(per_xcd * 8)), dim3(256), 0, st, xyz, grid, centres,
                       (int)n, (int)m, total, per_xcd, radius, radius * radius,
                       (int)nsample, idx);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

static int launch_brute(const float *xyz, const float *centres, int64_t batch, int64_t n, int64_t m, float r2,
                        int32_t nsample, int32_t *idx, hipStream_t st)
{
    const int64_t gpf = (m + kC - 1) / kC, groups = batch * gpf;
    const int64_t blocks = (groups + 3) / 4;
    REQUIRE(blocks <= 0x7fffffff, "lidar_ball_query_f32: too many centres");
    hipLaunchKernelGGL(ball_query_kernel, dim3((unsigned)blocks), dim3(256), 0, st, xyz, centres, (int)n,
                       (int)m, gpf, groups, r2, (int)nsample, idx);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

#define BQ_CHECK_ARGS(fn)                                                                    \
    REQUIRE(h && xyz && centres && idx, fn ": null pointer");                               \
    REQUIRE(batch >= 0 && n >= 1 && m >= 0 && nsample >= 1, fn ": bad sizes");               \
    REQUIRE(n < 0x3fffffff && m < 0x7fffffff, fn ": sizes exceed int32");                   \
    REQUIRE(batch <= 0x7fffffff, fn ": batch exceeds int32");                               \
    REQUIRE(radius >= 0.0f, fn ": negative radius")

LIDAR_EXPORT uint64_t lidar_ball_query_grid_bytes(int64_t batch, int64_t n)
{
    return batch <= 0 || n <= 0 ? 0 : (uint64_t)batch * grid_frame_bytes(n);
}

LIDAR_EXPORT int lidar_ball_query_mode_f32(lidar_handle *h, const float *xyz, const float *centres,
                                           int64_t batch, int64_t n, int64_t m, float radius, int32_t nsample,
                                           int32_t mode, int32_t *idx, void *stream)
{
    BQ_CHECK_ARGS("lidar_ball_query_f32");
    REQUIRE(mode >= 0 && mode <= 2, "lidar_ball_query_mode_f32: mode is 0 (auto), 1 (scan) or 2 (grid)");
    if (batch * m == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const float r2 = radius * radius;
    const bool grid = mode == 2 || (mode == 0 && n >= kGridMinN);
    if (!grid) return launch_brute(xyz, centres, batch, n, m, r2, nsample, idx, st);
    char *ws = static_cast<char *>(lidar::workspace(h, lidar_ball_query_grid_bytes(batch, n)));
    if (!ws) return LIDAR_ENOMEM;
    int rc = launch_bin(xyz, batch, n, radius, nsample, ws, st);
    if (rc) return rc;
    return launch_grid_query(xyz, ws, centres, batch, n, m, radius, nsample, idx, st);
}

LIDAR_EXPORT int lidar_ball_query_f32(lidar_handle *h, const float *xyz, const float *centres, int64_t batch,
                                      int64_t n, int64_t m, float radius, int32_t nsample, int32_t *idx,
                                      void *stream)
{
    return lidar_ball_query_mode_f32(h, xyz, centres, batch, n, m, radius, nsample, 0, idx, stream);
}

LIDAR_EXPORT int lidar_ball_query_bin_f32(lidar_handle *h, const float *xyz, int64_t batch, int64_t n,
                                          float radius, int32_t nsample, void *grid, void *stream)
{
    REQUIRE(h && xyz && grid, "lidar_ball_query_bin_f32: null pointer");
    REQUIRE(batch >= 0 && batch <= 0x7fffffff && n >= 1 && n < 0x3fffffff && nsample >= 1,
            "lidar_ball_query_bin_f32: bad sizes");
    REQUIRE(radius >= 0.0f, "lidar_ball_query_bin_f32: negative radius");
    if (batch == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    return launch_bin(xyz, batch, n, radius, nsample, static_cast<char *>(grid),
                      static_cast<hipStream_t>(stream));
}

LIDAR_EXPORT int lidar_ball_query_binned_f32(lidar_handle *h, const float *xyz, const void *grid,
                                             const float *centres, int64_t batch, int64_t n, int64_t m,
                                             float radius, int32_t nsample, int32_t *idx, void *stream)
{
    BQ_CHECK_ARGS("lidar_ball_query_binned_f32");
    REQUIRE(grid, "lidar_ball_query_binned_f32: null grid");
    if (batch * m == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    return launch_grid_query(xyz, static_cast<const char *>(grid), centres, batch, n, m, radius, nsample, idx,
                             static_cast<hipStream_t>(stream));
}
