// bq_grid.hpp — the grid ball query's per-frame layout and its per-centre query, shared by
// ball_query.hip (bq_bin_kernel / bq_grid_kernel) and the SA1 MLP kernel that answers its own
// ball queries (sa_mlp_x3.hip, sa_x3_kernel with BQ).  See ball_query.hip for the spec.
#pragma once
#include "common.hpp"

namespace lidar_bq {

constexpr int kTab = 16384;     // (window, cell) slots per frame: one int each in LDS (64 KiB)
#ifndef LIDAR_BQ_KCAP
#define LIDAR_BQ_KCAP 512
#endif
constexpr int kCap = LIDAR_BQ_KCAP;  // candidates per window a wavefront ranks in LDS
constexpr int kGridMinN = 1024;  // below this the index-order scan is as cheap

struct BqGrid {  // per frame, written by bq_bin_kernel
    float minx, miny, minz, inv_s;
    int dx, dy, dz, ncell;  // cells per axis; ncell = dx * dy * dz
    int win_shift, nwin;    // windows of 2^win_shift consecutive indices
    int pad[2];
};

// per frame: BqGrid (64 B) | tab[kTab + 64] | sorted float4[n]
__host__ __device__ constexpr uint64_t grid_frame_bytes(int64_t n)
{
    return 64 + (uint64_t)(kTab + 64) * 4 + (uint64_t)n * 16;
}

// cell coordinate of v on one axis; centres may lie outside the bbox (clamped to
// [-2, d+1] before the conversion, NaN -> -2), points inside land in [0, d-1]
__device__ __forceinline__ int cell_of(float v, float lo, float inv_s, int d)
{
    float u = __fmul_rn(__fsub_rn(v, lo), inv_s);
    u = fminf(fmaxf(u, -2.0f), (float)d + 1.0f);
    return (int)floorf(u);
}

__device__ __forceinline__ int point_slot(float x, float y, float z, int k, const BqGrid &g)
{
    const int ix = min(max(cell_of(x, g.minx, g.inv_s, g.dx), 0), g.dx - 1);
    const int iy = min(max(cell_of(y, g.miny, g.inv_s, g.dy), 0), g.dy - 1);
    const int iz = min(max(cell_of(z, g.minz, g.inv_s, g.dz), 0), g.dz - 1);
    return (k >> g.win_shift) * g.ncell + (ix * g.dy + iy) * g.dz + iz;
}

// index-order scan of points [lo, hi) for one centre (a window with too many candidates)
template <class Out>
__device__ __forceinline__ void scan_range(const float *__restrict__ p, int lo, int hi, float cx, float cy,
                                           float cz, float r2, int ns, int lane, uint64_t below, int &cnt,
                                           int &first, Out *o)
{
    for (int k0 = lo; k0 < hi && cnt < ns; k0 += 64) {
        const int k = k0 + lane;
        bool hit = false;
        if (k < hi) hit = lidar::dist2f(p[3 * k], p[3 * k + 1], p[3 * k + 2], cx, cy, cz) < r2;
        const uint64_t mk = __ballot(hit);
        if (mk) {
            if (first < 0) first = k0 + __ffsll((unsigned long long)mk) - 1;
            const int rk = cnt + __popcll(mk & below);
            if (hit && rk < ns) o[rk] = k;
            cnt += __popcll(mk);
        }
    }
}

__device__ __forceinline__ void lds_wave_sync()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// One wavefront answers the ball query of centre (cx, cy, cz) of the frame whose points are p
// (n of them) and whose grid (bq_bin_kernel) is fw: the first ns indices with d < r2 in index
// order into o[0, ns), unused slots repeating the first hit (0 with no hit).  hw: this wave's
// LDS scratch of CAP + 4 ints (8-byte aligned).
//
// A window's hits are put in index order by one of two rankings.  Bitmap (round 6; queries of ns >= 64,
// whose windows hold ~ns hits, and windows of up to 32 CAP indices, i.e. 16 384 at CAP = 512; BM = 0
// compiles it out, for the fused kernels of fewer samples): every hit sets its bit (index - window start) in an LDS
// bitmap (ds_or_b64), then lane l takes 64-bit word c 64 + l, and a popcount, a wave prefix sum and the
// word's own bit order give every hit its rank — O(window / 64) per lane, with no bound on the window's
// candidates.  List (fewer samples, larger windows): the hits go to an LDS list and each is ranked by counting
// the smaller ones, O(hits^2 / 64) per lane, cheaper up to ~64 hits (MSG: the bitmap took its ns = 128 branch's
// fused kernel from 7.95 to 6.96 ms per 96 frames but its ns = 32 one from 1.92 to 2.17); a window with more
// than CAP candidates is then scanned in index order.
// Both give the same indices in the same order (tests/test_gpu_tier_n.py::test_ball_query_*).
template <int CAP, class Out, bool BM = true>
__device__ __forceinline__ void grid_query_wave(const float *__restrict__ p, const char *__restrict__ fw, int n,
                                                float cx, float cy, float cz, float r, float r2, int ns,
                                                int lane, int *hw, Out *o)
{
    const BqGrid g = *reinterpret_cast<const BqGrid *>(fw);
    const int *tab = reinterpret_cast<const int *>(fw + 64);
    const float4 *sp = reinterpret_cast<const float4 *>(fw + 64 + (kTab + 64) * 4);
    const uint64_t below = (1ull << lane) - 1;

    // candidate cells per axis: a hit has |u_p - u_c| < r inv_s (1 + 2^-23) + the rounding of
    // the two cell coordinates (< 2^-12 at <= 1026 cells): floor(u_c -+ delta) bound its cell.
    // At the binned radius that is 3 cells per axis; smaller radii take 1-2.
    const float delta = __fadd_rn(__fmul_rn(__fmul_rn(r, g.inv_s), 1.0f + 1.0f / 1024.0f), 1.0f / 1024.0f);
    const float ux = __fmul_rn(__fsub_rn(cx, g.minx), g.inv_s), uy = __fmul_rn(__fsub_rn(cy, g.miny), g.inv_s),
                uz = __fmul_rn(__fsub_rn(cz, g.minz), g.inv_s);
    auto lo_of = [](float u, float dl, int d) {
        return max((int)floorf(fminf(fmaxf(__fsub_rn(u, dl), -2.0f), (float)d + 1.0f)), 0);
    };
    auto hi_of = [](float u, float dl, int d) {
        return min((int)floorf(fminf(fmaxf(__fadd_rn(u, dl), -2.0f), (float)d + 1.0f)), d - 1);
    };
    // (NaN centres: fmaxf(NaN, -2) = -2 -> an empty range; they have no hits)
    const int lox = lo_of(ux, delta, g.dx), hix = hi_of(ux, delta, g.dx);
    const int loy = lo_of(uy, delta, g.dy), hiy = hi_of(uy, delta, g.dy);
    const int loz = lo_of(uz, delta, g.dz), hiz = hi_of(uz, delta, g.dz);
    int cnt = 0, first = -1;
    // lane j < 9 owns the z-run of column (lox + j / 3, loy + j % 3); a radius above the
    // binned one can need more columns: such centres walk the windows by index-order scan
    const bool full = (hix - lox) > 2 || (hiy - loy) > 2;
    const int jx = lox + lane / 3, jy = loy + lane % 3;
    const bool col_ok = !full && lane < 9 && jx <= hix && jy <= hiy && loz <= hiz;
    const int colbase = (jx * g.dy + jy) * g.dz + loz;
    // the next window's slot-table entries are loaded while the current window is processed,
    // and up to 4 chunks of 64 candidates are loaded before any is tested: about one memory
    // round trip per window instead of one per table read and per candidate chunk
    int st = 0, len = 0;
    if (col_ok && g.nwin > 0) {
        st = tab[colbase];
        len = tab[colbase + (hiz - loz) + 1] - st;
    }
    // the bitmap ranking: 64-bit words of the window's index span in hw
    const bool bitmap = BM && ns >= 64 && !full && ((int64_t)1 << g.win_shift) <= 32 * (int64_t)CAP;
    unsigned long long *bm = reinterpret_cast<unsigned long long *>(hw);
    for (int win = 0; win < g.nwin && cnt < ns; ++win) {
        const int wlo = win << g.win_shift, whi = min(n, (win + 1) << g.win_shift);
        const int cst = st, clen = len;
        if (col_ok && win + 1 < g.nwin) {
            const int s1 = (win + 1) * g.ncell + colbase;
            st = tab[s1];
            len = tab[s1 + (hiz - loz) + 1] - st;
        }
        const int incl = lidar::row_incl_scan_i32(clen);  // lanes 0..8 (row 0): the columns' prefix
        const int tot = full ? CAP + 1 : __builtin_amdgcn_readlane(incl, 8);
        if (tot == 0) continue;
        if (!bitmap && tot > CAP) {
            scan_range(p, wlo, whi, cx, cy, cz, r2, ns, lane, below, cnt, first, o);
            continue;
        }
        const int nwords = (whi - wlo + 63) >> 6;
        if (bitmap) {
            for (int i = lane; i < nwords; i += 64) bm[i] = 0ull;
            lds_wave_sync();
        }
        const int excl = incl - clen;
        int e[9], s[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            e[j] = __builtin_amdgcn_readlane(excl, j);
            s[j] = __builtin_amdgcn_readlane(cst, j);
        }
        int hc = 0;
        for (int t0 = 0; t0 < tot; t0 += 256) {
            float4 qv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = t0 + 64 * u + lane;
                int pos = s[0] + t;
#pragma unroll
                for (int j = 1; j < 9; ++j)
                    if (t >= e[j]) pos = s[j] + (t - e[j]);
                qv[u] = t < tot ? sp[pos] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int t = t0 + 64 * u + lane;
                const bool hit = t < tot && lidar::dist2f(qv[u].x, qv[u].y, qv[u].z, cx, cy, cz) < r2;
                const uint64_t mk = __ballot(hit);
                if (hit) {
                    if (bitmap) {
                        const int o1 = __float_as_int(qv[u].w) - wlo;
                        atomicOr(&bm[o1 >> 6], 1ull << (o1 & 63));
                    } else {
                        hw[hc + __popcll(mk & below)] = __float_as_int(qv[u].w);
                    }
                }
                hc += __popcll(mk);
            }
        }
        if (hc == 0) continue;
        if (bitmap) {
            lds_wave_sync();
            // the window's hits in index order: word c 64 + lane, ranked by the set bits before it
            int base = 0, mnv = 0x7fffffff;
            for (int c0 = 0; c0 < nwords && cnt + base < ns; c0 += 64) {
                const int wi = c0 + lane;
                unsigned long long wd = wi < nwords ? bm[wi] : 0ull;
                const int pc = __popcll(wd);
                const int ex = lidar::wave_incl_scan_i32(pc) - pc;  // hits of the lower words of the chunk
                if (wd) mnv = min(mnv, wlo + 64 * wi + (int)__ffsll(wd) - 1);
                int rk = cnt + base + ex;
                while (wd && rk < ns) {
                    const int j = __ffsll(wd) - 1;
                    o[rk++] = wlo + 64 * wi + j;
                    wd &= wd - 1;
                }
                base += __builtin_amdgcn_readlane(ex + pc, 63);
            }
            if (first < 0) first = (int)lidar::wave_min_u32_dpp((uint32_t)mnv);
            cnt += hc;
            lds_wave_sync();
            continue;
        }
        if (lane < 4) hw[hc + lane] = 0x7fffffff;
        lds_wave_sync();
        // rank every hit by index among the window's hits (indices are distinct)
        int mnv = 0x7fffffff;
        for (int e0 = 0; e0 < hc; e0 += 64) {
            const int ei = e0 + lane;
            const int v = ei < hc ? hw[ei] : 0x7fffffff;
            int rank = 0;
            for (int i = 0; i < hc; i += 4) {
                const int4 h4 = *reinterpret_cast<const int4 *>(hw + i);
                rank += (h4.x < v) + (h4.y < v) + (h4.z < v) + (h4.w < v);
            }
            if (ei < hc && cnt + rank < ns) o[cnt + rank] = v;
            mnv = min(mnv, v);
        }
        if (first < 0) first = (int)lidar::wave_min_u32_dpp((uint32_t)mnv);
        cnt += hc;
        lds_wave_sync();
    }
    const int fill = first < 0 ? 0 : first;
    for (int s2 = min(cnt, ns) + lane; s2 < ns; s2 += 64) o[s2] = fill;
}

}  // namespace lidar_bq
