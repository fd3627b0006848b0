// voxel_grid.hpp — the voxel grid of voxel_downsample: calculate_grid_density's
// grid hash (utils/data_processing.py:305-319) per axis, extended to 3-D.
//
// Per axis, over the frame's own extent lo = min p, hi = max p (float32 widened exactly):
//   edges  = np.arange(lo - 2v, (hi + 2v) + v, v)    the reference's 2-cell margin (:305-309) and
//            arange (:312-313): L = ceil((stop - start) / v) edges, e[0] = start, e[1] = start + v,
//            e[i] = start + i * (e[1] - e[0]) (numpy's DOUBLE_fill)
//   bin(p) = searchsorted(edges, p, 'right') - 1 with p == e[L-1] moved into the last bin, -1 when
//            outside (histogram2d's rule, numpy histogramdd)
// key = (bx * ny + by) * nz + bz over the nx * ny * nz bins.  Summed over z, a frame's voxel counts
// are therefore the reference's own calculate_grid_density histogram of its (x, y) columns
// (tests/golden/gen_voxel.py captures that from the reference).  All arithmetic is float64 with one
// rounding per operation (the library is built with -ffp-contract=off), on the host and the device.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

namespace lidar_vox {

constexpr uint32_t kOutside = 0xffffffffu;  // key of a point outside every bin (sorts last)

struct Axis {
    double start, e1, delta;  // e[0], e[1], e[1] - e[0]
    double inv;               // 1 / delta (rounded: only the guess of `bin` uses it)
    double last;              // e[L - 1], the closed edge
    int64_t nb;               // bins (edges - 1)
};

// false when numpy's arange would not give >= 2 edges (non-finite or degenerate extents) or the
// axis alone has >= 2^32 bins
__host__ __device__ inline bool make_axis(double lo, double hi, double v, Axis &ax)
{
    const double m = v * 2.0;
    const double start = lo - m, stop = (hi + m) + v;
    const double len = ceil((stop - start) / v);
    if (!(len >= 2.0 && len <= 4294967296.0)) return false;
    ax.start = start;
    ax.e1 = start + v;
    ax.delta = ax.e1 - start;
    ax.inv = ax.delta > 0.0 ? 1.0 / ax.delta : 0.0;
    ax.nb = (int64_t)len - 1;
    ax.last = ax.nb == 0 ? start : (ax.nb == 1 ? ax.e1 : start + (double)ax.nb * ax.delta);
    return true;
}

__host__ __device__ inline double edge(const Axis &ax, int64_t i)
{
    return i == 0 ? ax.start : (i == 1 ? ax.e1 : ax.start + (double)i * ax.delta);
}

// e[i] for i in [0, L), -inf below, +inf above: branch-free (selects), the fast path of `bin`
__host__ __device__ inline double edge_or_inf(const Axis &ax, int64_t i, int64_t L)
{
    const uint32_t u = (uint32_t)(i < 0 ? 0 : (i >= L ? 0 : i));  // L - 1 <= 2^32 - 1 (make_axis)
    const double e = ax.start + (double)u * ax.delta;
    const double r = u == 0 ? ax.start : (u == 1 ? ax.e1 : e);
    return i < 0 ? -INFINITY : (i >= L ? INFINITY : r);
}

// histogram2d's bin of p on this axis, -1 outside
__host__ __device__ inline int64_t bin(const Axis &ax, double p)
{
    const int64_t L = ax.nb + 1;
    // c = number of edges <= p (the edges are non-decreasing): guess from the spacing (a multiply
    // by the rounded reciprocal; the guess only has to be within one edge), verify, step one edge
    // down or up when the verification fails (every candidate edge evaluated up front, branch-free:
    // the key launch runs this three times per point), else binary search
    int64_t c = -1;
    if (ax.delta > 0.0) {
        const double g = fmin(fmax(floor((p - ax.start) * ax.inv) + 1.0, 0.0), (double)L);  // NaN -> 0
        const int64_t t = (int64_t)g;
        const double em = edge_or_inf(ax, t - 2, L), ea = edge_or_inf(ax, t - 1, L);
        const double eb = edge_or_inf(ax, t, L), ep = edge_or_inf(ax, t + 1, L);
        c = (ea <= p && p < eb) ? t : ((ea > p && em <= p) ? t - 1 : ((eb <= p && p < ep) ? t + 1 : -1));
    }
    if (c < 0) {
        int64_t lo = 0, hi = L;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (edge(ax, mid) <= p) lo = mid + 1;
            else hi = mid;
        }
        c = lo;
    }
    if (p == ax.last) --c;  // the last edge is closed
    return (c >= 1 && c <= ax.nb) ? c - 1 : -1;
}

struct Grid {
    Axis ax[3];
    bool ok;       // every axis valid and nx * ny * nz < 2^32
    uint64_t keys; // nx * ny * nz
};

__host__ __device__ inline Grid make_grid(const double lo[3], const double hi[3], double v)
{
    Grid g;
    g.ok = true;
    g.keys = 1;
    for (int a = 0; a < 3; ++a) {
        g.ok = g.ok && make_axis(lo[a], hi[a], v, g.ax[a]);
        if (g.ok) g.keys *= (uint64_t)g.ax[a].nb;
        g.ok = g.ok && g.keys < 0xffffffffull;
    }
    return g;
}

// key of point p (kOutside when a coordinate lies outside its axis' bins)
__host__ __device__ inline uint32_t key(const Grid &g, float x, float y, float z)
{
    const int64_t bx = bin(g.ax[0], (double)x), by = bin(g.ax[1], (double)y), bz = bin(g.ax[2], (double)z);
    if (bx < 0 || by < 0 || bz < 0) return kOutside;
    return (uint32_t)(((uint64_t)bx * (uint64_t)g.ax[1].nb + (uint64_t)by) * (uint64_t)g.ax[2].nb + (uint64_t)bz);
}

// ---- the keys launch's float binning (voxel_batch.hip; tests/test_voxel_grid_host.py runs it on the host)
constexpr int kTabEdges = 8192;  // edges per axis of its LDS threshold tables (±200 m at 5 cm)

// The least float >= e: for every float p, p >= e (in float64) <=> p >= ru_float(e), as no float lies
// between e and it — so counting the float thresholds <= p counts the float64 edges <= p.
__host__ __device__ inline float ru_float(double e)
{
    const float f = (float)e;
    if (!((double)f < e)) return f;
    uint32_t u;
    memcpy(&u, &f, 4);
    u = f == 0.0f ? 1u : (f > 0.0f ? u + 1u : u - 1u);  // the next float up (e finite)
    float r;
    memcpy(&r, &u, 4);
    return r;
}

struct FAxis {     // one axis of the float binning
    bool ok;       // <= max_edges edges, a span within the float range: the table applies
    int L;         // edges (the table's length)
    float s0, inv; // the spacing guess: floor((p - s0) inv) ~ the bin
    float lastf;   // e[L - 1] when it is a float (the closed edge), else NaN
};
__host__ __device__ inline FAxis faxis(const Axis &ax, int max_edges)
{
    FAxis f;
    f.ok = ax.nb + 1 <= max_edges && ax.delta > 0.0 && fabs(ax.start) < 1e38 && fabs(ax.last) < 1e38;
    f.L = (int)(ax.nb + 1 < max_edges + 1 ? ax.nb + 1 : max_edges + 1);
    f.s0 = (float)ax.start;
    f.inv = (float)ax.inv;
    f.lastf = (double)(float)ax.last == ax.last ? (float)ax.last : NAN;
    return f;
}

// c = #{i : E[i] <= p} for a finite p from the spacing guess and its neighbouring thresholds, branch-free;
// -1 when the guess is off by more than one bin (bin_tab_search then).  E[-1] = -inf and E[L] = +inf
// (sentinels: the three thresholds are consecutive words, whatever the guess)
__host__ __device__ inline int bin_tab_c(const float *E, int L, float p, float s0, float inv)
{
    const float gf = floorf((p - s0) * inv);
    const int b = (int)fminf(fmaxf(gf, 0.f), (float)(L - 1));  // NaN -> 0
    const float e0 = E[b - 1], e1 = E[b], e2 = E[b + 1];
    return e1 <= p ? (p < e2 ? b + 1 : -1) : (e0 <= p ? b : -1);
}
__host__ __device__ inline int bin_tab_search(const float *E, int L, float p)
{
    int lo = 0, hi = L;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (E[mid] <= p) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// the bin (kOutside outside every bin) from the count c, the last edge closed
__host__ __device__ inline uint32_t bin_of_c(int c, float p, float lastf, int L)
{
    if (p == lastf) --c;
    return (c >= 1 && c <= L - 1) ? (uint32_t)(c - 1) : kOutside;
}

}  // namespace lidar_vox
