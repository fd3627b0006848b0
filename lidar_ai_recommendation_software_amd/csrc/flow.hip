// flow.hip — models/crowd_flow_model.py in native host code.  No device work.
//
// Why host: the flow model works on the 1 m grid nodes of a frame's extent (31 x 31 = 961
// for the +-15 m scenes), and every arithmetic step that decides its outputs goes through
// the HOST C library in the reference: np.sin / np.cos / np.float64 ** 2 on numpy scalars
// are glibc sin / cos / pow (pow(x, 2.0) is not x*x: it differs in ~0.1% of inputs), and
// sklearn's KDTree prunes nodes with libm pow(., 2.0) / pow(., 0.5) bounds, which decide
// which lattice neighbours at exactly r = 3 / 5 m are returned.  Reproducing those bit for
// bit means calling the same glibc routines, which a gfx950 kernel cannot; and the whole
// model is ~10^6 flops, below one kernel launch + PCIe round trip.  DESIGN.md §6.
//
//   lidar_flow_field_f64       crowd_flow_model.py:88-184  (_generate_simulated_flow)
//   lidar_flow_bottlenecks_f64 crowd_flow_model.py:186-279 (_identify_bottlenecks), with
//       sklearn's KDTree(positions) (leaf_size 40; build = std::nth_element with the
//       (value, index) comparator of sklearn/neighbors/_partition_nodes.pyx; depth-first
//       query_radius with the min/max node distances of _kd_tree.pyx.tp), so the neighbour
//       ORDER the reference's np.mean and convergence loop see is reproduced as well.
#include <algorithm>
#include <cmath>
#include <vector>

#include "common.hpp"

namespace {

// glibc's own sin / cos / pow, called opaquely: the compiler would otherwise rewrite
// pow(x, 2.0) as x * x (libcall simplification), which is NOT what glibc returns
double (*volatile libm_pow)(double, double) = ::pow;
double (*volatile libm_sin)(double) = ::sin;
double (*volatile libm_cos)(double) = ::cos;

// numpy's pairwise_sum (add.reduce of a contiguous float64 vector of < 8192 elements)
double np_pairwise_sum(const double *a, int64_t n)
{
    if (n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int k = 0; k < 8; ++k) r[k] = a[k];
        int64_t i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; ++k) r[k] += a[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise_sum(a, n2) + np_pairwise_sum(a + n2, n - n2);
}

double np_mean(const std::vector<double> &v)
{
    return np_pairwise_sum(v.data(), (int64_t)v.size()) / (double)v.size();
}

// sklearn KDTree over 2-D (or d-D) float64 rows
struct KDTree {
    const double *x;
    int64_t n, d, n_nodes;
    std::vector<int64_t> idx, s, e;
    std::vector<double> lo, hi;
    std::vector<char> leaf;

    KDTree(const double *x_, int64_t n_, int64_t d_, int64_t leaf_size) : x(x_), n(n_), d(d_)
    {
        const double ratio = (double)(n - 1) / (double)leaf_size;  // Cython true division
        const int64_t levels = (int64_t)(std::log2(std::fmax(1.0, ratio)) + 1.0);
        n_nodes = ((int64_t)1 << levels) - 1;
        idx.resize(n);
        for (int64_t i = 0; i < n; ++i) idx[i] = i;
        s.assign(n_nodes, 0);
        e.assign(n_nodes, 0);
        lo.assign(n_nodes * d, INFINITY);
        hi.assign(n_nodes * d, -INFINITY);
        leaf.assign(n_nodes, 0);
        build(0, 0, n);
    }

    void build(int64_t node, int64_t a, int64_t b)
    {
        s[node] = a;
        e[node] = b;
        for (int64_t i = a; i < b; ++i)
            for (int64_t j = 0; j < d; ++j) {
                lo[node * d + j] = std::fmin(lo[node * d + j], x[idx[i] * d + j]);
                hi[node * d + j] = std::fmax(hi[node * d + j], x[idx[i] * d + j]);
            }
        if (2 * node + 1 >= n_nodes || b - a < 2) {
            leaf[node] = 1;
            return;
        }
        // split dimension: the first of maximal spread (find_node_split_dim)
        int64_t jmax = 0;
        double best = 0.0;
        for (int64_t j = 0; j < d; ++j) {
            double mx = x[idx[a] * d + j], mn = mx;
            for (int64_t i = a + 1; i < b; ++i) {
                mx = std::fmax(mx, x[idx[i] * d + j]);
                mn = std::fmin(mn, x[idx[i] * d + j]);
            }
            if (mx - mn > best) {
                best = mx - mn;
                jmax = j;
            }
        }
        const int64_t mid = (b - a) / 2;
        const double *xx = x;
        const int64_t dd = d;
        std::nth_element(idx.begin() + a, idx.begin() + a + mid, idx.begin() + b, [xx, dd, jmax](int64_t p, int64_t q) {
            const double u = xx[p * dd + jmax], v = xx[q * dd + jmax];
            return u == v ? p < q : u < v;
        });
        build(2 * node + 1, a, a + mid);
        build(2 * node + 2, a + mid, b);
    }

    // query_radius([pt], r)[0] in sklearn's order (depth-first; whole nodes by their bounds)
    void query(int64_t node, const double *pt, double r, std::vector<int64_t> &out) const
    {
        double lb = 0.0, ub = 0.0;
        for (int64_t j = 0; j < d; ++j) {
            const double dlo = lo[node * d + j] - pt[j];
            const double dhi = pt[j] - hi[node * d + j];
            const double dd2 = (dlo + std::fabs(dlo)) + (dhi + std::fabs(dhi));
            lb += libm_pow(0.5 * dd2, 2.0);
            ub += libm_pow(std::fmax(std::fabs(dlo), std::fabs(dhi)), 2.0);
        }
        lb = libm_pow(lb, 0.5);
        ub = libm_pow(ub, 0.5);
        if (lb > r) return;
        if (ub <= r) {
            for (int64_t i = s[node]; i < e[node]; ++i) out.push_back(idx[i]);
            return;
        }
        if (leaf[node]) {
            const double rr = r * r;
            for (int64_t i = s[node]; i < e[node]; ++i) {
                double acc = 0.0;
                for (int64_t j = 0; j < d; ++j) {
                    const double t = pt[j] - x[idx[i] * d + j];
                    acc += t * t;
                }
                if (acc <= rr) out.push_back(idx[i]);
            }
            return;
        }
        query(2 * node + 1, pt, r, out);
        query(2 * node + 2, pt, r, out);
    }
};

}  // namespace

// _generate_simulated_flow (crowd_flow_model.py:88-184) after the host RNG draws: positions
// (nx*ny, 2) = meshgrid(x_grid, y_grid) raveled (row j, column i -> (x_grid[i], y_grid[j]));
// vectors (m, 2) and magnitudes (m) exactly as the reference's per-node numpy-scalar loop
// and its array epilogue compute them.  Host pointers.
LIDAR_EXPORT int lidar_flow_field_f64(const double *x_grid, int64_t nx, const double *y_grid, int64_t ny,
                                      double exit_x, double exit_y, int32_t complexity, const double *bottlenecks,
                                      int32_t nb, double speed_min, double speed_max, double *positions,
                                      double *vectors, double *magnitudes)
{
    REQUIRE(x_grid && y_grid && positions && vectors && magnitudes && (nb == 0 || bottlenecks) && nx >= 1 &&
                ny >= 1 && nb >= 0,
            "lidar_flow_field_f64: bad arguments");
    const int64_t m = nx * ny;
    const double cplx = (double)complexity;
    for (int64_t j = 0; j < ny; ++j)
        for (int64_t i = 0; i < nx; ++i) {
            const int64_t p = j * nx + i;
            const double x = x_grid[i], y = y_grid[j];
            positions[2 * p] = x;
            positions[2 * p + 1] = y;
            double dx = exit_x - x, dy = exit_y - y;
            const double dist = std::sqrt(dx * dx + dy * dy);
            if (dist > 0.0) {
                dx /= dist;
                dy /= dist;
                const double ang = libm_sin(x * cplx) * libm_cos(y * cplx) * 0.5;
                const double c = libm_cos(ang), s = libm_sin(ang);
                vectors[2 * p] = dx * c - dy * s;
                vectors[2 * p + 1] = dx * s + dy * c;
            } else {
                vectors[2 * p] = 0.0;
                vectors[2 * p + 1] = 0.0;
            }
        }
    // bottlenecks (:151-165): every node within 3 m slowed by dist / 3, bottleneck by bottleneck;
    // (x - bx) ** 2 on numpy scalars is libm pow
    for (int32_t k = 0; k < nb; ++k) {
        const double bx = bottlenecks[2 * k], by = bottlenecks[2 * k + 1];
        for (int64_t p = 0; p < m; ++p) {
            const double dist = std::sqrt(libm_pow(positions[2 * p] - bx, 2.0) + libm_pow(positions[2 * p + 1] - by, 2.0));
            if (dist < 3.0) {
                const double f = dist / 3.0;
                vectors[2 * p] *= f;
                vectors[2 * p + 1] *= f;
            }
        }
    }
    // :168-175 (array ** 2 is a plain square on arrays)
    double mx = -INFINITY;
    for (int64_t p = 0; p < m; ++p) {
        magnitudes[p] = std::sqrt(vectors[2 * p] * vectors[2 * p] + vectors[2 * p + 1] * vectors[2 * p + 1]);
        mx = std::fmax(mx, magnitudes[p]);
    }
    const double scale = mx > 0.0 ? (speed_max - speed_min) / mx : 1.0;
    for (int64_t p = 0; p < m; ++p) {
        vectors[2 * p] *= scale;
        vectors[2 * p + 1] *= scale;
        const double v = std::sqrt(vectors[2 * p] * vectors[2 * p] + vectors[2 * p + 1] * vectors[2 * p + 1]);
        magnitudes[p] = v < speed_min ? speed_min : (v > speed_max ? speed_max : v);
    }
    return LIDAR_OK;
}

// _identify_bottlenecks (crowd_flow_model.py:186-279): for every node with magnitude <= slow
// and enough neighbours, the severity the reference computes; candidates with severity > 1
// are written in node order as (x, y, severity = min(10, round-half-even(severity))) — the
// caller sorts them (stable, descending) and keeps 5.  *n_out = number of candidates.
// np.dot / np.linalg.norm of 2-vectors are OpenBLAS ddot: fma(a1, b1, a0 * b0).
LIDAR_EXPORT int lidar_flow_bottlenecks_f64(const double *positions, const double *vectors,
                                            const double *magnitudes, int64_t m, double slow, double r_close,
                                            double r_far, int32_t min_close, int32_t min_far, double *out_x,
                                            double *out_y, int64_t *out_severity, double *out_raw, int64_t cap,
                                            int64_t *n_out)
{
    REQUIRE(positions && vectors && magnitudes && out_x && out_y && out_severity && n_out && m >= 1 && cap >= 0,
            "lidar_flow_bottlenecks_f64: bad arguments");
    KDTree tree(positions, m, 2, 40);
    std::vector<int64_t> close, far;
    std::vector<char> in_close(m, 0);
    std::vector<double> sp;
    int64_t k = 0;
    for (int64_t i = 0; i < m; ++i) {
        if (magnitudes[i] > slow) continue;
        const double *pos = positions + 2 * i;
        close.clear();
        tree.query(0, pos, r_close, close);
        if ((int64_t)close.size() < min_close) continue;
        sp.clear();
        for (int64_t j : close) sp.push_back(magnitudes[j]);
        const double near_mean = np_mean(sp);
        far.clear();
        tree.query(0, pos, r_far, far);
        for (int64_t j : close) in_close[j] = 1;
        std::sort(far.begin(), far.end());
        far.erase(std::unique(far.begin(), far.end()), far.end());
        sp.clear();
        for (int64_t j : far)
            if (!in_close[j]) sp.push_back(magnitudes[j]);
        for (int64_t j : close) in_close[j] = 0;
        if ((int64_t)sp.size() < min_far) continue;
        const double far_mean = np_mean(sp);
        const double grad = far_mean - near_mean;
        double conv = 0.0;
        for (int64_t j : close) {
            double d0 = pos[0] - positions[2 * j], d1 = pos[1] - positions[2 * j + 1];
            const double nrm = std::sqrt(std::fma(d1, d1, d0 * d0));
            if (nrm > 0.0) {
                d0 /= nrm;
                d1 /= nrm;
                const double dot = std::fma(d1, vectors[2 * j + 1], d0 * vectors[2 * j]);
                if (dot > 0.0) conv += dot;
            }
        }
        conv /= (double)close.size();
        const double sev = (grad * 5.0 + conv * 5.0) / 2.0;
        if (sev > 1.0) {
            if (k < cap) {
                out_x[k] = pos[0];
                out_y[k] = pos[1];
                const double rnd = std::nearbyint(sev);  // Python round(): half to even
                out_severity[k] = rnd < 10.0 ? (int64_t)rnd : 10;
                if (out_raw) out_raw[k] = sev;
            }
            ++k;
        }
    }
    *n_out = k;
    return k > cap ? lidar::fail(LIDAR_EINVAL, "lidar_flow_bottlenecks_f64: output capacity exceeded") : LIDAR_OK;
}

// the KDTree(x).get_arrays()[1] permutation (validation hook for the sklearn build replica)
LIDAR_EXPORT int lidar_kdtree_order_f64(const double *x, int64_t n, int32_t d, int32_t leaf_size, int64_t *perm)
{
    REQUIRE(x && perm && n >= 1 && d >= 1 && leaf_size >= 1, "lidar_kdtree_order_f64: bad arguments");
    KDTree tree(x, n, d, leaf_size);
    std::copy(tree.idx.begin(), tree.idx.end(), perm);
    return LIDAR_OK;
}
