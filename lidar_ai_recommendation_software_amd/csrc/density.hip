// density.hip — the reference density path (Tier R) on gfx950, bit-exact with the CPU path.
//
// Replaces, kernel for kernel:
//   preprocess_kernel  utils/data_processing.py:143-195 — height colours, 3-sigma filter
//                      (numpy sequential axis-0 sums), 30th-percentile ground split
//                      (radix select + numpy's _lerp), ground plane (TSQR + Jacobi SVD with gelsd's
//                      rank rule; gelsd is not bit-reproducible, see plane_solve), StandardScaler
//                      (sklearn's corrected two-pass variance, near-constant mask), eps heuristic.
//   dbscan_*           data_processing.py:197 sklearn DBSCAN(eps, min_samples=5):
//                      counting-sort voxel hash (cells > eps, 27-cell stencil), fp64
//                      ((dx*dx+dy*dy)+dz*dz) <= eps*eps counts, union-find over core-core
//                      edges (root = min index), rank by min core index, border = min
//                      adjacent label.  Order-independent: identical to dbscan_inner's DFS.
//   people_kernel      data_processing.py:251-280 per-cluster mean, sequential index-order sums
//   density_kernel     data_processing.py:282-328 + crowd_density_model.py:56-82: np.arange
//                      edges, histogram2d binning, /g^2, cell centres, max, numpy pairwise
//                      mean of the occupied cells, hotspot threshold, stable top-5.
// Sequential sums are one lane each (numpy's axis-0 order is sequential: reproducing it
// bit for bit leaves no freedom); everything else is wave/workgroup parallel.
#include <cmath>

#include "common.hpp"

namespace {

constexpr int kT = 1024;  // threads of the one-workgroup-per-frame kernels
constexpr int kW = kT / 64;

// ------------------------------------------------------------------ scalars layout
enum : int {
    S_NIN = 0, S_NGROUND = 1, S_NNG = 2, S_ZT = 3, S_EPS = 4, S_DIMS = 5,   // 5..10
    S_PLANE = 11,                                                            // 11..14
    S_STATUS = 15, S_MEAN = 16, S_STD = 19, S_SMEAN = 22, S_SSCALE = 25,
    S_SLO = 28, S_SHI = 31, S_CELL = 34, S_CDIM = 35, S_NCELL = 38, S_NCLUST = 39,
    S_PLANE_KIND = 40, S_N = 41, S_MINPTS = 42, S_COUNT = 64
};

// ------------------------------------------------------------------ frame batching
// Every Tier R kernel runs one frame per blockIdx.y.  Frame f's scratch lives at
// f * wss bytes into one workspace allocation (same sub-buffer offsets in every frame),
// its rows of the caller's arrays start at row offs[f] (CSR; offs == nullptr: a single
// frame of the given n), and its scalars at S + f * S_COUNT.
struct FrameMap {
    int64_t wss = 0;
    const int64_t *offs = nullptr;
    template <class T> __device__ __forceinline__ T *ws(T *p) const
    {
        return reinterpret_cast<T *>(reinterpret_cast<uintptr_t>(p) + (uintptr_t)((int64_t)blockIdx.y * wss));
    }
    template <class T> __device__ __forceinline__ T *rows(T *p, int width) const
    {
        return offs ? p + offs[blockIdx.y] * width : p;
    }
    __device__ __forceinline__ int64_t n(int64_t single) const
    {
        return offs ? offs[blockIdx.y + 1] - offs[blockIdx.y] : single;
    }
    template <class T> __device__ __forceinline__ T *scal(T *S) const { return S + (int64_t)blockIdx.y * S_COUNT; }
};

__device__ __forceinline__ double dadd(double a, double b) { return __dadd_rn(a, b); }
__device__ __forceinline__ double dsub(double a, double b) { return __dsub_rn(a, b); }
__device__ __forceinline__ double dmul(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double ddiv(double a, double b) { return __ddiv_rn(a, b); }

// ---- workgroup helpers (1024 threads)
struct BlockScratch {
    double d[6][kW];
    int i[kW + 1];
    unsigned hist[2][256];
    double bc[16];  // broadcast
    double chain[6];  // block_sum_chain results: [accumulator * 3 + column]
};

__device__ double block_min(BlockScratch &s, double v)
{
    for (int m = 32; m >= 1; m >>= 1) v = fmin(v, __shfl_xor(v, m, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s.d[0][threadIdx.x >> 6] = v;
    __syncthreads();
    double r = s.d[0][0];
    for (int w = 1; w < kW; ++w) r = fmin(r, s.d[0][w]);
    return r;
}
__device__ double block_max(BlockScratch &s, double v)
{
    for (int m = 32; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s.d[1][threadIdx.x >> 6] = v;
    __syncthreads();
    double r = s.d[1][0];
    for (int w = 1; w < kW; ++w) r = fmax(r, s.d[1][w]);
    return r;
}
// deterministic (fixed tree) block sum — used only where the reference itself is not
// bit-reproducible (the gelsd plane fit)
__device__ double block_sum(BlockScratch &s, double v, int slot)
{
    for (int m = 32; m >= 1; m >>= 1) v = dadd(v, __shfl_xor(v, m, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s.d[2 + slot][threadIdx.x >> 6] = v;
    __syncthreads();
    double r = s.d[2 + slot][0];
    for (int w = 1; w < kW; ++w) r = dadd(r, s.d[2 + slot][w]);
    return r;
}
// exclusive scan of a 0/1 flag over the workgroup; returns the position, *total set
__device__ int block_flag_scan(BlockScratch &s, bool f, int *total)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t m = __ballot(f);
    const int inwave = __popcll(m & ((1ull << lane) - 1));
    __syncthreads();
    if (lane == 0) s.i[wave] = __popcll(m);
    __syncthreads();
    int base = 0, tot = 0;
    for (int w = 0; w < kW; ++w) {
        int c = s.i[w];
        base += w < wave ? c : 0;
        tot += c;
    }
    *total = tot;
    return base + inwave;
}

// ---- index-order fp64 chains with the rows streamed through LDS
// numpy's axis-0 reductions of a row-major (n, 3) array are sequential per column, so the
// result depends on every rounding in index order.  The rows are staged into LDS in 1024-row
// chunks (double buffered) by the waves that do not run a chain.  Two ways to run a chain:
// block_seq_chain, the dependent adds themselves (lanes 0..2 of wave 0, lane c = column c), for
// sums of signed values (coordinates, deviations: their accumulator wanders across binades near
// zero), and block_sum_chain below, a parallel emulation, for sums of squares.
#ifndef LIDAR_SEQ_ROWS
#define LIDAR_SEQ_ROWS 3072
#endif
// rows per staged chunk: 3 072 (147 KiB double-buffered; the kernel is one 1 024-thread workgroup per CU
// by its registers anyway): preprocess 2.70 ms per 32 frames vs 2.79 at 2 048 and 2.98 at 1 024
// (round-3 A/B): fewer chunk barriers, each waiting on the next chunk's staging
constexpr int kSeqRows = LIDAR_SEQ_ROWS;
// rows whose LDS reads are issued before their dependent adds (32 measured equal, 64 slower: the
// chain is bound by the dependent fp64 adds, not by the LDS reads)
constexpr int kSeqBatch = 16;
struct SeqStage {
    double v[2][kSeqRows * 3];
};

// one staged chunk's rows of the index-order chain of column c (lane c of wave 0): b = the chunk's column c
template <class Step>
__device__ __forceinline__ void seq_chain_rows(const double *b, int rows, int c, Step step, double &a0, double &a1)
{
    // reads of a 16-row batch first, then its dependent adds (an explicit two-batch
    // software pipeline measured 2.4x slower: 7.6 vs 3.2 ms per 65k frame)
    int i = 0;
    for (; i + kSeqBatch <= rows; i += kSeqBatch) {
        double v[kSeqBatch];
#pragma unroll
        for (int u = 0; u < kSeqBatch; ++u) v[u] = b[3 * (i + u)];
#pragma unroll
        for (int u = 0; u < kSeqBatch; ++u) step(c, v[u], a0, a1);
    }
    for (; i < rows; ++i) step(c, b[3 * i], a0, a1);
}

template <class Step>
__device__ void block_seq_chain(const double *x, int64_t n, SeqStage &st, Step step, double &a0, double &a1)
{
    const int tid = threadIdx.x;
    const int64_t nch = (n + kSeqRows - 1) / kSeqRows;
    auto stage = [&](int64_t k) {
        if (tid < 64 || k >= nch) return;  // wave 0 never waits on global loads
        const int64_t r0 = k * kSeqRows;
        const int64_t cnt = (n - r0 < kSeqRows ? n - r0 : kSeqRows) * 3;
        double *d = st.v[k & 1];
        const double *src = x + 3 * r0;
        for (int64_t e = tid - 64; e < cnt; e += kT - 64) d[e] = src[e];
    };
    stage(0);
    __syncthreads();
    for (int64_t k = 0; k < nch; ++k) {
        stage(k + 1);
        if (tid < 3) {
            const int64_t r0 = k * kSeqRows;
            const int rows = (int)(n - r0 < kSeqRows ? n - r0 : kSeqRows);
            seq_chain_rows(st.v[k & 1] + tid, rows, tid, step, a0, a1);
        }
        __syncthreads();
    }
}

// ---- the same index-order chains, emulated in parallel, bit for bit
// A chain a <- fl(a + inc_i) (i = 0..n-1, a = +0.0 first) is reproduced without n dependent adds.
// While a stays in one binade [2^e, 2^(e+1)) (or its negative), with u = 2^(e-52), every partial
// result is a multiple of u, and fl(a + v) = a + u * rint(v / u) as long as the exact sum stays in
// that binade and v / u is not an exact tie (the tie goes to the even neighbour, which depends on a).
// So a wavefront takes 256 rows at a time (4 consecutive rows per lane): every row's increment is
// scaled to k = rint(inc * 2^(53-E)) (a = m 2^E, 0.5 <= |m| < 1: exact power-of-two scaling), a
// lane-local prefix plus a DPP scan of the lane totals (integers of at most 2^44 each, so every
// partial sum is exact in fp64) gives A_j = A + P_j, and the rows up to the first one whose A_j
// leaves (2^52, 2^53) in magnitude, or whose increment is a tie, huge (> 2^44 u), inf or NaN, are
// accepted at once: a = A_j * u.  The violating row is added with one
// dadd, exactly as the sequential chain does, and the scan restarts after it.  Near zero (a = 0,
// subnormal, non-finite) the rows go one dadd at a time; after a scan accepts fewer than
// kChainMinRun rows (an accumulator hovering near a binade edge, as a centred column's sum does),
// the next kChainSeqRun rows go one dadd at a time before the next scan.  Every accepted row has the
// value the dependent add would have produced, so the result is the sequential one bit for bit
// (tests/test_gpu_tier_r.py: the reference's goldens, byte-equal).
constexpr int kChainMinRun = 16, kChainSeqRun = 32, kChainRowsPerLane = 4;

// wave-uniform fp64 helpers (scalar registers: the chain's control flow stays scalar)
__device__ __forceinline__ double readlane_d(double v, int l)
{
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double uniform_d(double v)
{
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// DPP move of an fp64 value (both halves), 0 where the row / bank masks or the row bounds leave
// a lane without a source
template <int CTRL, int RM, bool BC>
__device__ __forceinline__ double dpp_d(double v)
{
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, RM, 0xf, BC);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, RM, 0xf, BC);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// inclusive wave scan of integer-valued doubles whose partial sums stay below 2^53 (exact):
// row_shr 1 / 2 / 4 / 8 within each 16-lane row, then row_bcast 15 (rows 1, 3) and 31 (rows 2, 3)
__device__ __forceinline__ double wave_scan_exact_d(double P)
{
    P = dadd(P, dpp_d<0x111, 0xf, true>(P));
    P = dadd(P, dpp_d<0x112, 0xf, true>(P));
    P = dadd(P, dpp_d<0x114, 0xf, true>(P));
    P = dadd(P, dpp_d<0x118, 0xf, true>(P));
    P = dadd(P, dpp_d<0x142, 0xa, false>(P));
    P = dadd(P, dpp_d<0x143, 0xc, false>(P));
    return P;
}

// chain (column c = wave % 3, accumulator q = wave / 3) of rows [0, n) of x (row-major (n, 3)):
// a_q[c] <- fl(a_q[c] + inc(c, q, x[i][c])).  Waves 0 .. 3 NQ - 1 run the chains; the other waves
// stage 1024-row chunks into LDS (double buffered).  Results land in s.chain[q * 3 + c] (ends with
// a barrier).
// one staged chunk's rows of the emulated chain a <- fl(a + inc(c, q, x_i[c])) (one wavefront; b = the chunk's
// column c; a and forced carry over from chunk to chunk)
template <class Inc>
__device__ __forceinline__ void sum_chain_rows(const double *b, int rows, int c, int q, Inc inc, double &a, int &forced)
{
    constexpr double kTwo52 = 4503599627370496.0, kTwo53 = 9007199254740992.0, kTwo44 = 17592186044416.0;
    const int lane = threadIdx.x & 63;
    int i = 0;
    while (i < rows) {
        a = uniform_d(a);
        i = __builtin_amdgcn_readfirstlane(i);
        forced = __builtin_amdgcn_readfirstlane(forced);
        if (forced > 0 || !(fabs(a) >= 2.2250738585072014e-308) || !(fabs(a) < INFINITY)) {
            // one dadd per row (wave-uniform): near zero, non-finite, or a forced run
            const int run = forced > 0 ? (forced < rows - i ? forced : rows - i) : 1;
            int t = 0;
            for (; t + 8 <= run; t += 8) {
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = inc(c, q, b[3 * (i + t + u)]);
#pragma unroll
                for (int u = 0; u < 8; ++u) a = dadd(a, v[u]);
            }
            for (; t < run; ++t) a = dadd(a, inc(c, q, b[3 * (i + t)]));
            i += run;
            forced = forced > run ? forced - run : 0;
            continue;
        }
        int e2;
        (void)frexp(a, &e2);  // a = m 2^e2, 0.5 <= |m| < 1
        const int sh = __builtin_amdgcn_readfirstlane(53 - e2);
        const double A = ldexp(a, sh);  // |A| in [2^52, 2^53), exact
        // lane l takes rows i + 4l .. i + 4l + 3: a window of 256 rows per scan
        double v[kChainRowsPerLane], L[kChainRowsPerLane], raw[kChainRowsPerLane];
        bool bad[kChainRowsPerLane], valid[kChainRowsPerLane];
        double run = 0.0;  // the lane's own prefix of its rounded increments
        // the window's LDS reads all issued first and unconditionally (rows past the end read row i, and
        // their values are dropped below): one wait, not one branch and wait per row
#pragma unroll
        for (int r = 0; r < kChainRowsPerLane; ++r) {
            const int j = i + kChainRowsPerLane * lane + r;
            valid[r] = j < rows;
            raw[r] = b[3 * (valid[r] ? j : i)];
        }
#pragma unroll
        for (int r = 0; r < kChainRowsPerLane; ++r) {
            v[r] = valid[r] ? inc(c, q, raw[r]) : 0.0;
            const double xs = ldexp(v[r], sh);
            double kq = rint(xs);
            bad[r] = valid[r] && (!(fabs(kq) <= kTwo44) || dsub(xs, floor(xs)) == 0.5);
            if (!valid[r] || bad[r]) kq = 0.0;
            run = dadd(run, kq);  // integers below 2^46: exact
            L[r] = run;
        }
        // exclusive prefix of the lane totals (<= 256 increments of <= 2^44: below 2^52, exact)
        const double E = dsub(wave_scan_exact_d(run), run);
        int first = kChainRowsPerLane;  // the lane's first violating row
#pragma unroll
        for (int r = kChainRowsPerLane - 1; r >= 0; --r) {
            const double Aj = dadd(A, dadd(E, L[r]));  // exact below 2^53; >= 2^53 stays
            const double sAj = a > 0.0 ? Aj : -Aj;
            if (valid[r] && (bad[r] || !(sAj > kTwo52 && sAj < kTwo53))) first = r;
        }
        const uint64_t vm = __ballot(first < kChainRowsPerLane);
        const int nv = rows - i < 64 * kChainRowsPerLane ? rows - i : 64 * kChainRowsPerLane;
        // the accumulator after the rows before window row t (t >= 1), and row t's increment
        // (the row choices read every candidate out of lane ln and select among the scalars: a select of
        // per-row registers with a runtime row made the compiler keep L[] and v[] in scratch memory)
        auto pick_at = [&](const double (&arr)[kChainRowsPerLane], int ln, int r) {
            double p = readlane_d(arr[0], ln);
#pragma unroll
            for (int u = 1; u < kChainRowsPerLane; ++u) {
                const double x = readlane_d(arr[u], ln);
                p = r == u ? x : p;
            }
            return p;
        };
        auto after = [&](int t) {
            const int ln = (t - 1) / kChainRowsPerLane, r = (t - 1) % kChainRowsPerLane;
            return ldexp(dadd(A, dadd(readlane_d(E, ln), pick_at(L, ln, r))), -sh);
        };
        if (vm == 0) {
            a = after(nv);
            i += nv;
        } else {
            const int ln = __builtin_amdgcn_readfirstlane(__ffsll((unsigned long long)vm) - 1);
            const int rv = __builtin_amdgcn_readlane(first, ln);
            const int j0 = kChainRowsPerLane * ln + rv;
            if (j0 > 0) a = after(j0);
            a = dadd(a, pick_at(v, ln, rv));  // the violating row: the sequential add itself
            i += j0 + 1;
            if (j0 < kChainMinRun) forced = kChainSeqRun;
        }
    }
}

template <int NQ, class Inc>
__device__ void block_sum_chain(const double *x, int64_t n, SeqStage &st, BlockScratch &s, Inc inc)
{
    constexpr int kCW = 3 * NQ;  // chain waves
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t nch = (n + kSeqRows - 1) / kSeqRows;
    auto stage = [&](int64_t k) {
        if (wave < kCW || k >= nch) return;  // the chain waves never wait on global loads
        const int64_t r0 = k * kSeqRows;
        const int64_t cnt = (n - r0 < kSeqRows ? n - r0 : kSeqRows) * 3;
        double *d = st.v[k & 1];
        const double *src = x + 3 * r0;
        for (int64_t e = tid - 64 * kCW; e < cnt; e += kT - 64 * kCW) d[e] = src[e];
    };
    const int c = wave % 3, q = wave / 3;
    double a = 0.0;
    int forced = 0;
    stage(0);
    __syncthreads();
    for (int64_t k = 0; k < nch; ++k) {
        stage(k + 1);
        if (wave < kCW) {
            const int64_t r0 = k * kSeqRows;
            const int rows = (int)(n - r0 < kSeqRows ? n - r0 : kSeqRows);
            const double *b = st.v[k & 1] + c;
            sum_chain_rows(b, rows, c, q, inc, a, forced);
        }
        __syncthreads();
    }
    if (wave < kCW && lane == 0) s.chain[q * 3 + c] = a;
    __syncthreads();
}

// both kinds at once over the same staged rows: the index-order chain `step` (lanes 0..2 of wave 0, as
// block_seq_chain) and the emulated chain of `inc` (waves 1..3, column = wave - 1, as block_sum_chain with
// NQ = 1, result in s.chain[column]); waves 4.. stage.  One pass instead of two, or instead of a step
// carrying both: the StandardScaler's second pass (its correction sum stays sequential, its sum of
// squared deviations is emulated beside it)
template <class Step, class Inc>
__device__ void block_seq_sum_chain(const double *x, int64_t n, SeqStage &st, BlockScratch &s, Step step, double &a0,
                                    double &a1, Inc inc)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t nch = (n + kSeqRows - 1) / kSeqRows;
    auto stage = [&](int64_t k) {
        if (wave < 4 || k >= nch) return;
        const int64_t r0 = k * kSeqRows;
        const int64_t cnt = (n - r0 < kSeqRows ? n - r0 : kSeqRows) * 3;
        double *d = st.v[k & 1];
        const double *src = x + 3 * r0;
        for (int64_t e = tid - 256; e < cnt; e += kT - 256) d[e] = src[e];
    };
    const int c = wave >= 1 && wave <= 3 ? wave - 1 : 0;
    double a = 0.0;
    int forced = 0;
    stage(0);
    __syncthreads();
    for (int64_t k = 0; k < nch; ++k) {
        stage(k + 1);
        const int64_t r0 = k * kSeqRows;
        const int rows = (int)(n - r0 < kSeqRows ? n - r0 : kSeqRows);
        if (wave == 0) {
            if (tid < 3) seq_chain_rows(st.v[k & 1] + tid, rows, tid, step, a0, a1);
        } else if (wave <= 3) {
            sum_chain_rows(st.v[k & 1] + c, rows, c, 0, inc, a, forced);
        }
        __syncthreads();
    }
    if (wave >= 1 && wave <= 3 && lane == 0) s.chain[c] = a;
    __syncthreads();
}

// ---- ground plane: numpy.linalg.lstsq(A, z, rcond=None), A = [x y 1] (data_processing.py:171-177)
// LAPACK gelsd returns the minimum-norm least-squares solution of A's SVD truncated at
// rcond = eps * max(M, 3): singular values s_i <= rcond * s_1 count as zero.  That decision is what
// makes a frame far from the origin (|x| ~ 1e12 with a unit spread) or at tiny magnitudes (1e-140)
// rank-deficient, and the truncated solution differs there from the plain least-squares plane.
// The device reproduces the decision and the solution: (1) a Givens QR of the centred rows
// w = [(x - mx) sx, (y - my) sx, 1, (z - mz) sz] (sx, sz powers of two: no overflow, exact
// unscaling), per thread over its rows, then merged as a fixed tree (TSQR); (2) since
// [x y 1] = [x - mx, y - my, 1] T with T = [[1,0,0],[0,1,0],[mx,my,1]], A = Q (R3 T) and Q^T z =
// R[:3,3] + mz R[:3,2], so A's singular values and the solution are those of the 3x3 system
// B = R3 T, c; (3) one-sided Jacobi SVD of B (high relative accuracy), the same rank rule, and
// x = sum over the kept i of v_i (u_i . c) / s_i.  The centring perturbs A far less than gelsd's own
// backward error, so the result agrees with gelsd to ~eps * s_1 / s_rank relative (both are
// backward-stable solvers of the same truncated problem); tests/test_gpu_tier_r.py states that
// tolerance.  Row 3 of R (the residual) is not needed and not formed.
__device__ __forceinline__ constexpr int plane_ro(int k) { return k == 0 ? 0 : k == 1 ? 4 : k == 2 ? 7 : 9; }
template <int K0>
__device__ __forceinline__ void plane_row(double (&r)[10], double (&w)[4])
{
#pragma unroll
    for (int k = K0; k < 3; ++k) {
        const double a = r[plane_ro(k)], b = w[k];
        const double h = __dsqrt_rn(dadd(dmul(a, a), dmul(b, b)));
        const bool skip = b == 0.0 || h == 0.0;  // h == 0: b's square underflowed (negligible)
        const double inv = skip ? 0.0 : ddiv(1.0, h);
        const double c = skip ? 1.0 : dmul(a, inv), s = skip ? 0.0 : dmul(b, inv);
        r[plane_ro(k)] = skip ? a : h;
#pragma unroll
        for (int j = k + 1; j < 4; ++j) {
            const double t = r[plane_ro(k) + j - k];
            r[plane_ro(k) + j - k] = dadd(dmul(c, t), dmul(s, w[j]));
            w[j] = dsub(dmul(c, w[j]), dmul(s, t));
        }
    }
}
__device__ __forceinline__ void plane_merge(double (&r)[10], const double (&p)[10])
{
    double w0[4] = {p[0], p[1], p[2], p[3]};
    plane_row<0>(r, w0);
    double w1[4] = {0.0, p[4], p[5], p[6]};
    plane_row<1>(r, w1);
    double w2[4] = {0.0, 0.0, p[7], p[8]};
    plane_row<2>(r, w2);
}
// the truncated minimum-norm solution from the merged R (one thread); returns the rank
__device__ int plane_solve(const double (&r)[10], double sx_inv_exp, double sz_inv_exp, double mx, double my,
                           double mz, double m_rows, double (&x)[3])
{
    auto R = [&](int i, int j) { return j < i ? 0.0 : r[plane_ro(i) + j - i]; };
    const int ex = (int)sx_inv_exp, ez = (int)sz_inv_exp;
    double B[3][3], c[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        B[i][0] = dadd(ldexp(R(i, 0), ex), dmul(R(i, 2), mx));
        B[i][1] = dadd(ldexp(R(i, 1), ex), dmul(R(i, 2), my));
        B[i][2] = R(i, 2);
        c[i] = dadd(ldexp(R(i, 3), ez), dmul(mz, R(i, 2)));
    }
    double bm = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) bm = fmax(bm, fabs(B[i][j]));
    int eb = 0;
    if (bm > 0.0 && bm < INFINITY) (void)frexp(bm, &eb);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        c[i] = ldexp(c[i], -eb);
#pragma unroll
        for (int j = 0; j < 3; ++j) B[i][j] = ldexp(B[i][j], -eb);
    }
    double V[3][3] = {{1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {0.0, 0.0, 1.0}};
    constexpr double kEps = 2.220446049250313e-16;  // numpy.finfo(float64).eps
    for (int sweep = 0; sweep < 40; ++sweep) {
        bool rot = false;
#pragma unroll
        for (int pq = 0; pq < 3; ++pq) {
            const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
            double al = 0.0, be = 0.0, ga = 0.0;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                al = dadd(al, dmul(B[i][p], B[i][p]));
                be = dadd(be, dmul(B[i][q], B[i][q]));
                ga = dadd(ga, dmul(B[i][p], B[i][q]));
            }
            if (ga == 0.0 || fabs(ga) <= dmul(kEps, dmul(__dsqrt_rn(al), __dsqrt_rn(be)))) continue;
            rot = true;
            const double zeta = ddiv(dsub(be, al), dmul(2.0, ga));
            const double t = fabs(zeta) > 1e150 ? ddiv(0.5, zeta)
                                                : ddiv(copysign(1.0, zeta),
                                                       dadd(fabs(zeta), __dsqrt_rn(dadd(1.0, dmul(zeta, zeta)))));
            const double cs = ddiv(1.0, __dsqrt_rn(dadd(1.0, dmul(t, t)))), sn = dmul(cs, t);
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const double bp = B[i][p], bq = B[i][q];
                B[i][p] = dsub(dmul(cs, bp), dmul(sn, bq));
                B[i][q] = dadd(dmul(sn, bp), dmul(cs, bq));
                const double vp = V[i][p], vq = V[i][q];
                V[i][p] = dsub(dmul(cs, vp), dmul(sn, vq));
                V[i][q] = dadd(dmul(sn, vp), dmul(cs, vq));
            }
        }
        if (!rot) break;
    }
    double s2[3], sv[3], smax = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        s2[k] = dadd(dadd(dmul(B[0][k], B[0][k]), dmul(B[1][k], B[1][k])), dmul(B[2][k], B[2][k]));
        sv[k] = __dsqrt_rn(s2[k]);
        smax = fmax(smax, sv[k]);
    }
    const double tol = dmul(dmul(kEps, fmax(m_rows, 3.0)), smax);  // numpy: rcond = eps * max(M, N)
    int rank = 0;
    x[0] = x[1] = x[2] = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const bool keep = sv[k] > tol;
        rank += keep ? 1 : 0;
        const double coef = keep ? ddiv(dadd(dadd(dmul(B[0][k], c[0]), dmul(B[1][k], c[1])), dmul(B[2][k], c[2])), s2[k])
                                 : 0.0;
#pragma unroll
        for (int i = 0; i < 3; ++i) x[i] = keep ? dadd(x[i], dmul(V[i][k], coef)) : x[i];
    }
    return rank;
}

__device__ __forceinline__ uint64_t ordkey(double v)
{
    uint64_t u = (uint64_t)__double_as_longlong(v);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double unordkey(uint64_t k)
{
    uint64_t u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)u);
}


// ------------------------------------------------------------------ preprocess
// LIDAR_PRE_DIAG builds (tools/micro/pre_phases.py only): shader-clock stamps of the sections
// A..I into the frame's scalars 48..57 (cycles since the kernel start)
#ifdef LIDAR_PRE_DIAG
#define PRE_STAMP(k)                                                                   \
    do {                                                                               \
        __syncthreads();                                                               \
        if (threadIdx.x == 0) S[48 + (k)] = (double)(clock64() - pre_t0);              \
    } while (0)
#else
#define PRE_STAMP(k) \
    do {             \
    } while (0)
#endif
__global__ __launch_bounds__(kT) void preprocess_kernel(const double *__restrict__ xyz_in, int64_t n_in,
                                                        uint8_t *__restrict__ mask_in,
                                                        double *__restrict__ colors_in,
                                                        double *__restrict__ normals_in,
                                                        double *__restrict__ comp_in,
                                                        double *__restrict__ sc_in,
                                                        int32_t *__restrict__ ng_pos_in,
                                                        double *__restrict__ S_in, FrameMap fm,
                                                        double fixed_eps)
{
    __shared__ BlockScratch s;
    __shared__ SeqStage st;
    const int tid = threadIdx.x;
    const int64_t n = fm.n(n_in);
    const double *xyz = fm.rows(xyz_in, 3);
    uint8_t *mask = fm.rows(mask_in, 1);
    double *colors = fm.rows(colors_in, 3), *normals = fm.rows(normals_in, 3), *comp = fm.rows(comp_in, 3);
    double *sc = fm.ws(sc_in);
    int32_t *ng_pos = fm.ws(ng_pos_in);
    double *S = fm.scal(S_in);
#ifdef LIDAR_PRE_DIAG
    const long long pre_t0 = clock64();
#endif
    if (n == 0) {  // an empty frame of a batch: the reference raises ValueError (status 2)
        if (tid == 0) S[S_STATUS] = 2.0;
        return;
    }

    PRE_STAMP(0);
    // ---- A: colours over ALL points (data_processing.py:143-147)
    double lo = INFINITY, hi = -INFINITY;
    for (int64_t i = tid; i < n; i += kT) {
        const double z = xyz[3 * i + 2];
        lo = fmin(lo, z);
        hi = fmax(hi, z);
    }
    const double zmin = block_min(s, lo), zmax = block_max(s, hi);
    const double denom = dadd(dsub(zmax, zmin), 1e-10);

    PRE_STAMP(1);
    // ---- B: mean / std with numpy's sequential axis-0 sums (:151-152)
    {
        double sum = 0.0, unused = 0.0;
        block_seq_chain(xyz, n, st, [](int, double v, double &a, double &) { a = dadd(a, v); }, sum, unused);
        if (tid < 3) s.bc[tid] = ddiv(sum, (double)n);
        __syncthreads();
        const double mw = s.bc[(tid >> 6) % 3];  // the mean of this wave's chain column
        block_sum_chain<1>(xyz, n, st, s, [mw](int, int, double v) {
            const double d = dsub(v, mw);
            return dmul(d, d);
        });
        if (tid < 3) s.bc[3 + tid] = __dsqrt_rn(ddiv(s.chain[tid], (double)n));
    }
    __syncthreads();
    double mean[3], thr[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        mean[c] = s.bc[c];
        thr[c] = dmul(3.0, s.bc[3 + c]);
    }
    if (tid < 3) {
        S[S_MEAN + tid] = mean[tid];
        S[S_STD + tid] = s.bc[3 + tid];
    }

    PRE_STAMP(2);
    // ---- C: strict 3-sigma mask, order-preserving compaction (:155-157)
    int64_t nin = 0;
    for (int64_t b0 = 0; b0 < n; b0 += kT) {
        const int64_t i = b0 + tid;
        bool f = false;
        double p[3] = {0, 0, 0};
        if (i < n) {
            f = true;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                p[c] = xyz[3 * i + c];
                f = f && (fabs(dsub(p[c], mean[c])) < thr[c]);
            }
            mask[i] = f ? 1 : 0;
        }
        int tot;
        const int pos = block_flag_scan(s, f, &tot);
        if (f) {
            const int64_t o = nin + pos;
#pragma unroll
            for (int c = 0; c < 3; ++c) comp[3 * o + c] = p[c];
            // colours of the inliers (:143-147, masked at :157), normals (:160-161)
            const double nh = ddiv(dsub(p[2], zmin), denom);
            colors[3 * o] = nh;
            colors[3 * o + 1] = dmul(0.5, dsub(1.0, nh));
            colors[3 * o + 2] = 0.5;
            normals[3 * o] = 0.0;
            normals[3 * o + 1] = 0.0;
            normals[3 * o + 2] = 1.0;
        }
        nin += tot;
    }
    if (tid == 0) {
        S[S_NIN] = (double)nin;
        S[S_STATUS] = nin == 0 ? 1.0 : 0.0;
        S[S_N] = (double)n;
    }
    if (nin == 0) return;  // reference: IndexError from np.percentile on an empty array
    __threadfence_block();
    __syncthreads();

    PRE_STAMP(3);
    // ---- D: z threshold = np.percentile(z, 30) 'linear' (:164)
    const double q = ddiv(30.0, 100.0);
    const double v = dmul((double)(nin - 1), q);
    const double prev = floor(v);
    int64_t klo, khi;
    if (v >= (double)(nin - 1)) {
        klo = khi = nin - 1;
    } else {
        klo = (int64_t)prev;
        khi = klo + 1;
    }
    double za, zb;
    {
        // z column of the compacted points, strided view
        // (select reads comp[3*i+2] through a small lambda-free loop)
        uint64_t pre[2] = {0, 0};
        int64_t kk[2] = {klo, khi};
        // per-wave histograms (16 waves x 2 targets x 256 bins) in the chain staging memory, idle
        // here: the early digits of a coordinate column share a few values, and one shared
        // histogram serialised every wave's atomics on them
        unsigned *wh = reinterpret_cast<unsigned *>(&st.v[0][0]);
        static_assert(sizeof(SeqStage) >= kW * 2 * 256 * sizeof(unsigned), "per-wave histograms");
        const int lane = tid & 63, wave = tid >> 6;
        for (int pass = 0; pass < 8; ++pass) {
            const int shift = 56 - 8 * pass;
            for (int i = tid; i < kW * 2 * 256; i += kT) wh[i] = 0;
            __syncthreads();
            unsigned *mine = wh + wave * 2 * 256;
            for (int64_t i = tid; i < nin; i += kT) {
                const uint64_t key = ordkey(comp[3 * i + 2]);
                const uint64_t hk = pass == 0 ? 0 : key >> (shift + 8);
                const unsigned dig = (unsigned)(key >> shift) & 255u;
                if (hk == pre[0]) atomicAdd(&mine[dig], 1u);
                if (hk == pre[1]) atomicAdd(&mine[256 + dig], 1u);
            }
            __syncthreads();
            if (tid < 512) {
                unsigned sum = 0;
                for (int w = 0; w < kW; ++w) sum += wh[w * 512 + tid];
                (&s.hist[0][0])[tid] = sum;
            }
            __syncthreads();
            if (wave < 2) {  // wave r selects target r: the first bin whose running count passes kk[r]
                const int r = wave;
                unsigned h[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) h[j] = s.hist[r][4 * lane + j];
                const int64_t loc = (int64_t)h[0] + h[1] + h[2] + h[3];
                int64_t incl = loc;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int64_t t = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += t;
                }
                int64_t cum = incl - loc;
                int d = -1;
                int64_t before = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (d < 0 && cum + h[j] > kk[r]) {
                        d = 4 * lane + j;
                        before = cum;
                    }
                    cum += h[j];
                }
                const uint64_t hit = __ballot(d >= 0);
                const int wl = hit ? __ffsll((unsigned long long)hit) - 1 : 63;
                const int dsel = hit ? __shfl(d, wl, 64) : 256;
                const int64_t bsel = hit ? __shfl(before, wl, 64) : __shfl(cum, 63, 64);
                if (lane == 0) {
                    s.d[4 + r][0] = __longlong_as_double((long long)((pre[r] << 8) | (uint64_t)dsel));
                    s.d[4 + r][1] = __longlong_as_double((long long)(kk[r] - bsel));
                }
            }
            __syncthreads();
            for (int r = 0; r < 2; ++r) {
                pre[r] = (uint64_t)__double_as_longlong(s.d[4 + r][0]);
                kk[r] = (int64_t)__double_as_longlong(s.d[4 + r][1]);
            }
            __syncthreads();
        }
        za = unordkey(pre[0]);
        zb = unordkey(pre[1]);
    }
    const double t = dsub(v, prev);
    const double diff = dsub(zb, za);
    double zt = dadd(za, dmul(diff, t));
    if (t >= 0.5) zt = dsub(zb, dmul(diff, dsub(1.0, t)));

    PRE_STAMP(4);
    // ---- E: ground count and plane (:165-183)
    double cnt = 0, sx = 0, sy = 0, sz = 0, imin[3] = {INFINITY, INFINITY, INFINITY},
           imax[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = tid; i < nin; i += kT) {
        const double px = comp[3 * i], py = comp[3 * i + 1], pz = comp[3 * i + 2];
        imin[0] = fmin(imin[0], px);
        imin[1] = fmin(imin[1], py);
        imin[2] = fmin(imin[2], pz);
        imax[0] = fmax(imax[0], px);
        imax[1] = fmax(imax[1], py);
        imax[2] = fmax(imax[2], pz);
        if (pz <= zt) {
            cnt += 1.0;
            sx = dadd(sx, px);
            sy = dadd(sy, py);
            sz = dadd(sz, pz);
        }
    }
    double dmin[3], dmax[3];
    for (int c = 0; c < 3; ++c) {
        dmin[c] = block_min(s, imin[c]);
        dmax[c] = block_max(s, imax[c]);
    }
    const double ng = block_sum(s, cnt, 0);
    const int64_t nground = (int64_t)ng;
    double plane[4] = {0.0, 0.0, 1.0, -dmin[2]};
    double pkind = 1.0;
    if (nground > 10) {
        const double mx = block_sum(s, sx, 1) / ng, my = block_sum(s, sy, 2) / ng,
                     mz = block_sum(s, sz, 3) / ng;
        // TSQR of the centred, power-of-two-scaled rows (see plane_solve): |w| < 1 per entry
        int exy = 0, ezz = 0;
        const double extxy = fmax(dmax[0] - dmin[0], dmax[1] - dmin[1]), extz = dmax[2] - dmin[2];
        if (extxy > 0.0 && extxy < INFINITY) (void)frexp(extxy, &exy);
        if (extz > 0.0 && extz < INFINITY) (void)frexp(extz, &ezz);
        double r[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int64_t i = tid; i < nin; i += kT) {
            const double pz = comp[3 * i + 2];
            if (pz <= zt) {
                double w[4] = {ldexp(dsub(comp[3 * i], mx), -exy), ldexp(dsub(comp[3 * i + 1], my), -exy), 1.0,
                               ldexp(dsub(pz, mz), -ezz)};
                plane_row<0>(r, w);
            }
        }
        for (int m = 1; m < 64; m <<= 1) {  // fixed butterfly: lane 0 ends with the wave's R
            double p[10];
#pragma unroll
            for (int k = 0; k < 10; ++k) p[k] = __shfl_xor(r[k], m, 64);
            plane_merge(r, p);
        }
        __syncthreads();  // st is free between the chains; its first 160 doubles hold the waves' R
        if ((tid & 63) == 0)
#pragma unroll
            for (int k = 0; k < 10; ++k) st.v[0][(tid >> 6) * 10 + k] = r[k];
        __syncthreads();
        if (tid < 64) {
#pragma unroll
            for (int k = 0; k < 10; ++k) r[k] = tid < kW ? st.v[0][tid * 10 + k] : 0.0;
            for (int m = 1; m < kW; m <<= 1) {
                double p[10];
#pragma unroll
                for (int k = 0; k < 10; ++k) p[k] = __shfl_xor(r[k], m, 64);
                plane_merge(r, p);
            }
            if (tid == 0) {
                double x[3];
                const int rank = plane_solve(r, (double)exy, (double)ezz, mx, my, mz, ng, x);
                plane[0] = x[0];
                plane[1] = x[1];
                plane[2] = -1.0;
                plane[3] = x[2];
                pkind = rank == 3 ? 0.0 : 2.0;
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        S[S_ZT] = zt;
        S[S_NGROUND] = ng;
        for (int c = 0; c < 3; ++c) {
            S[S_DIMS + 2 * c] = dmin[c];
            S[S_DIMS + 2 * c + 1] = dmax[c];
        }
        for (int c = 0; c < 4; ++c) S[S_PLANE + c] = plane[c];
        S[S_PLANE_KIND] = pkind;
    }

    PRE_STAMP(5);
    // ---- F: non-ground compaction (:186)
    int64_t nng = 0;
    for (int64_t b0 = 0; b0 < nin; b0 += kT) {
        const int64_t i = b0 + tid;
        const bool f = i < nin && !(comp[3 * i + 2] <= zt);
        int tot;
        const int pos = block_flag_scan(s, f, &tot);
        if (f) {
            for (int c = 0; c < 3; ++c) sc[3 * (nng + pos) + c] = comp[3 * i + c];
            ng_pos[nng + pos] = (int32_t)i;
        }
        nng += tot;
    }
    if (tid == 0) S[S_NNG] = (double)nng;
    if (nng <= 10) return;  // reference: all non-ground labelled 0, no DBSCAN (:199-200)
    __threadfence_block();
    __syncthreads();
    if (fixed_eps > 0.0) {
        // app_simplified.py:104-108 / app_with_db.py:108-112 variant: DBSCAN(eps) on the
        // UNSCALED non-ground points — no StandardScaler, no eps heuristic; bbox of sc only
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int64_t i = tid; i < nng; i += kT)
            for (int c = 0; c < 3; ++c) {
                lo[c] = fmin(lo[c], sc[3 * i + c]);
                hi[c] = fmax(hi[c], sc[3 * i + c]);
            }
        for (int c = 0; c < 3; ++c) {
            const double a = block_min(s, lo[c]), b = block_max(s, hi[c]);
            if (tid == 0) {
                S[S_SLO + c] = a;
                S[S_SHI + c] = b;
                S[S_SMEAN + c] = 0.0;
                S[S_SSCALE + c] = 1.0;
            }
        }
        if (tid == 0) S[S_EPS] = fixed_eps;
        return;
    }

    PRE_STAMP(6);
    // ---- G: StandardScaler fit (sklearn _incremental_mean_and_var, zero prior) (:190-191)
    {
        const double nn = (double)nng;
        double sum = 0.0, unused = 0.0;
        block_seq_chain(sc, nng, st, [](int, double v, double &a, double &) { a = dadd(a, v); }, sum, unused);
        if (tid < 3) s.bc[6 + tid] = ddiv(sum, nn);
        __syncthreads();
        const double Tc = tid < 3 ? s.bc[6 + tid] : 0.0;
        // the second pass: sum of deviations (sequential) and, beside it, the sum of their squares (emulated)
        const double Tw = s.bc[6 + ((tid >> 6) + 2) % 3];  // waves 1..3: the mean of column wave - 1
        double corr = 0.0, unused2 = 0.0;
        block_seq_sum_chain(sc, nng, st, s, [Tc](int, double v, double &cr, double &) { cr = dadd(cr, dsub(v, Tc)); },
                            corr, unused2, [Tw](int, int, double v) {
                                const double d = dsub(v, Tw);
                                return dmul(d, d);
                            });
        if (tid < 3) {
        const double T = Tc;
        double un = s.chain[tid];
        un = dsub(un, ddiv(dmul(corr, corr), nn));
        const double var = ddiv(un, nn);
        const double e = 2.220446049250313e-16;
        const double ub = dadd(dmul(dmul(nn, e), var), dmul(dmul(dmul(nn, T), e), dmul(dmul(nn, T), e)));
        const double scale = var <= ub ? 1.0 : __dsqrt_rn(var);
        s.bc[6 + tid] = T;
        s.bc[9 + tid] = scale;
        }
    }
    __syncthreads();
    double smean[3], sscale[3];
    for (int c = 0; c < 3; ++c) {
        smean[c] = s.bc[6 + c];
        sscale[c] = s.bc[9 + c];
    }
    if (tid < 3) {
        S[S_SMEAN + tid] = smean[tid];
        S[S_SSCALE + tid] = sscale[tid];
    }
    PRE_STAMP(7);
    // ---- H: transform (X -= mean_; X /= scale_) and bbox of the scaled cloud
    double slo[3] = {INFINITY, INFINITY, INFINITY}, shi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = tid; i < nng; i += kT)
        for (int c = 0; c < 3; ++c) {
            const double y = ddiv(dsub(sc[3 * i + c], smean[c]), sscale[c]);
            sc[3 * i + c] = y;
            slo[c] = fmin(slo[c], y);
            shi[c] = fmax(shi[c], y);
        }
    double blo[3], bhi[3];
    for (int c = 0; c < 3; ++c) {
        blo[c] = block_min(s, slo[c]);
        bhi[c] = block_max(s, shi[c]);
    }
    __threadfence_block();
    __syncthreads();
    PRE_STAMP(8);
    // ---- I: eps = max(0.2, min(0.5, mean(std(scaled, axis=0)) * 0.5)) (:194-195)
    {
        const double nn = (double)nng;
        double sum = 0.0, unused = 0.0;
        block_seq_chain(sc, nng, st, [](int, double v, double &a, double &) { a = dadd(a, v); }, sum, unused);
        if (tid < 3) s.bc[12 + tid] = ddiv(sum, nn);
        __syncthreads();
        const double mw = s.bc[12 + (tid >> 6) % 3];
        block_sum_chain<1>(sc, nng, st, s, [mw](int, int, double v) {
            const double d = dsub(v, mw);
            return dmul(d, d);
        });
        if (tid < 3) s.bc[12 + tid] = __dsqrt_rn(ddiv(s.chain[tid], nn));
    }
    __syncthreads();
    if (tid == 0) {
        const double avg = dmul(ddiv(dadd(dadd(dadd(0.0, s.bc[12]), s.bc[13]), s.bc[14]), 3.0), 0.5);
        const double mn = avg < 0.5 ? avg : 0.5;
        const double eps = 0.2 >= mn ? 0.2 : mn;
        S[S_EPS] = eps;
        for (int c = 0; c < 3; ++c) {
            S[S_SLO + c] = blo[c];
            S[S_SHI + c] = bhi[c];
        }
    }
    PRE_STAMP(9);
}

// ------------------------------------------------------------------ DBSCAN
// params (double) P: [0] n, [1] eps, [2..4] lo, [5..7] hi, [8] cell, [9..11] dims,
// [12] ncell, [13] clusters, [14] active (n > 10 for the preprocess path), [15] stencil radius
// R in cells (1 or 2), [16] same-cell shortcut (1: cells of side eps/sqrt(3), see dbscan_setup)
enum : int { P_N = 0, P_EPS = 1, P_LO = 2, P_HI = 5, P_CELL = 8, P_DIM = 9, P_NCELL = 12,
             P_NCLUST = 13, P_ACTIVE = 14, P_R = 15, P_INTRA = 16, P_COUNT = 20 };

__global__ void dbscan_params_from_preprocess(const double *S_in, double *P_in, int64_t max_cells, FrameMap fm)
{
    if (threadIdx.x) return;
    const double *S = fm.scal(S_in);
    double *P = fm.ws(P_in);
    const double nng = S[S_NNG];
    P[P_N] = nng;
    P[P_EPS] = S[S_EPS];
    P[P_ACTIVE] = (S[S_STATUS] == 0.0 && nng > 10.0) ? 1.0 : 0.0;
    for (int c = 0; c < 3; ++c) {
        P[P_LO + c] = S[S_SLO + c];
        P[P_HI + c] = S[S_SHI + c];
    }
}

__global__ __launch_bounds__(kT) void dbscan_bbox_kernel(const double *x_in, double *P_in, FrameMap fm)
{
    const double *x = fm.ws(x_in);
    double *P = fm.ws(P_in);
    __shared__ BlockScratch s;
    const int64_t n = (int64_t)P[P_N];
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = threadIdx.x; i < n; i += kT)
        for (int c = 0; c < 3; ++c) {
            lo[c] = fmin(lo[c], x[3 * i + c]);
            hi[c] = fmax(hi[c], x[3 * i + c]);
        }
    for (int c = 0; c < 3; ++c) {
        const double a = block_min(s, lo[c]), b = block_max(s, hi[c]);
        if (threadIdx.x == 0) {
            P[P_LO + c] = a;
            P[P_HI + c] = b;
        }
    }
}

// Cell side.  Preferred: s = eps / sqrt(3) * (1 - 2^-20) ("fine" cells).  Any two points of one
// fine cell are eps-neighbours under the fp64 test: the cell coordinate floor((v - lo) / s) of a
// point inside the bbox carries < 2^-29 relative rounding at < 2^22 cells per axis, so the per-axis
// gaps inside a cell stay below s (1 + 2^-29), and the computed ((dx*dx + dy*dy) + dz*dz) below
// 3 s^2 (1 + 2^-26) < eps*eps (1 - 2^-20); a neighbour lies at most ceil(eps / s) = 2 cells away
// per axis (R = 2).  When the fine grid exceeds the cell cap: cells strictly larger than eps
// (R = 1, no same-cell shortcut), grown by 1.5 until they fit.
__global__ void dbscan_setup_kernel(double *P_in, int64_t max_cells, FrameMap fm)
{
    if (threadIdx.x) return;
    double *P = fm.ws(P_in);
    const double n = P[P_N], eps = P[P_EPS];
    const double cap = fmin(8.0 * n + 64.0, (double)max_cells);
    double dims[3] = {1.0, 1.0, 1.0}, tot = 1.0, cell = 1.0, R = 1.0, intra = 0.0;
    auto fits = [&](double c) {
        tot = 1.0;
        for (int k = 0; k < 3; ++k) {
            dims[k] = floor((P[P_HI + k] - P[P_LO + k]) / c) + 1.0;
            tot *= dims[k];
        }
        return tot <= cap;  // a non-finite box never fits
    };
    const double fine = eps / sqrt(3.0) * (1.0 - 1.0 / 1048576.0);
    if (P[P_ACTIVE] == 0.0 || !(eps > 0.0) || !(eps < INFINITY)) {
        P[P_ACTIVE] = 0.0;
    } else if (fits(fine)) {
        cell = fine;
        R = 2.0;
        intra = 1.0;
    } else {
        // cells strictly larger than eps: a 27-cell stencil sees every pair the fp64 test accepts
        cell = eps * (1.0 + 1.0 / 1048576.0);
        bool fit = false;
        for (int it = 0; it < 256 && !(fit = fits(cell)); ++it) cell *= 1.5;  // bounded: 1.5^256
        if (!fit) {  // non-finite box: one cell (still exact, only slower)
            dims[0] = dims[1] = dims[2] = 1.0;
            tot = 1.0;
            cell = INFINITY;
        }
    }
    P[P_CELL] = cell;
    for (int c = 0; c < 3; ++c) P[P_DIM + c] = dims[c];
    P[P_NCELL] = tot;
    P[P_R] = R;
    P[P_INTRA] = intra;
}

__device__ __forceinline__ int64_t cell_coord(double v, double lo, double cell, int64_t dim)
{
    int64_t c = (int64_t)floor((v - lo) / cell);
    return c < 0 ? 0 : (c >= dim ? dim - 1 : c);
}

struct Grid {
    double lo[3], cell, eps2;
    int64_t dim[3], n;
    int R;       // stencil radius in cells per axis
    bool intra;  // fine cells: any two points of one cell are neighbours
    __device__ void load(const double *P)
    {
        for (int c = 0; c < 3; ++c) {
            lo[c] = P[P_LO + c];
            dim[c] = (int64_t)P[P_DIM + c];
        }
        cell = P[P_CELL];
        eps2 = dmul(P[P_EPS], P[P_EPS]);
        n = (int64_t)P[P_N];
        R = (int)P[P_R];
        intra = P[P_INTRA] != 0.0;
    }
    __device__ int64_t cid(const double *p) const
    {
        return (cell_coord(p[0], lo[0], cell, dim[0]) * dim[1] + cell_coord(p[1], lo[1], cell, dim[1])) * dim[2] +
               cell_coord(p[2], lo[2], cell, dim[2]);
    }
};

__global__ void fill_u32_kernel(uint32_t *a_in, const double *P_in, int idx, int64_t extra, uint32_t v, FrameMap fm)
{
    uint32_t *a = fm.ws(a_in);
    const double *P = fm.ws(P_in);
    const int64_t n = (int64_t)P[idx] + extra;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        a[i] = v;
}

__global__ void dbscan_cells_kernel(const double *x_in, const double *P_in, uint32_t *cid_in, uint32_t *cellcnt_in,
                                    int32_t *parent_in, FrameMap fm)
{
    const double *x = fm.ws(x_in), *P = fm.ws(P_in);
    uint32_t *cid = fm.ws(cid_in), *cellcnt = fm.ws(cellcnt_in);
    int32_t *parent = fm.ws(parent_in);
    if (P[P_ACTIVE] == 0.0) return;
    Grid g;
    g.load(P);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < g.n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t c = (uint32_t)g.cid(x + 3 * i);
        cid[i] = c;
        parent[i] = (int32_t)i;
        atomicAdd(&cellcnt[c], 1u);
    }
}

// --- exclusive scan of u32 over count = P[idx] (+extra) entries; out[count] = total
constexpr int kScanPer = 4 * kT;
__global__ __launch_bounds__(kT) void scan_partial_kernel(const uint32_t *in_in, const double *P_in, int idx,
                                                          int64_t extra, uint32_t *partial_in, FrameMap fm)
{
    const uint32_t *in = fm.ws(in_in);
    const double *P = fm.ws(P_in);
    uint32_t *partial = fm.ws(partial_in);
    const int64_t n = (int64_t)P[idx] + extra;
    const int64_t b0 = (int64_t)blockIdx.x * kScanPer;
    uint32_t v = 0;
    for (int u = 0; u < 4; ++u) {
        const int64_t i = b0 + threadIdx.x * 4 + u;
        v += i < n ? in[i] : 0;
    }
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    __shared__ uint32_t ws[kW];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kW; ++w) t += ws[w];
        partial[blockIdx.x] = t;
    }
}
__global__ __launch_bounds__(kT) void scan_top_kernel(uint32_t *partial_in, int64_t nblk, FrameMap fm)
{
    uint32_t *partial = fm.ws(partial_in);
    // nblk <= 4 * kT
    __shared__ uint32_t ws[kW];
    uint32_t v[4], s = 0;
    for (int u = 0; u < 4; ++u) {
        const int64_t i = threadIdx.x * 4 + u;
        v[u] = i < nblk ? partial[i] : 0;
        s += v[u];
    }
    uint32_t incl = s;
    const int lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) ws[threadIdx.x >> 6] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) base += ws[w];
    uint32_t e = base + incl - s;
    for (int u = 0; u < 4; ++u) {
        const int64_t i = threadIdx.x * 4 + u;
        if (i < nblk) partial[i] = e;
        e += v[u];
    }
}
__global__ __launch_bounds__(kT) void scan_final_kernel(const uint32_t *in_in, uint32_t *out_in, const double *P_in,
                                                        int idx, int64_t extra, const uint32_t *partial_in, FrameMap fm)
{
    const uint32_t *in = fm.ws(in_in), *partial = fm.ws(partial_in);
    uint32_t *out = fm.ws(out_in);
    const double *P = fm.ws(P_in);
    const int64_t n = (int64_t)P[idx] + extra;
    const int64_t b0 = (int64_t)blockIdx.x * kScanPer;
    if (b0 > n) return;
    __shared__ uint32_t ws[kW];
    uint32_t v[4], s = 0;
    for (int u = 0; u < 4; ++u) {
        const int64_t i = b0 + threadIdx.x * 4 + u;
        v[u] = i < n ? in[i] : 0;
        s += v[u];
    }
    uint32_t incl = s;
    const int lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) ws[threadIdx.x >> 6] = incl;
    __syncthreads();
    uint32_t base = partial[blockIdx.x];
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) base += ws[w];
    uint32_t e = base + incl - s;
    for (int u = 0; u < 4; ++u) {
        const int64_t i = b0 + threadIdx.x * 4 + u;
        if (i <= n) out[i] = e;  // out[n] = total
        e += v[u];
    }
}

__global__ void dbscan_scatter_kernel(const double *x_in, const double *P_in, const uint32_t *cid_in,
                                      uint32_t *fill_in, uint32_t *order_in, double *sxyz_in, FrameMap fm)
{
    const double *x = fm.ws(x_in), *P = fm.ws(P_in);
    const uint32_t *cid = fm.ws(cid_in);
    uint32_t *fill = fm.ws(fill_in), *order = fm.ws(order_in);
    double *sxyz = fm.ws(sxyz_in);
    if (P[P_ACTIVE] == 0.0) return;
    const int64_t n = (int64_t)P[P_N];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t pos = atomicAdd(&fill[cid[i]], 1u);
        order[pos] = (uint32_t)i;
        sxyz[3 * pos] = x[3 * i];
        sxyz[3 * pos + 1] = x[3 * i + 1];
        sxyz[3 * pos + 2] = x[3 * i + 2];
    }
}

__global__ void copy_u32_kernel(uint32_t *dst_in, const uint32_t *src_in, const double *P_in, int idx, int64_t extra,
                                FrameMap fm)
{
    uint32_t *dst = fm.ws(dst_in);
    const uint32_t *src = fm.ws(src_in);
    const int64_t n = (int64_t)fm.ws(P_in)[idx] + extra;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// visit every sorted slot u whose point is within eps of point (px,py,pz) in cell c: the
// (2R+1)^2 columns around c, each a contiguous z-run of 2R+1 cells in the sorted order
template <class F>
__device__ __forceinline__ void for_neighbours(const Grid &g, const uint32_t *start, const double *sxyz,
                                               double px, double py, double pz, uint32_t c, F &&f)
{
    const int64_t cz = c % g.dim[2], cy = (c / g.dim[2]) % g.dim[1], cx = c / (g.dim[2] * g.dim[1]);
    const int64_t z0 = cz - g.R > 0 ? cz - g.R : 0, z1 = cz + g.R < g.dim[2] ? cz + g.R : g.dim[2] - 1;
    for (int64_t X = cx - g.R; X <= cx + g.R; ++X) {
        if (X < 0 || X >= g.dim[0]) continue;
        for (int64_t Y = cy - g.R; Y <= cy + g.R; ++Y) {
            if (Y < 0 || Y >= g.dim[1]) continue;
            const int64_t col = (X * g.dim[1] + Y) * g.dim[2];
            const uint32_t u0 = start[col + z0], u1 = start[col + z1 + 1];
            for (uint32_t u = u0; u < u1; ++u) {
                const double d = lidar::dist2d(px, py, pz, sxyz[3 * u], sxyz[3 * u + 1], sxyz[3 * u + 2]);
                if (d <= g.eps2) f(u);
            }
        }
    }
}

// eps-neighbour count of a point, stopping once it reaches `limit`: DBSCAN only asks whether
// cnt >= min_samples, and a standardized dense frame (eps 0.5 on unit-variance data) has hundreds
// of neighbours per point among thousands of candidates
__device__ __forceinline__ int32_t count_neighbours(const Grid &g, const uint32_t *start, const double *sxyz,
                                                    double px, double py, double pz, uint32_t c, int32_t limit)
{
    const int64_t cz = c % g.dim[2], cy = (c / g.dim[2]) % g.dim[1], cx = c / (g.dim[2] * g.dim[1]);
    const int64_t z0 = cz - g.R > 0 ? cz - g.R : 0, z1 = cz + g.R < g.dim[2] ? cz + g.R : g.dim[2] - 1;
    const int W = 2 * g.R + 1, centre = g.R * W + g.R;
    int32_t k = 0;
    // the point's own (X, Y) column first: the likeliest place to find `limit` hits
    for (int r = 0; r < W * W; ++r) {
        const int q = r == 0 ? centre : (r <= centre ? r - 1 : r);  // row-major columns, centre moved first
        const int64_t X = cx + q / W - g.R, Y = cy + q % W - g.R;
        if (X < 0 || X >= g.dim[0] || Y < 0 || Y >= g.dim[1]) continue;
        const int64_t col = (X * g.dim[1] + Y) * g.dim[2];
        const uint32_t u0 = start[col + z0], u1 = start[col + z1 + 1];
        for (uint32_t u = u0; u < u1; ++u) {
            const double d = lidar::dist2d(px, py, pz, sxyz[3 * u], sxyz[3 * u + 1], sxyz[3 * u + 2]);
            if (d <= g.eps2 && ++k >= limit) return k;
        }
    }
    return k;
}

constexpr uint32_t kNoCore = 0xffffffffu;

// eps-neighbour counts (stopping at `limit`); with `core_in` set also the core flag of every sorted
// slot and rep[c] = the smallest core index of cell c (rep initialised to kNoCore).  Fine cells:
// every point of a cell is a neighbour, so a cell of >= limit points settles its points' counts
// without a distance test.
__global__ void dbscan_count_kernel(const double *P_in, const uint32_t *cid_in, const uint32_t *start_in,
                                    const uint32_t *order_in, const double *sxyz_in, int32_t *cnt_in,
                                    int32_t limit, int32_t min_samples, uint8_t *core_in, uint32_t *rep_in,
                                    FrameMap fm)
{
    const double *P = fm.ws(P_in), *sxyz = fm.ws(sxyz_in);
    const uint32_t *cid = fm.ws(cid_in), *start = fm.ws(start_in), *order = fm.ws(order_in);
    int32_t *cnt = fm.ws(cnt_in);
    uint8_t *core = core_in ? fm.ws(core_in) : nullptr;
    uint32_t *rep = rep_in ? fm.ws(rep_in) : nullptr;
    if (P[P_ACTIVE] == 0.0) return;
    Grid g;
    g.load(P);
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < g.n; t += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t i = order[t], c = cid[i];
        const int64_t in_cell = (int64_t)start[c + 1] - start[c];
        const int32_t k = g.intra && in_cell >= limit
                              ? (int32_t)in_cell
                              : count_neighbours(g, start, sxyz, sxyz[3 * t], sxyz[3 * t + 1], sxyz[3 * t + 2], c, limit);
        cnt[i] = k;
        if (core) {
            const bool is_core = k >= min_samples;
            core[t] = is_core ? 1 : 0;
            if (is_core) atomicMin(rep + c, i);
        }
    }
}

__device__ __forceinline__ int32_t ld(const int32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st(int32_t *p, int32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// find with path halving.  Invariant: parent[x] <= x (roots hook under smaller roots), so
// every pointer moves toward the component minimum and the halving stores (x's parent
// becomes its grandparent, an ancestor in the same component) are benign under races.
__device__ int32_t uf_find(int32_t *parent, int32_t x)
{
    int32_t p = ld(parent + x);
    while (p != x) {
        const int32_t gp = ld(parent + p);
        if (gp != p) st(parent + x, gp);
        x = p;
        p = gp;
    }
    return x;
}
// read-only find: the roots pass publishes parent[i] = root for the labels pass, and a
// halving store racing behind that publish would leave a non-root there
__device__ int32_t uf_find_ro(const int32_t *parent, int32_t x)
{
    int32_t p = ld(parent + x);
    while (p != x) {
        x = p;
        p = ld(parent + x);
    }
    return x;
}
// join the components of roots-or-members a and b; returns the (current) smaller root
__device__ int32_t uf_unite(int32_t *parent, int32_t a, int32_t b)
{
    for (;;) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return a;
        if (a < b) {
            const int32_t t = a;
            a = b;
            b = t;
        }
        // hook the larger root under the smaller: the final root is the component minimum
        const int32_t old = atomicCAS(parent + a, a, b);
        if (old == a) return b;
        a = old;
    }
}

__global__ void dbscan_union_kernel(const double *P_in, const uint32_t *cid_in, const uint32_t *start_in,
                                    const uint32_t *order_in, const double *sxyz_in, const int32_t *cnt_in,
                                    int32_t min_samples, int32_t *parent_in, FrameMap fm)
{
    const double *P = fm.ws(P_in), *sxyz = fm.ws(sxyz_in);
    const uint32_t *cid = fm.ws(cid_in), *start = fm.ws(start_in), *order = fm.ws(order_in);
    const int32_t *cnt = fm.ws(cnt_in);
    int32_t *parent = fm.ws(parent_in);
    if (P[P_ACTIVE] == 0.0 || P[P_INTRA] != 0.0) return;  // fine cells: dbscan_intra + dbscan_cross
    Grid g;
    g.load(P);
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < g.n; t += (int64_t)gridDim.x * blockDim.x) {
        const int32_t i = (int32_t)order[t];
        if (cnt[i] < min_samples) continue;
        // i's root is cached across its neighbours: a neighbour already in the same
        // component costs one (halving) find, not two
        int32_t ri = uf_find(parent, i);
        for_neighbours(g, start, sxyz, sxyz[3 * t], sxyz[3 * t + 1], sxyz[3 * t + 2], cid[i], [&](uint32_t u) {
            const int32_t j = (int32_t)order[u];
            if (j < i && cnt[j] >= min_samples) {
                if (ld(parent + j) == ri) return;  // already hooked straight under i's root
                const int32_t rj = uf_find(parent, j);
                if (rj != ri) ri = uf_unite(parent, ri, rj);
            }
        });
    }
}

// Fine cells, step 1: every core point of a cell hooks straight under the cell's smallest core
// index (all of a cell's points are mutually eps-neighbours; parent[i] <= i holds, and no other
// kernel writes parent meanwhile).
__global__ void dbscan_intra_kernel(const double *P_in, const uint32_t *cid_in, const uint32_t *order_in,
                                    const uint8_t *core_in, const uint32_t *rep_in, int32_t *parent_in, FrameMap fm)
{
    const double *P = fm.ws(P_in);
    if (P[P_ACTIVE] == 0.0 || P[P_INTRA] == 0.0) return;
    const uint32_t *cid = fm.ws(cid_in), *order = fm.ws(order_in), *rep = fm.ws(rep_in);
    const uint8_t *core = fm.ws(core_in);
    int32_t *parent = fm.ws(parent_in);
    const int64_t n = (int64_t)P[P_N];
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        if (!core[t]) continue;
        const uint32_t i = order[t], r = rep[cid[i]];
        if (r != i) parent[i] = (int32_t)r;
    }
}

// Fine cells, step 2: one thread per (cell A, offset o) over the 62 offsets of [-2, 2]^3 that come
// lexicographically after (0, 0, 0) — every pair of cells within the stencil once.  If A and B =
// A + o both hold core points that are not yet one component, any core of A within eps of any
// core of B links them.  Each cell's cores are one component (step 1), so the components after
// this pass are exactly those of the core-core eps graph.
//
// The 62 offsets run in two launches: first the 13 touching cells (Chebyshev distance 1), which in
// a dense frame link almost every pair at the first core tested and merge nearly everything into
// few components; then the 49 offsets two cells out, most of whose pairs are by then already one
// component (two finds and out) instead of a full core x core scan that finds no link.  Union-find
// yields the connected components whatever the order of the unions, so the split is exact.
// A core u of A whose gap to B's cell box exceeds eps is skipped: the box is taken one part in 2^10
// of a cell larger on every side, far beyond the rounding of floor((v - lo) / s), so it contains
// every point binned into B, and the gap never overstates a true distance.
constexpr int kPairOffsets = 62, kNearOffsets = 13;
struct PairOffsets {
    int o[kPairOffsets];
    constexpr PairOffsets() : o{}
    {
        int k = 0;
        for (int pass = 0; pass < 2; ++pass)
            for (int v = 63; v < 125; ++v) {  // 5x5x5 row-major; (0,0,0) is 62, after it come the 62
                const int dx = v / 25 - 2, dy = (v / 5) % 5 - 2, dz = v % 5 - 2;
                const bool near = dx >= -1 && dx <= 1 && dy >= -1 && dy <= 1 && dz >= -1 && dz <= 1;
                if (near == (pass == 0)) o[k++] = v;
            }
    }
};
__constant__ PairOffsets kOffsets = PairOffsets();

__device__ __forceinline__ double box_gap(double v, double lo, double hi)
{
    const double a = lo - v, b = v - hi;
    return a > 0.0 ? a : (b > 0.0 ? b : 0.0);
}

__global__ void dbscan_cross_kernel(const double *P_in, const uint32_t *start_in, const double *sxyz_in,
                                    const uint8_t *core_in, const uint32_t *rep_in, int32_t *parent_in, int o0,
                                    int no, FrameMap fm)
{
    const double *P = fm.ws(P_in);
    if (P[P_ACTIVE] == 0.0 || P[P_INTRA] == 0.0) return;
    const double *sxyz = fm.ws(sxyz_in);
    const uint32_t *start = fm.ws(start_in), *rep = fm.ws(rep_in);
    const uint8_t *core = fm.ws(core_in);
    int32_t *parent = fm.ws(parent_in);
    Grid g;
    g.load(P);
    const double slack = g.cell * (1.0 / 1024.0);
    const int64_t work = (int64_t)P[P_NCELL] * no;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < work; w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t A = w / no;
        const uint32_t ra0 = rep[A];
        if (ra0 == kNoCore) continue;
        const int o = kOffsets.o[o0 + (int)(w - A * no)];
        const int64_t ax = A / (g.dim[1] * g.dim[2]), ay = (A / g.dim[2]) % g.dim[1], az = A % g.dim[2];
        const int64_t bx = ax + o / 25 - 2, by = ay + (o / 5) % 5 - 2, bz = az + o % 5 - 2;
        if (bx < 0 || bx >= g.dim[0] || by < 0 || by >= g.dim[1] || bz < 0 || bz >= g.dim[2]) continue;
        const int64_t B = (bx * g.dim[1] + by) * g.dim[2] + bz;
        const uint32_t rb0 = rep[B];
        if (rb0 == kNoCore) continue;
        const int32_t ra = uf_find(parent, (int32_t)ra0), rb = uf_find(parent, (int32_t)rb0);
        if (ra == rb) continue;
        double blo[3], bhi[3];
        const int64_t bc[3] = {bx, by, bz};
        for (int k = 0; k < 3; ++k) {
            blo[k] = g.lo[k] + (double)bc[k] * g.cell - slack;
            bhi[k] = g.lo[k] + (double)(bc[k] + 1) * g.cell + slack;
        }
        bool linked = false;
        const uint32_t b0 = start[B], b1 = start[B + 1];
        for (uint32_t u = start[A], u1 = start[A + 1]; u < u1 && !linked; ++u) {
            if (!core[u]) continue;
            const double px = sxyz[3 * u], py = sxyz[3 * u + 1], pz = sxyz[3 * u + 2];
            const double gx = box_gap(px, blo[0], bhi[0]), gy = box_gap(py, blo[1], bhi[1]),
                         gz = box_gap(pz, blo[2], bhi[2]);
            if ((gx * gx + gy * gy) + gz * gz > g.eps2) continue;
            for (uint32_t v = b0; v < b1; ++v)
                if (core[v] && lidar::dist2d(px, py, pz, sxyz[3 * v], sxyz[3 * v + 1], sxyz[3 * v + 2]) <= g.eps2) {
                    linked = true;
                    break;
                }
        }
        if (linked) uf_unite(parent, ra, rb);
    }
}

__global__ void dbscan_roots_kernel(const double *P_in, const int32_t *cnt_in, int32_t min_samples,
                                    int32_t *parent_in, uint32_t *flag_in, FrameMap fm)
{
    const double *P = fm.ws(P_in);
    const int32_t *cnt = fm.ws(cnt_in);
    int32_t *parent = fm.ws(parent_in);
    uint32_t *flag = fm.ws(flag_in);
    const int64_t n = (int64_t)P[P_N];
    const bool active = P[P_ACTIVE] != 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t f = 0;
        if (active && cnt[i] >= min_samples) {
            const int32_t r = uf_find_ro(parent, (int32_t)i);
            parent[i] = r;
            f = r == (int32_t)i ? 1u : 0u;
        }
        flag[i] = f;
    }
}

__global__ void dbscan_labels_kernel(double *P_in, const uint32_t *cid_in, const uint32_t *start_in,
                                     const uint32_t *order_in, const double *sxyz_in, const int32_t *cnt_in,
                                     int32_t min_samples, const int32_t *parent_in, const uint32_t *rank_in,
                                     const uint8_t *core_in, int64_t *labels_in, FrameMap fm)
{
    double *P = fm.ws(P_in);
    const uint8_t *core = fm.ws(core_in);
    const double *sxyz = fm.ws(sxyz_in);
    const uint32_t *cid = fm.ws(cid_in), *start = fm.ws(start_in), *order = fm.ws(order_in), *rank = fm.ws(rank_in);
    const int32_t *cnt = fm.ws(cnt_in), *parent = fm.ws(parent_in);
    int64_t *labels = fm.ws(labels_in);
    if (P[P_ACTIVE] == 0.0) return;
    Grid g;
    g.load(P);
    if (blockIdx.x == 0 && threadIdx.x == 0) P[P_NCLUST] = (double)rank[g.n];
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < g.n; t += (int64_t)gridDim.x * blockDim.x) {
        const int32_t i = (int32_t)order[t];
        int64_t lab;
        if (cnt[i] >= min_samples) {
            lab = rank[parent[i]];
        } else {
            int64_t best = -1;
            for_neighbours(g, start, sxyz, sxyz[3 * t], sxyz[3 * t + 1], sxyz[3 * t + 2], cid[i], [&](uint32_t u) {
                if (core[u]) {
                    const int64_t l = rank[parent[order[u]]];
                    if (best < 0 || l < best) best = l;
                }
            });
            lab = best;
        }
        labels[i] = lab;
    }
}

// full labels over the inliers: ground -1, non-ground = DBSCAN label (or 0 when <= 10)
__global__ void scatter_labels_kernel(const double *S_in, const int64_t *ng_labels_in, const int32_t *ng_pos_in,
                                      int64_t *full_in, FrameMap fm)
{
    const double *S = fm.scal(S_in);
    int64_t *full = fm.rows(full_in, 1);
    if (S[S_STATUS] != 0.0) return;
    const int64_t nin = (int64_t)S[S_NIN];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nin; i += stride) full[i] = -1;
    __syncthreads();
}
__global__ void scatter_labels2_kernel(const double *S_in, const int64_t *ng_labels_in, const int32_t *ng_pos_in,
                                       int64_t *full_in, FrameMap fm)
{
    const double *S = fm.scal(S_in);
    const int64_t *ng_labels = fm.ws(ng_labels_in);
    const int32_t *ng_pos = fm.ws(ng_pos_in);
    int64_t *full = fm.rows(full_in, 1);
    if (S[S_STATUS] != 0.0) return;
    const int64_t nng = (int64_t)S[S_NNG];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nng; i += stride)
        full[ng_pos[i]] = nng > 10 ? ng_labels[i] : 0;
}

// ------------------------------------------------------------------ people
// One workgroup per cluster: waves 1..15 compact the cluster's members of a 960-point chunk
// (wave w owns points [64(w-1), 64w) of every chunk) into LDS contiguously in index order
// (double-buffered rows, triple-buffered per-wave counts), and lanes 0 / 1 of wave 0 run the
// x / y chains over the chunk's members in one run, as np.mean of the member rows does
// (sequential axis-0 sums starting from the first row).  Per chunk: the staging waves place
// chunk k+1 (its counts were published a phase earlier) and count chunk k+2 while wave 0 adds
// chunk k; one barrier per chunk.
__global__ __launch_bounds__(kT) void people_kernel(const double *xyz_in, const int64_t *labels_in, int64_t n_in,
                                                    const int64_t *kdev_in, double *out_in, const double *S_in,
                                                    FrameMap fm)
{
    // a batch frame's rows are its inliers: n = scalars[S_NIN] (0 for a failed frame)
    const int64_t n = S_in ? (fm.scal(S_in)[S_STATUS] == 0.0 ? (int64_t)fm.scal(S_in)[S_NIN] : 0) : n_in;
    const double *xyz = fm.rows(xyz_in, 3);
    const int64_t *labels = fm.rows(labels_in, 1);
    const int64_t *kdev = kdev_in + blockIdx.y;
    double *out = fm.rows(out_in, 2);
    constexpr int kChunk = kT - 64;
    __shared__ double mem[2][kChunk * 2];
    __shared__ int wcnt[3][kW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t K = *kdev;
    const int64_t nch = (n + kChunk - 1) / kChunk;
    for (int64_t c = blockIdx.x; c < K; c += gridDim.x) {
        // members of this wave's 64 points of chunk k (0 for wave 0 and past the end), published
        // as the wave's count of chunk k
        auto count = [&](int64_t k) -> uint64_t {
            if (wave == 0) return 0;
            const int64_t i = k * kChunk + (tid - 64);
            const uint64_t m = __ballot(k < nch && i < n && labels[i] == c);
            if (lane == 0) wcnt[k % 3][wave] = __popcll(m);
            return m;
        };
        auto place = [&](int64_t k, uint64_t m) {
            if (wave == 0 || k >= nch || !((m >> lane) & 1)) return;
            int base = 0;
            for (int w = 1; w < wave; ++w) base += wcnt[k % 3][w];
            const int64_t i = k * kChunk + (tid - 64);
            const int r = base + __popcll(m & ((1ull << lane) - 1));
            mem[k & 1][2 * r] = xyz[3 * i];
            mem[k & 1][2 * r + 1] = xyz[3 * i + 1];
        };
        double acc = 0.0;
        int64_t cnt = 0;
        uint64_t m_next = count(0);
        __syncthreads();
        place(0, m_next);
        m_next = count(1);
        __syncthreads();
        for (int64_t k = 0; k < nch; ++k) {
            if (wave != 0) {
                place(k + 1, m_next);
                m_next = count(k + 2);
            } else if (tid < 2) {
                int tot = 0;
                for (int w = 1; w < kW; ++w) tot += wcnt[k % 3][w];
                const double *b = mem[k & 1] + tid;
                int j = 0;
                if (cnt == 0 && tot > 0) {  // np.add.reduce starts from the first row
                    acc = b[0];
                    j = 1;
                }
                for (; j + 16 <= tot; j += 16) {  // reads first, then the dependent adds
                    double v[16];
#pragma unroll
                    for (int u = 0; u < 16; ++u) v[u] = b[2 * (j + u)];
#pragma unroll
                    for (int u = 0; u < 16; ++u) acc = dadd(acc, v[u]);
                }
                for (; j < tot; ++j) acc = dadd(acc, b[2 * j]);
                cnt += tot;
            }
            __syncthreads();
        }
        if (tid < 2) out[2 * c + tid] = ddiv(acc, (double)cnt);
        __syncthreads();  // the next cluster's first counts reuse wcnt[0..1]
    }
}

__global__ void max_label_kernel(const int64_t *labels_in, int64_t n_in, int64_t *kout_in, const double *S_in,
                                 FrameMap fm)
{
    const int64_t n = S_in ? (fm.scal(S_in)[S_STATUS] == 0.0 ? (int64_t)fm.scal(S_in)[S_NIN] : 0) : n_in;
    const int64_t *labels = fm.rows(labels_in, 1);
    int64_t *kout = kout_in + blockIdx.y;
    // K = number of distinct labels >= 0 = max + 1 (labels are dense ranks)
    int64_t m = -1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        m = labels[i] > m ? labels[i] : m;
    for (int o = 32; o >= 1; o >>= 1) {
        const int64_t t = __shfl_xor(m, o, 64);
        m = t > m ? t : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax((unsigned long long *)kout, (unsigned long long)(m + 1));
}

// ------------------------------------------------------------------ density grid
// numpy float64 add.reduce of a contiguous 1-D array: 8192-element buffer chunks,
// each summed by pairwise_sum (8-way unrolled leaves of <= 128), chunks added in order
__device__ double np_pairwise(const double *a, int64_t n)
{
    if (n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < n; ++i) r = dadd(r, a[i]);
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] = dadd(r[j], a[i + j]);
        double res = dadd(dadd(dadd(r[0], r[1]), dadd(r[2], r[3])), dadd(dadd(r[4], r[5]), dadd(r[6], r[7])));
        for (; i < n; ++i) res = dadd(res, a[i]);
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return dadd(np_pairwise(a, n2), np_pairwise(a + n2, n - n2));
}
__device__ double np_sum(const double *a, int64_t n)
{
    double out = 0.0;
    for (int64_t i = 0; i < n; i += 8192) out = dadd(out, np_pairwise(a + i, n - i < 8192 ? n - i : 8192));
    return out;
}

__device__ int64_t searchsorted_right(const double *e, int64_t len, double v)
{
    int64_t lo = 0, hi = len;  // first index with e[idx] > v
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (e[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ void density_body(const double *people, const int64_t *kdev,
                             double xa, double ya, double g, int64_t nx, int64_t ny,
                             double *xe, double *ye, uint32_t *count,
                             double *grid_x, double *grid_y, double *density,
                             double *flat_x, double *flat_y, double *pos_scratch,
                             double *stats, int64_t *hot)
{
    const int64_t K = *kdev;
    const int tid = threadIdx.x;
    // np.arange: e[0] = a, e[1] = a + g, e[i] = a + i * (e[1] - e[0])
    const double dx = dsub(dadd(xa, g), xa), dy = dsub(dadd(ya, g), ya);
    for (int64_t i = tid; i <= nx; i += kT) xe[i] = i == 0 ? xa : (i == 1 ? dadd(xa, g) : dadd(xa, dmul((double)i, dx)));
    for (int64_t i = tid; i <= ny; i += kT) ye[i] = i == 0 ? ya : (i == 1 ? dadd(ya, g) : dadd(ya, dmul((double)i, dy)));
    for (int64_t i = tid; i < nx * ny; i += kT) count[i] = 0;
    __threadfence_block();
    __syncthreads();
    for (int64_t k = tid; k < K; k += kT) {
        const double px = people[2 * k], py = people[2 * k + 1];
        int64_t bx = searchsorted_right(xe, nx + 1, px), by = searchsorted_right(ye, ny + 1, py);
        if (px == xe[nx]) --bx;
        if (py == ye[ny]) --by;
        if (bx >= 1 && bx <= nx && by >= 1 && by <= ny) atomicAdd(&count[(bx - 1) * ny + (by - 1)], 1u);
    }
    __threadfence_block();
    __syncthreads();
    const double g2 = dmul(g, g);
    for (int64_t i = tid; i < nx; i += kT) grid_x[i] = ddiv(dadd(xe[i], xe[i + 1]), 2.0);
    for (int64_t i = tid; i < ny; i += kT) grid_y[i] = ddiv(dadd(ye[i], ye[i + 1]), 2.0);
    for (int64_t i = tid; i < nx * ny; i += kT) {
        density[i] = ddiv((double)count[i], g2);
        flat_x[i] = ddiv(dadd(xe[i / ny], xe[i / ny + 1]), 2.0);
        flat_y[i] = ddiv(dadd(ye[i % ny], ye[i % ny + 1]), 2.0);
    }
    __threadfence_block();
    __syncthreads();
    if (tid == 0) {
        // max, occupied cells in flat order, numpy mean, threshold, stable top-5
        double mx = -INFINITY;
        int64_t np_ = 0;
        for (int64_t i = 0; i < nx * ny; ++i) {
            const double d = density[i];
            mx = d > mx ? d : mx;
            if (d > 0.0) pos_scratch[np_++] = d;
        }
        const double avg = np_ > 0 ? ddiv(np_sum(pos_scratch, np_), (double)np_) : 0.0;
        const double a15 = dmul(avg, 1.5);
        const double thr = 0.5 >= a15 ? 0.5 : a15;
        int64_t nh = 0;
        double last = INFINITY;
        int64_t last_i = -1;
        for (; nh < 5; ++nh) {
            // next hotspot: highest density below (last, last_i) in (desc density, asc index) order
            int64_t best = -1;
            double bd = -INFINITY;
            for (int64_t i = 0; i < nx * ny; ++i) {
                const double d = density[i];
                if (!(d >= thr)) continue;
                const bool after = d < last || (d == last && i > last_i);
                if (!after) continue;
                if (best < 0 || d > bd) {
                    best = i;
                    bd = d;
                }
            }
            if (best < 0) break;
            hot[nh] = best;
            last = bd;
            last_i = best;
        }
        stats[0] = mx;
        stats[1] = avg;
        stats[2] = thr;
        stats[3] = (double)nh;
        stats[4] = (double)np_;
        stats[5] = (double)K;
    }
}

__global__ __launch_bounds__(kT) void density_kernel(const double *people, const int64_t *kdev,
                                                     double xa, double ya, double g, int64_t nx, int64_t ny,
                                                     double *xe, double *ye, uint32_t *count,
                                                     double *grid_x, double *grid_y, double *density,
                                                     double *flat_x, double *flat_y, double *pos_scratch,
                                                     double *stats, int64_t *hot)
{
    density_body(people, kdev, xa, ya, g, nx, ny, xe, ye, count, grid_x, grid_y, density, flat_x, flat_y,
                 pos_scratch, stats, hot);
}

// one workgroup per frame; job row f (8 doubles): xa, ya, g, nx, ny, out offset, scratch
// offset (doubles), unused.  out at its offset: grid_x | grid_y | density | flat_x | flat_y |
// stats(8) | hot(5 int64); scratch: xe (nx+1) | ye (ny+1) | pos (nx*ny) | count (nx*ny u32).
// Frames with no people (k == 0) are skipped (the caller returns the reference's empty dict).
__global__ __launch_bounds__(kT) void density_batch_kernel(const double *people_in, const int64_t *offs,
                                                           const int64_t *kdev, const double *jobs, double *out,
                                                           double *scratch)
{
    const int f = blockIdx.y;
    const double *J = jobs + 8 * (int64_t)f;
    if (kdev[f] <= 0) return;
    const int64_t nx = (int64_t)J[3], ny = (int64_t)J[4], m = nx * ny;
    double *o = out + (int64_t)J[5];
    double *sc = scratch + (int64_t)J[6];
    double *xe = sc, *ye = xe + nx + 1, *pos = ye + ny + 1;
    uint32_t *count = reinterpret_cast<uint32_t *>(pos + m);
    double *gx = o, *gy = gx + nx, *dens = gy + ny, *fx = dens + m, *fy = fx + m, *st = fy + m;
    density_body(people_in + 2 * offs[f], kdev + f, J[0], J[1], J[2], nx, ny, xe, ye, count, gx, gy, dens, fx, fy,
                 pos, st, reinterpret_cast<int64_t *>(st + 8));
}

__global__ void nclust_kernel(const double *P_in, double *S_in, FrameMap fm)
{
    if (threadIdx.x == 0) fm.scal(S_in)[S_NCLUST] = fm.ws(P_in)[P_NCLUST];
}

// ------------------------------------------------------------------ workspace plan
struct DbscanWs {
    double *P;
    uint32_t *cid, *cellcnt, *cellstart, *fill, *order, *flag, *rank, *partial;
    double *sxyz;
    int32_t *cnt, *parent;
    uint8_t *core;  // per sorted slot; `fill` doubles as the cells' smallest core index after the scatter
    int64_t max_cells, nblk_cells, nblk_pts;
};

constexpr int kDbscanParts = 13;
int64_t max_cells_for(int64_t n) { return std::min<int64_t>(8 * n + 64, 1 << 22); }

void plan_dbscan(lidar::Carver &cv, int64_t n, uint64_t *off)
{
    const int64_t mc = max_cells_for(n);
    off[0] = cv.take<double>(P_COUNT);
    off[1] = cv.take<uint32_t>(n);           // cid
    off[2] = cv.take<uint32_t>(mc + 1);      // cellcnt
    off[3] = cv.take<uint32_t>(mc + 1);      // cellstart
    off[4] = cv.take<uint32_t>(mc + 1);      // fill
    off[5] = cv.take<uint32_t>(n + 1);       // order
    off[6] = cv.take<uint32_t>(n + 1);       // flag
    off[7] = cv.take<uint32_t>(n + 1);       // rank
    off[8] = cv.take<uint32_t>(4 * kT);      // partial
    off[9] = cv.take<double>(3 * n);         // sxyz
    off[10] = cv.take<int32_t>(n);           // cnt
    off[11] = cv.take<int32_t>(n);           // parent
    off[12] = cv.take<uint8_t>(n);           // core (sorted slots)
}

DbscanWs bind_dbscan(char *base, const uint64_t *off, int64_t n)
{
    DbscanWs w;
    w.P = reinterpret_cast<double *>(base + off[0]);
    w.cid = reinterpret_cast<uint32_t *>(base + off[1]);
    w.cellcnt = reinterpret_cast<uint32_t *>(base + off[2]);
    w.cellstart = reinterpret_cast<uint32_t *>(base + off[3]);
    w.fill = reinterpret_cast<uint32_t *>(base + off[4]);
    w.order = reinterpret_cast<uint32_t *>(base + off[5]);
    w.flag = reinterpret_cast<uint32_t *>(base + off[6]);
    w.rank = reinterpret_cast<uint32_t *>(base + off[7]);
    w.partial = reinterpret_cast<uint32_t *>(base + off[8]);
    w.sxyz = reinterpret_cast<double *>(base + off[9]);
    w.cnt = reinterpret_cast<int32_t *>(base + off[10]);
    w.parent = reinterpret_cast<int32_t *>(base + off[11]);
    w.core = reinterpret_cast<uint8_t *>(base + off[12]);
    w.max_cells = max_cells_for(n);
    w.nblk_cells = (w.max_cells + 1 + kScanPer - 1) / kScanPer;
    w.nblk_pts = (n + 1 + kScanPer - 1) / kScanPer;
    return w;
}

int run_scan(const uint32_t *in, uint32_t *out, const double *P, int idx, int64_t extra, uint32_t *partial,
             int64_t nblk, hipStream_t s, FrameMap fm, int frames)
{
    hipLaunchKernelGGL(scan_partial_kernel, dim3((unsigned)nblk, frames), dim3(kT), 0, s, in, P, idx, extra, partial, fm);
    hipLaunchKernelGGL(scan_top_kernel, dim3(1, frames), dim3(kT), 0, s, partial, nblk, fm);
    hipLaunchKernelGGL(scan_final_kernel, dim3((unsigned)nblk, frames), dim3(kT), 0, s, in, out, P, idx, extra, partial,
                       fm);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

// blocks per frame of a per-point kernel: enough to fill the chip across all frames
unsigned point_blocks(int64_t nmax, int frames)
{
    const int64_t cap = std::max<int64_t>(8, 4096 / std::max(1, frames));
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((nmax + 255) / 256, cap));
}

// the DBSCAN pipeline on x (P[P_N] points, eps P[P_EPS], bbox in P) -> labels, for every frame
// exact_counts: cnt[i] is the full eps-neighbour count (radius counts, the standalone API's
// counts output); otherwise counting stops at min_samples.  h: profiling spans (may be null).
int run_dbscan(lidar_handle *h, const double *x, int64_t nmax, int32_t min_samples, DbscanWs &w, int64_t *labels,
               hipStream_t s, FrameMap fm, int frames, bool count_only = false, bool exact_counts = false)
{
    const int32_t limit = (count_only || exact_counts) ? 0x7fffffff : min_samples;
    const unsigned gp = point_blocks(nmax, frames);
    const unsigned gc = point_blocks(w.max_cells, frames);
    const unsigned gx = point_blocks(w.max_cells * (kPairOffsets - kNearOffsets), frames);
    const unsigned gn = point_blocks(w.max_cells * kNearOffsets, frames);
    const dim3 F1(1, frames), FP(gp, frames), FC(gc, frames), FX(gx, frames), FN(gn, frames);
    {
        lidar::Span sp(h, "dbscan_grid", s);  // cell sizes, counting sort by cell
        hipLaunchKernelGGL(dbscan_setup_kernel, F1, dim3(64), 0, s, w.P, w.max_cells, fm);
        hipLaunchKernelGGL(fill_u32_kernel, FC, dim3(256), 0, s, w.cellcnt, w.P, P_NCELL, 1, 0u, fm);
        hipLaunchKernelGGL(dbscan_cells_kernel, FP, dim3(256), 0, s, x, w.P, w.cid, w.cellcnt, w.parent, fm);
        int rc = run_scan(w.cellcnt, w.cellstart, w.P, P_NCELL, 0, w.partial, w.nblk_cells, s, fm, frames);
        if (rc) return rc;
        hipLaunchKernelGGL(copy_u32_kernel, FC, dim3(256), 0, s, w.fill, w.cellstart, w.P, P_NCELL, 1, fm);
        hipLaunchKernelGGL(dbscan_scatter_kernel, FP, dim3(256), 0, s, x, w.P, w.cid, w.fill, w.order, w.sxyz, fm);
        if (!count_only)  // `fill` is free after the scatter: the cells' smallest core index
            hipLaunchKernelGGL(fill_u32_kernel, FC, dim3(256), 0, s, w.fill, w.P, P_NCELL, 1, kNoCore, fm);
    }
    {
        lidar::Span sp(h, "dbscan_count", s);
        hipLaunchKernelGGL(dbscan_count_kernel, FP, dim3(256), 0, s, w.P, w.cid, w.cellstart, w.order, w.sxyz, w.cnt,
                           limit, min_samples, count_only ? nullptr : w.core, count_only ? nullptr : w.fill, fm);
    }
    if (count_only) {
        LAUNCH_CHECK();
        return LIDAR_OK;
    }
    {
        lidar::Span sp(h, "dbscan_union", s);  // fine cells: intra + cross; coarse cells: per-point union
        hipLaunchKernelGGL(dbscan_intra_kernel, FP, dim3(256), 0, s, w.P, w.cid, w.order, w.core, w.fill, w.parent, fm);
        hipLaunchKernelGGL(dbscan_cross_kernel, FN, dim3(256), 0, s, w.P, w.cellstart, w.sxyz, w.core, w.fill,
                           w.parent, 0, kNearOffsets, fm);
        hipLaunchKernelGGL(dbscan_cross_kernel, FX, dim3(256), 0, s, w.P, w.cellstart, w.sxyz, w.core, w.fill,
                           w.parent, kNearOffsets, kPairOffsets - kNearOffsets, fm);
        hipLaunchKernelGGL(dbscan_union_kernel, FP, dim3(256), 0, s, w.P, w.cid, w.cellstart, w.order, w.sxyz,
                           w.cnt, min_samples, w.parent, fm);
    }
    {
        lidar::Span sp(h, "dbscan_labels", s);  // roots, rank scan, labels
        hipLaunchKernelGGL(dbscan_roots_kernel, FP, dim3(256), 0, s, w.P, w.cnt, min_samples, w.parent, w.flag, fm);
        int rc = run_scan(w.flag, w.rank, w.P, P_N, 0, w.partial, w.nblk_pts, s, fm, frames);
        if (rc) return rc;
        hipLaunchKernelGGL(dbscan_labels_kernel, FP, dim3(256), 0, s, w.P, w.cid, w.cellstart, w.order, w.sxyz,
                           w.cnt, min_samples, w.parent, w.rank, w.core, labels, fm);
    }
    LAUNCH_CHECK();
    return LIDAR_OK;
}

// preprocess + DBSCAN + label scatter for `frames` frames (CSR rows, offs on the device;
// offs == nullptr: one frame of n points)
int run_preprocess(lidar_handle *h, const double *xyz, int64_t n, const int64_t *offs, int frames, uint8_t *mask,
                   double *colors, double *normals, double *compact_xyz, int64_t *labels, double *scalars,
                   hipStream_t s, double fixed_eps = 0.0)
{
    lidar::Carver cv;
    const uint64_t o_sc = cv.take<double>(3 * n);
    const uint64_t o_pos = cv.take<int32_t>(n);
    const uint64_t o_lab = cv.take<int64_t>(n);
    uint64_t off[kDbscanParts];
    plan_dbscan(cv, n, off);
    const uint64_t wss = lidar::align_up(cv.off, 256);
    char *base = static_cast<char *>(lidar::workspace(h, wss * (uint64_t)frames));
    if (!base) return LIDAR_ENOMEM;
    double *sc = reinterpret_cast<double *>(base + o_sc);
    int32_t *ng_pos = reinterpret_cast<int32_t *>(base + o_pos);
    int64_t *ng_lab = reinterpret_cast<int64_t *>(base + o_lab);
    DbscanWs w = bind_dbscan(base, off, n);
    FrameMap fm;
    fm.wss = (int64_t)wss;
    fm.offs = offs;
    HIP_TRY(hipMemsetAsync(scalars, 0, sizeof(double) * S_COUNT * frames, s));
    {
        lidar::Span sp(h, "preprocess", s);
        hipLaunchKernelGGL(preprocess_kernel, dim3(1, frames), dim3(kT), 0, s, xyz, n, mask, colors, normals,
                           compact_xyz, sc, ng_pos, scalars, fm, fixed_eps);
        hipLaunchKernelGGL(dbscan_params_from_preprocess, dim3(1, frames), dim3(64), 0, s, scalars, w.P, w.max_cells,
                           fm);
    }
    int rc = run_dbscan(h, sc, n, 5, w, ng_lab, s, fm, frames);
    if (rc) return rc;
    const unsigned gp = point_blocks(n, frames);
    lidar::Span sp(h, "label_scatter", s);
    hipLaunchKernelGGL(scatter_labels_kernel, dim3(gp, frames), dim3(256), 0, s, scalars, ng_lab, ng_pos, labels, fm);
    hipLaunchKernelGGL(scatter_labels2_kernel, dim3(gp, frames), dim3(256), 0, s, scalars, ng_lab, ng_pos, labels, fm);
    hipLaunchKernelGGL(nclust_kernel, dim3(1, frames), dim3(64), 0, s, w.P, scalars, fm);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

}  // namespace

// ====================================================================== C-ABI
LIDAR_EXPORT int lidar_dbscan_f64(lidar_handle *h, const double *x, int64_t n, double eps,
                                  int32_t min_samples, int64_t *labels, int32_t *counts, void *stream)
{
    REQUIRE(h && x && labels, "lidar_dbscan_f64: null pointer");
    REQUIRE(n >= 0 && n < 0x7fffffff, "lidar_dbscan_f64: n out of range");
    REQUIRE(eps > 0.0, "lidar_dbscan_f64: eps must be > 0");
    REQUIRE(min_samples >= 1, "lidar_dbscan_f64: min_samples must be >= 1");
    if (n == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    lidar::Carver cv;
    uint64_t off[kDbscanParts];
    plan_dbscan(cv, n, off);
    char *base = static_cast<char *>(lidar::workspace(h, cv.off));
    if (!base) return LIDAR_ENOMEM;
    DbscanWs w = bind_dbscan(base, off, n);
    double hp[P_COUNT] = {};
    hp[P_N] = (double)n;
    hp[P_EPS] = eps;
    hp[P_ACTIVE] = 1.0;
    HIP_TRY(hipMemcpyAsync(w.P, hp, sizeof hp, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(dbscan_bbox_kernel, dim3(1), dim3(kT), 0, s, x, w.P, FrameMap{});
    int rc = run_dbscan(h, x, n, min_samples, w, labels, s, FrameMap{}, 1, false, counts != nullptr);
    if (rc) return rc;
    if (counts) HIP_TRY(hipMemcpyAsync(counts, w.cnt, sizeof(int32_t) * n, hipMemcpyDeviceToDevice, s));
    // hp is a stack buffer: make sure the H2D copy has consumed it
    HIP_TRY(hipStreamSynchronize(s));
    return LIDAR_OK;
}

LIDAR_EXPORT int lidar_preprocess_f64(lidar_handle *h, const double *xyz, int64_t n, uint8_t *mask,
                                      double *colors, double *normals, double *compact_xyz,
                                      int64_t *labels, double *scalars, void *stream)
{
    REQUIRE(h && xyz && mask && colors && normals && compact_xyz && labels && scalars,
            "lidar_preprocess_f64: null pointer");
    REQUIRE(n >= 1 && n < 0x7fffffff, "lidar_preprocess_f64: need 1 <= n < 2^31");
    ON_DEVICE(h->device);
    return run_preprocess(h, xyz, n, nullptr, 1, mask, colors, normals, compact_xyz, labels, scalars,
                          static_cast<hipStream_t>(stream));
}

LIDAR_EXPORT int lidar_preprocess_batch_f64(lidar_handle *h, const double *xyz, const int64_t *offsets,
                                            int32_t frames, int64_t max_n, uint8_t *mask, double *colors,
                                            double *normals, double *compact_xyz, int64_t *labels,
                                            double *scalars, void *stream)
{
    REQUIRE(h && xyz && offsets && mask && colors && normals && compact_xyz && labels && scalars,
            "lidar_preprocess_batch_f64: null pointer");
    REQUIRE(frames >= 1 && frames <= 65535, "lidar_preprocess_batch_f64: need 1 <= frames <= 65535");
    REQUIRE(max_n >= 1 && max_n < 0x7fffffff, "lidar_preprocess_batch_f64: need 1 <= max_n < 2^31");
    ON_DEVICE(h->device);
    return run_preprocess(h, xyz, max_n, offsets, frames, mask, colors, normals, compact_xyz, labels, scalars,
                          static_cast<hipStream_t>(stream));
}

// the variant pipeline's preprocess (app_simplified.py:76-137, app_with_db.py:80-141):
// lidar_preprocess_batch_f64's phases with DBSCAN(eps, min_samples=5) on the unscaled
// non-ground points.  offsets == nullptr: one frame of max_n points.
LIDAR_EXPORT int lidar_preprocess_eps_batch_f64(lidar_handle *h, const double *xyz, const int64_t *offsets,
                                                int32_t frames, int64_t max_n, double eps, uint8_t *mask,
                                                double *colors, double *normals, double *compact_xyz,
                                                int64_t *labels, double *scalars, void *stream)
{
    REQUIRE(h && xyz && mask && colors && normals && compact_xyz && labels && scalars,
            "lidar_preprocess_eps_batch_f64: null pointer");
    REQUIRE(frames >= 1 && frames <= 65535 && (offsets || frames == 1),
            "lidar_preprocess_eps_batch_f64: need 1 <= frames <= 65535 (offsets for frames > 1)");
    REQUIRE(max_n >= 1 && max_n < 0x7fffffff, "lidar_preprocess_eps_batch_f64: need 1 <= max_n < 2^31");
    REQUIRE(eps > 0.0 && eps < INFINITY, "lidar_preprocess_eps_batch_f64: eps must be finite and > 0");
    ON_DEVICE(h->device);
    return run_preprocess(h, xyz, max_n, offsets, frames, mask, colors, normals, compact_xyz, labels, scalars,
                          static_cast<hipStream_t>(stream), eps);
}

LIDAR_EXPORT int lidar_people_f64(lidar_handle *h, const double *xyz, const int64_t *labels, int64_t n,
                                  double *people, int64_t *k_host, void *stream)
{
    REQUIRE(h && xyz && labels && people && k_host, "lidar_people_f64: null pointer");
    REQUIRE(n >= 0, "lidar_people_f64: n < 0");
    *k_host = 0;
    if (n == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int64_t *kd = static_cast<int64_t *>(lidar::workspace(h, 256));
    if (!kd) return LIDAR_ENOMEM;
    HIP_TRY(hipMemsetAsync(kd, 0, sizeof(int64_t), s));
    const unsigned gp = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1024));
    hipLaunchKernelGGL(max_label_kernel, dim3(gp), dim3(256), 0, s, labels, n, kd, nullptr, FrameMap{});
    hipLaunchKernelGGL(people_kernel, dim3(256), dim3(kT), 0, s, xyz, labels, n, kd, people, nullptr, FrameMap{});
    LAUNCH_CHECK();
    int64_t *hk = static_cast<int64_t *>(h->host_pinned);
    HIP_TRY(hipMemcpyAsync(hk, kd, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *k_host = *hk;
    return LIDAR_OK;
}

LIDAR_EXPORT int lidar_grid_dims(double xmin, double xmax, double ymin, double ymax, double grid,
                                 int64_t *nx, int64_t *ny)
{
    REQUIRE(nx && ny && grid > 0.0, "lidar_grid_dims: bad arguments");
    // data_processing.py:305-313: margin 2g, np.arange(min - 2g, max + 2g + g, g)
    const double m = grid * 2.0;
    const double x0 = xmin - m, x1 = (xmax + m) + grid;
    const double y0 = ymin - m, y1 = (ymax + m) + grid;
    const double lx = std::ceil((x1 - x0) / grid), ly = std::ceil((y1 - y0) / grid);
    // numpy's errors (np.arange, then histogram2d's (nx, ny) float64 array): a length it cannot
    // compute or hold (not finite, >= 2^63 elements, or >= 2^63 bytes) is a ValueError ("Maximum
    // allowed size exceeded" / "array is too big") -> LIDAR_EINVAL; a representable grid of more
    // than 2^40 cells (8 TiB of float64) a MemoryError -> LIDAR_ENOMEM
    const double kBig = 1152921504606846976.0;  // 2^60 float64 elements = 2^63 bytes
    if (!(std::isfinite(lx) && std::isfinite(ly) && lx < kBig && ly < kBig && (lx - 1) * (ly - 1) < kBig)) {
        lidar::set_error("lidar_grid_dims: Maximum allowed size exceeded");
        return LIDAR_EINVAL;
    }
    REQUIRE(lx >= 2 && ly >= 2, "lidar_grid_dims: degenerate grid");
    if ((lx - 1) * (ly - 1) > 1099511627776.0) {
        lidar::set_error("lidar_grid_dims: the grid has more than 2^40 cells");
        return LIDAR_ENOMEM;
    }
    *nx = (int64_t)lx - 1;
    *ny = (int64_t)ly - 1;
    return LIDAR_OK;
}

// people (k, 2) -> grid_x (nx), grid_y (ny), density (nx*ny), flat_x, flat_y (nx*ny),
// stats [max, avg, thr, n_hot, n_occupied, k], hot (5) int64.  `out` layout (doubles):
// grid_x | grid_y | density | flat_x | flat_y | stats(8) | hot(5, int64)
LIDAR_EXPORT int lidar_density_grid_f64(lidar_handle *h, const double *people, int64_t k, double xmin,
                                        double xmax, double ymin, double ymax, double grid, int64_t nx,
                                        int64_t ny, double *grid_x, double *grid_y, double *density,
                                        void *stream)
{
    REQUIRE(h && people && grid_x && grid_y && density, "lidar_density_grid_f64: null pointer");
    REQUIRE(nx >= 1 && ny >= 1 && k >= 0, "lidar_density_grid_f64: bad sizes");
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    lidar::Carver cv;
    const uint64_t o_xe = cv.take<double>(nx + 1), o_ye = cv.take<double>(ny + 1);
    const uint64_t o_cnt = cv.take<uint32_t>(nx * ny), o_pos = cv.take<double>(nx * ny);
    const uint64_t o_k = cv.take<int64_t>(1);
    char *base = static_cast<char *>(lidar::workspace(h, cv.off));
    if (!base) return LIDAR_ENOMEM;
    int64_t *kd = reinterpret_cast<int64_t *>(base + o_k);
    int64_t *hk = static_cast<int64_t *>(h->host_pinned);
    *hk = k;
    HIP_TRY(hipMemcpyAsync(kd, hk, sizeof(int64_t), hipMemcpyHostToDevice, s));
    const double m = grid * 2.0;
    // density points at: density (nx*ny) | flat_x | flat_y | stats (8) | hot (5)
    double *flat_x = density + nx * ny, *flat_y = flat_x + nx * ny, *stats = flat_y + nx * ny;
    int64_t *hot = reinterpret_cast<int64_t *>(stats + 8);
    hipLaunchKernelGGL(density_kernel, dim3(1), dim3(kT), 0, s, people, kd, xmin - m, ymin - m, grid, nx, ny,
                       reinterpret_cast<double *>(base + o_xe), reinterpret_cast<double *>(base + o_ye),
                       reinterpret_cast<uint32_t *>(base + o_cnt), grid_x, grid_y, density, flat_x, flat_y,
                       reinterpret_cast<double *>(base + o_pos), stats, hot);
    LAUNCH_CHECK();
    HIP_TRY(hipStreamSynchronize(s));  // hk is reused by the next call
    return LIDAR_OK;
}

// people of every frame of a preprocess batch (CSR rows, device offsets, scalars of the
// batch): people rows of frame f start at row offsets[f]; kdev (device int64[frames])
// receives K per frame.  Asynchronous.
LIDAR_EXPORT int lidar_people_batch_f64(lidar_handle *h, const double *compact_xyz, const int64_t *labels,
                                        const int64_t *offsets, int32_t frames, int64_t max_n,
                                        const double *scalars, double *people, int64_t *kdev, void *stream)
{
    REQUIRE(h && compact_xyz && labels && offsets && scalars && people && kdev, "lidar_people_batch_f64: null pointer");
    REQUIRE(frames >= 1 && frames <= 65535 && max_n >= 1, "lidar_people_batch_f64: bad sizes");
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    FrameMap fm;
    fm.offs = offsets;
    HIP_TRY(hipMemsetAsync(kdev, 0, sizeof(int64_t) * frames, s));
    lidar::Span sp(h, "people", s);
    hipLaunchKernelGGL(max_label_kernel, dim3(point_blocks(max_n, frames), frames), dim3(256), 0, s, labels, max_n,
                       kdev, scalars, fm);
    const unsigned pb = (unsigned)std::max(1, std::min(256, 2048 / std::max(1, (int)frames)));
    hipLaunchKernelGGL(people_kernel, dim3(pb, frames), dim3(kT), 0, s, compact_xyz, labels, max_n, kdev, people,
                       scalars, fm);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

// density grids of every frame (see density_batch_kernel for the job / output layout);
// scratch_doubles = the sum over frames of nx*ny + ceil(nx*ny/2) + nx + ny + 2.  Asynchronous.
LIDAR_EXPORT int lidar_density_batch_f64(lidar_handle *h, const double *people, const int64_t *offsets,
                                         const int64_t *kdev, int32_t frames, const double *jobs, double *out,
                                         int64_t scratch_doubles, void *stream)
{
    REQUIRE(h && people && offsets && kdev && jobs && out, "lidar_density_batch_f64: null pointer");
    REQUIRE(frames >= 1 && frames <= 65535 && scratch_doubles >= 0, "lidar_density_batch_f64: bad sizes");
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    double *scratch = static_cast<double *>(lidar::workspace(h, (uint64_t)std::max<int64_t>(1, scratch_doubles) * 8));
    if (!scratch) return LIDAR_ENOMEM;
    lidar::Span sp(h, "density_grid", s);
    hipLaunchKernelGGL(density_batch_kernel, dim3(1, frames), dim3(kT), 0, s, people, offsets, kdev, jobs, out,
                       scratch);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

__global__ void widen_counts_kernel(const int32_t *c, int64_t n, int64_t *out)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = c[i];
}

// KDTree(x).query_radius(x, r, count_only=True) (the reference's density colouring,
// utils/visualization.py:41-48 and :165-168, app_simplified.py:156-159): per point the
// number of points (itself included) with ((dx*dx + dy*dy) + dz*dz) <= r*r in fp64 —
// sklearn's rdist test, the one DBSCAN's neighbour count uses.  2-D data: z = 0.
LIDAR_EXPORT int lidar_radius_count_f64(lidar_handle *h, const double *x, int64_t n, double r, int64_t *counts,
                                        void *stream)
{
    REQUIRE(h && x && counts, "lidar_radius_count_f64: null pointer");
    REQUIRE(n >= 0 && n < 0x7fffffff, "lidar_radius_count_f64: n out of range");
    REQUIRE(r >= 0.0, "lidar_radius_count_f64: r must be >= 0");
    if (n == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    lidar::Carver cv;
    uint64_t off[kDbscanParts];
    plan_dbscan(cv, n, off);
    char *base = static_cast<char *>(lidar::workspace(h, cv.off));
    if (!base) return LIDAR_ENOMEM;
    DbscanWs w = bind_dbscan(base, off, n);
    double *hp = static_cast<double *>(h->host_pinned);
    for (int i = 0; i < P_COUNT; ++i) hp[i] = 0.0;
    hp[P_N] = (double)n;
    // r = 0: a tiny positive cell size keeps the grid finite; only exact duplicates count
    hp[P_EPS] = r > 0.0 ? r : 1e-300;
    hp[P_ACTIVE] = 1.0;
    HIP_TRY(hipMemcpyAsync(w.P, hp, sizeof(double) * P_COUNT, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(dbscan_bbox_kernel, dim3(1), dim3(kT), 0, s, x, w.P, FrameMap{});
    int rc = run_dbscan(h, x, n, 1, w, nullptr, s, FrameMap{}, 1, true);
    if (rc) return rc;
    hipLaunchKernelGGL(widen_counts_kernel, dim3(point_blocks(n, 1)), dim3(256), 0, s, w.cnt, n, counts);
    LAUNCH_CHECK();
    HIP_TRY(hipStreamSynchronize(s));  // the pinned parameter block is reused by the next call
    return LIDAR_OK;
}

// np.histogram2d(a, b, bins=(bx, by), range=...) binning (the reference's heatmaps,
// utils/visualization.py:125-137, app_simplified.py:205-209): the edges are numpy's own
// (np.linspace, passed in); a value lands in bin searchsorted(edges, v, 'right') - 1, a value
// equal to the last edge in the last bin, anything outside (or NaN) nowhere.  counts is
// bx * by float64 (row-major, a-bins x b-bins), zeroed here.
__global__ void hist2d_kernel(const double *a, const double *b, int64_t n, const double *xe, int64_t bx,
                              const double *ye, int64_t by, unsigned long long *cnt)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double va = a[i], vb = b[i];
        int64_t ia = searchsorted_right(xe, bx + 1, va), ib = searchsorted_right(ye, by + 1, vb);
        if (va == xe[bx]) --ia;
        if (vb == ye[by]) --ib;
        if (ia >= 1 && ia <= bx && ib >= 1 && ib <= by) atomicAdd(&cnt[(ia - 1) * by + (ib - 1)], 1ull);
    }
}
__global__ void hist2d_finish_kernel(const unsigned long long *cnt, int64_t m, double *out)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (double)cnt[i];
}

LIDAR_EXPORT int lidar_histogram2d_f64(lidar_handle *h, const double *a, const double *b, int64_t n,
                                       const double *xedges, int64_t bx, const double *yedges, int64_t by,
                                       double *counts, void *stream)
{
    REQUIRE(h && xedges && yedges && counts && (n == 0 || (a && b)), "lidar_histogram2d_f64: null pointer");
    REQUIRE(n >= 0 && bx >= 1 && by >= 1, "lidar_histogram2d_f64: bad sizes");
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t m = bx * by;
    auto *cnt = static_cast<unsigned long long *>(lidar::workspace(h, (uint64_t)m * 8));
    if (!cnt) return LIDAR_ENOMEM;
    HIP_TRY(hipMemsetAsync(cnt, 0, (size_t)m * 8, s));
    if (n > 0)
        hipLaunchKernelGGL(hist2d_kernel, dim3(point_blocks(n, 1)), dim3(256), 0, s, a, b, n, xedges, bx, yedges, by,
                           cnt);
    hipLaunchKernelGGL(hist2d_finish_kernel, dim3(point_blocks(m, 1)), dim3(256), 0, s, cnt, m, counts);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

// the variant's grid density (app_simplified.py:262-282, app_with_db.py:266-286): cell (i, j)
// of the edges xg (nxg), yg (nyg) has centre ((xg[i] + xg[i+1]) / 2, (yg[j] + yg[j+1]) / 2);
// out[j * (nxg - 1) + i] = #{people p : (cx - px)^2 + (cy - py)^2 <= r*r} / divisor — the
// count of KDTree(people).query_radius([centre], r) (sklearn's rdist test, no FMA).
__global__ void cell_radius_density_kernel(const double *__restrict__ people, int64_t k,
                                           const double *__restrict__ xg, int64_t nx,
                                           const double *__restrict__ yg, int64_t ny, double r2, double divisor,
                                           double *__restrict__ out)
{
    extern __shared__ double pp[];  // people tile (x, y)
    const int64_t m = nx * ny;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < m; base += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = base + threadIdx.x;
        double cx = 0.0, cy = 0.0;
        if (c < m) {
            const int64_t i = c % nx, j = c / nx;
            cx = ddiv(dadd(xg[i], xg[i + 1]), 2.0);
            cy = ddiv(dadd(yg[j], yg[j + 1]), 2.0);
        }
        int64_t cnt = 0;
        for (int64_t t0 = 0; t0 < k; t0 += blockDim.x) {
            const int64_t tn = k - t0 < (int64_t)blockDim.x ? k - t0 : (int64_t)blockDim.x;
            __syncthreads();
            if (threadIdx.x < tn) {
                pp[2 * threadIdx.x] = people[2 * (t0 + threadIdx.x)];
                pp[2 * threadIdx.x + 1] = people[2 * (t0 + threadIdx.x) + 1];
            }
            __syncthreads();
            for (int64_t u = 0; u < tn; ++u) {
                const double dx = dsub(cx, pp[2 * u]), dy = dsub(cy, pp[2 * u + 1]);
                cnt += dadd(dmul(dx, dx), dmul(dy, dy)) <= r2;
            }
        }
        if (c < m) out[c] = ddiv((double)cnt, divisor);  // row j = c / nx, column i = c % nx
    }
}

LIDAR_EXPORT int lidar_cell_radius_density_f64(lidar_handle *h, const double *people, int64_t k, const double *xg,
                                               int64_t nxg, const double *yg, int64_t nyg, double r, double divisor,
                                               double *out, void *stream)
{
    REQUIRE(h && xg && yg && out && (k == 0 || people), "lidar_cell_radius_density_f64: null pointer");
    REQUIRE(k >= 0 && nxg >= 2 && nyg >= 2, "lidar_cell_radius_density_f64: bad sizes");
    REQUIRE(r >= 0.0 && divisor != 0.0, "lidar_cell_radius_density_f64: bad r / divisor");
    ON_DEVICE(h->device);
    const int64_t nx = nxg - 1, ny = nyg - 1, m = nx * ny;
    const int64_t blocks = std::min<int64_t>((m + 255) / 256, 65535);
    hipLaunchKernelGGL(cell_radius_density_kernel, dim3((unsigned)blocks), dim3(256), 2 * 256 * sizeof(double),
                       static_cast<hipStream_t>(stream), people, k, xg, nx, yg, ny, r * r, divisor, out);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

// ------------------------------------------------------------------ venue grid
// calculate_grid_density's binning (utils/data_processing.py:312-319) over a FIXED venue grid:
// edges np.arange(x0, ..., g) (e[0] = a, e[1] = a + g, e[i] = a + i * ((a + g) - a), numpy's
// DOUBLE_fill), searchsorted right with the last edge closed, points outside dropped.  Counts
// add into int32 cells, so the frames of a rank and then the ranks (one RCCL all-reduce) sum.
__device__ __forceinline__ double arange_edge(double a, double g, int64_t i)
{
    return i == 0 ? a : (i == 1 ? dadd(a, g) : dadd(a, dmul((double)i, dsub(dadd(a, g), a))));
}
__device__ __forceinline__ int64_t arange_bin(double a, double g, int64_t nb, double v)
{
    int64_t lo = 0, hi = nb + 1;  // first edge index with e[idx] > v
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (arange_edge(a, g, mid) <= v) lo = mid + 1;
        else hi = mid;
    }
    if (v == arange_edge(a, g, nb)) --lo;  // the last edge is closed
    return lo;                             // bin lo - 1 when 1 <= lo <= nb
}
__global__ void venue_counts_kernel(const double *__restrict__ people, int64_t k, double x0, double y0, double g,
                                    int64_t nx, int64_t ny, int32_t *__restrict__ counts)
{
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < k; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t bx = arange_bin(x0, g, nx, people[2 * i]), by = arange_bin(y0, g, ny, people[2 * i + 1]);
        if (bx >= 1 && bx <= nx && by >= 1 && by <= ny) atomicAdd(&counts[(bx - 1) * ny + (by - 1)], 1);
    }
}

LIDAR_EXPORT int lidar_venue_counts_f64(lidar_handle *h, const double *people, int64_t k, double x0, double y0,
                                        double grid, int64_t nx, int64_t ny, int32_t *counts, void *stream)
{
    REQUIRE(h && counts && (k == 0 || people), "lidar_venue_counts_f64: null pointer");
    REQUIRE(k >= 0 && nx >= 1 && ny >= 1 && grid > 0.0, "lidar_venue_counts_f64: bad sizes");
    if (k == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    const unsigned blocks = (unsigned)std::min<int64_t>((k + 255) / 256, 4096);
    hipLaunchKernelGGL(venue_counts_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), people, k,
                       x0, y0, grid, nx, ny, counts);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
