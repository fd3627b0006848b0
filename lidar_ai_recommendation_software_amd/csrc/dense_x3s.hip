// dense_x3s.hip — the x3 dense GEMM (SA2's per-point layer 1, group_all's three layers).
//
// Splitting every fp32 activation into bf16 hi / lo inside the GEMM loop costs each element one
// split per wave that reads it and per column tile of the grid (~4 VALU per MFMA, which left the
// MFMA pipe ~30 % busy in round 1's first x3 GEMM).  Here the activations arrive split: two bf16
// planes (hi, lo) of row-major (rows, lda)
// elements, lda a multiple of 32, elements k >= K zero — written once, by the producing
// layer's epilogue (mode 1 below) or by lidar_split_x3_f32 from fp32 rows.  A product is still
// ah*bh + ah*bl + al*bh on v_mfma_f32_32x32x16_bf16 with fp32 accumulation (the x3 contract of
// DESIGN.md §3), so results are the x3 contract's up to the accumulation order.
//
// Tile: 128 rows x 128 output channels per 4-wave workgroup (64 x 64 per wave = 2 x 2 MFMA
// tiles), K in stages of 32 double-buffered in LDS by global_load_lds:
//   A stage: per plane 128 rows x 64 B; row r's 16-byte chunk q (8 consecutive k) sits at slot
//            q ^ ((r >> 2) & 3), so the fragment reads (ds_read_b128, 32 consecutive rows, one
//            chunk) hit 16 distinct 16-byte bank groups per 16 lanes;
//   B stage: x3_pack.hip's packed weight fragments (lidar_dense_x3_pack_f32), read lane-linear.
// Output modes:
//   0 fp32 rows (rows, ldo) [+ ReLU]             — computed transposed (D = W^T X^T): a lane
//   1 split planes (rows, ldo) x 2 [+ ReLU]        holds 4 consecutive channels of one row, so
//                                                   a store is 16 B (fp32) or 8 B per plane
//   2 fp32 max-pool over runs of pool_rows rows  — computed untransposed (rows in registers:
//     (rows / pool_rows, ldo), ReLU, out zeroed     the pool is a register max + one swap, then
//     by the caller                                 an atomic max on the bits, exact)
#include "common.hpp"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef DENSE_SBK
#define DENSE_SBK 32
#endif
constexpr int SBM = 128, SBN = 128, SBK = DENSE_SBK;  // K per LDS stage: 32 (64 KiB of LDS) or 16 (32 KiB)
constexpr int NSS = SBK / 16;                        // MFMA k-steps per stage
constexpr int CPR = SBK / 8;                         // 16-byte chunks per A row and plane
constexpr int kPlaneStage = SBM * SBK;               // bf16 per plane per A stage
constexpr int kStageB = 4 * 2 * NSS * 512;           // bf16 per B stage
static_assert(SBK == 16 || SBK == 32, "DENSE_SBK must be 16 or 32");
// chunk swizzle: row r's chunk q sits at slot q ^ sw(r), so a fragment read (32 consecutive rows,
// one chunk) hits 16 distinct 16-byte bank groups per 16 lanes
__device__ __forceinline__ int swz(int r) { return CPR == 4 ? (r >> 2) & 3 : (r >> 3) & 1; }
__device__ __forceinline__ int swzf(int r) { return CPR == 4 ? (r >> 1) & 7 : (r >> 2) & 3; }  // fp32 rows

__host__ __device__ constexpr int rho(int r) { return (r & 3) + 8 * (r >> 2); }

__device__ __forceinline__ f32x16 mfma_bf(bf16x8 a, bf16x8 b, f32x16 c)
{
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void lds_dma16(const void *g, void *l)
{
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)l, 16, 0, 0);
}

__device__ __forceinline__ float relu_i(float v) { return __int_as_float(max(__float_as_int(v), 0)); }

__device__ __forceinline__ void split8(const f32x4 &a0, const f32x4 &a1, bf16x8 &hi, bf16x8 &lo)
{
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v = j < 4 ? a0[j] : a1[j - 4];
        const __bf16 hb = (__bf16)v;
        hi[j] = hb;
        lo[j] = (__bf16)(v - (float)hb);
    }
}

// MODE 0 / 1 / 2 as in the header.  AF32: A is fp32 rows (rows, lda) instead of split planes
// (a layer whose input nobody split, e.g. the first of a chain: the A stage holds 128 rows x
// 32 fp32 with row r's chunk q at slot q ^ ((r >> 1) & 7), and each wave splits the fragments
// it reads; worth it where cout / 128 column tiles re-read little)
// X1: one product ah*bh per MFMA — bf16(x) bf16(w) with fp32 accumulation, the bf16 spec's
// arithmetic (BASELINE configs[4]), on the same operands
template <int MODE, bool AF32, bool X1 = false>
__global__ __launch_bounds__(256, 2) void dense_x3s_kernel(const __bf16 *__restrict__ a, int64_t a_plane, int lda,
                                                           const __bf16 *__restrict__ wp, int ks,
                                                           const float *__restrict__ bias, int relu_on,
                                                           int pool_rows, void *__restrict__ out, int64_t o_plane,
                                                           int64_t ldo, int cout, int ntn, int64_t total,
                                                           int64_t per_xcd, int kdim)
{
    constexpr bool TRANS = MODE != 2;
    // the two stage buffers are separate LDS variables (distinct alias scopes) and the stage loop is
    // unrolled by two, so a stage's reads need not wait for the next stage streaming into the other
    // buffer (with one array indexed by st & 1 the compiler waited for the stage it had just issued)
    __shared__ __attribute__((aligned(16))) __bf16 As0[2][kPlaneStage], As1[2][kPlaneStage];
    __shared__ __attribute__((aligned(16))) __bf16 Bs0[kStageB], Bs1[kStageB];
    auto Asb = [&](int buf) { return buf ? As1 : As0; };
    auto Bsb = [&](int buf) { return buf ? Bs1 : Bs0; };
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5, col = lane & 31;
    const int wm = wave >> 1, wn = wave & 1;
    const int64_t L = blockIdx.x;
    const int64_t logical = (L & 7) * per_xcd + (L >> 3);  // a row tile's column tiles share an XCD
    if (logical >= total) return;                           // whole workgroup
    const int64_t row0 = logical / ntn * SBM;
    const int tn = (int)(logical % ntn);
    // stages that hold k < kdim (a 16-deep stage past kdim would be all padding: zero weights, and
    // for fp32 rows a read past the row)
    const int nst = (kdim + SBK - 1) / SBK;

    // A: wave w loads plane w >> 1, rows 64 (w & 1) .. +63: CPR instructions of 64 / CPR rows;
    // lane i of instruction t fills slot i % CPR of row (64 / CPR) t + i / CPR with chunk slot ^ swz(row)
    const int pl = wave >> 1, rbase = 64 * (wave & 1);
    const __bf16 *ap = a + pl * a_plane;
    const float *af = reinterpret_cast<const float *>(a);
    auto load_stage = [&](int st, int buf) {
        const int k0 = st * SBK;
        if constexpr (AF32) {  // wave w: rows 32 w .. 32 w + 31 of 2 CPR 16-byte chunks, CPR instructions
            constexpr int CF = 2 * CPR, RPI = 64 / CF;
            float *dst = reinterpret_cast<float *>(&Asb(buf)[0][0]);
#pragma unroll
            for (int i = 0; i < CPR; ++i) {
                const int r = 32 * wave + RPI * i + lane / CF;
                const int kq = (lane % CF) ^ swzf(r);
                // chunks at or past k (the weights there are zero) re-read the stage's first
                // chunk: finite, in bounds, and no stale LDS in the products
                const int kc = k0 + 4 * kq < kdim ? k0 + 4 * kq : k0;
                lds_dma16(af + (row0 + r) * lda + kc, dst + (32 * wave + RPI * i) * SBK);
            }
        } else {
            constexpr int RPI = 64 / CPR;
#pragma unroll
            for (int t = 0; t < CPR; ++t) {
                const int r = rbase + RPI * t + lane / CPR;
                const int q = (lane % CPR) ^ swz(r);
                lds_dma16(ap + (row0 + r) * lda + k0 + 8 * q, &Asb(buf)[pl][(rbase + RPI * t) * SBK]);
            }
        }
        // B: wave w loads column tile 4 tn + w, k-steps NSS st .. NSS st + NSS - 1, hi / lo (contiguous)
        const __bf16 *src = wp + (((int64_t)(4 * tn + wave) * ks + NSS * st) * 2) * 512;
#pragma unroll
        for (int i = 0; i < 2 * NSS; ++i) lds_dma16(src + i * 512 + lane * 8, &Bsb(buf)[(wave * 2 * NSS + i) * 512]);
        __builtin_amdgcn_sched_barrier(0);  // issued before the stage's reads and MFMAs
    };

    f32x16 acc[2][2] = {};
    auto compute = [&](int buf) {
#pragma unroll
        for (int ss = 0; ss < NSS; ++ss) {
            bf16x8 xh[2], xl[2], wh[2], wl[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = wm * 64 + i * 32 + col;
                if constexpr (AF32) {
                    const float *as = reinterpret_cast<const float *>(&Asb(buf)[0][0]);
                    const int kq = 4 * ss + 2 * h;
                    const int sl = kq ^ swzf(r);  // kq even: the pair (sl, sl ^ 1)
                    const f32x4 a0 = *reinterpret_cast<const f32x4 *>(as + r * SBK + 4 * sl);
                    const f32x4 a1 = *reinterpret_cast<const f32x4 *>(as + r * SBK + 4 * (sl ^ 1));
                    split8(a0, a1, xh[i], xl[i]);
                } else {
                    const int slot = (2 * ss + h) ^ swz(r);
                    xh[i] = *reinterpret_cast<const bf16x8 *>(&Asb(buf)[0][(r * CPR + slot) * 8]);
                    xl[i] = *reinterpret_cast<const bf16x8 *>(&Asb(buf)[1][(r * CPR + slot) * 8]);
                }
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int tt = 2 * wn + j;
                wh[j] = *reinterpret_cast<const bf16x8 *>(&Bsb(buf)[((tt * NSS + ss) * 2 + 0) * 512 + lane * 8]);
                wl[j] = *reinterpret_cast<const bf16x8 *>(&Bsb(buf)[((tt * NSS + ss) * 2 + 1) * 512 + lane * 8]);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if constexpr (TRANS && X1) {
                        acc[i][j] = mfma_bf(wh[j], xh[i], acc[i][j]);
                    } else if constexpr (TRANS) {  // D[channel][row]
                        acc[i][j] = mfma_bf(wh[j], xh[i], acc[i][j]);
                        acc[i][j] = mfma_bf(wl[j], xh[i], acc[i][j]);
                        acc[i][j] = mfma_bf(wh[j], xl[i], acc[i][j]);
                    } else {  // D[row][channel]
                        acc[i][j] = mfma_bf(xh[i], wh[j], acc[i][j]);
                        acc[i][j] = mfma_bf(xh[i], wl[j], acc[i][j]);
                        acc[i][j] = mfma_bf(xl[i], wh[j], acc[i][j]);
                    }
                }
        }
    };
    load_stage(0, 0);
    for (int st = 0; st < nst; st += 2) {
        __syncthreads();  // (vmcnt(0)) stage st landed everywhere; buffer 1 no longer read
        if (st + 1 < nst) load_stage(st + 1, 1);
        compute(0);
        if (st + 1 < nst) {
            __syncthreads();  // stage st + 1 landed; buffer 0 no longer read
            if (st + 2 < nst) load_stage(st + 2, 0);
            compute(1);
        }
    }

    const int cbase = tn * SBN + wn * 64;
    if constexpr (TRANS) {
        // lane (col, h) of tile (i, j): row row0 + 64 wm + 32 i + col, channels
        // cbase + 32 j + 8 g + 4 h + t (register 4 g + t)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int64_t row = row0 + wm * 64 + i * 32 + col;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int c = cbase + 32 * j + 8 * g + 4 * h;
                    const f32x4 b4 = *reinterpret_cast<const f32x4 *>(bias + c);
                    f32x4 v;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const float y = acc[i][j][4 * g + t] + b4[t];
                        v[t] = relu_on ? relu_i(y) : y;
                    }
                    if constexpr (MODE == 0) {
                        *reinterpret_cast<f32x4 *>(static_cast<float *>(out) + row * ldo + c) = v;
                    } else {
                        bf16x4 hi, lo;
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const __bf16 hb = (__bf16)v[t];
                            hi[t] = hb;
                            lo[t] = (__bf16)(v[t] - (float)hb);
                        }
                        __bf16 *o = static_cast<__bf16 *>(out) + row * ldo + c;
                        *reinterpret_cast<bf16x4 *>(o) = hi;
                        *reinterpret_cast<bf16x4 *>(o + o_plane) = lo;
                    }
                }
        }
    } else {
        // lane (col, h) of tile (i, j): channel cbase + 32 j + col, rows 64 wm + 32 i + rho(r) + 4 h
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = cbase + j * 32 + col;
            float v = -INFINITY;  // raw accumulators: the bias and ReLU come after the max
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) v = __builtin_elementwise_maximum(v, acc[i][j][r]);
            v = __builtin_elementwise_maximum(v, __shfl_xor(v, 32, 64));
            // relu(max + b) == max relu(x + b): x -> relu(x + b) is monotone in fp32
            v = relu_i(v + bias[c]);
            if (h == 0) {  // non-negative floats order as their bits: exact, order-free
                unsigned *dst = reinterpret_cast<unsigned *>(static_cast<float *>(out) + (row0 / pool_rows) * ldo + c);
                atomicMax(dst, __float_as_uint(v));
            }
        }
    }
}

// fp32 rows (rows, k) with row stride ldx -> split planes (rows, lda), k..lda-1 zero; one thread
// per 8 elements (one 16-byte chunk per plane)
__global__ void split_x3_kernel(const float *__restrict__ x, int64_t rows, int k, int64_t ldx,
                                __bf16 *__restrict__ planes, int64_t plane, int lda)
{
    const int chunks = lda / 8;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * chunks) return;
    const int64_t r = i / chunks;
    const int c0 = (int)(i % chunks) * 8;
    bf16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v = c0 + j < k ? x[r * ldx + c0 + j] : 0.0f;
        const __bf16 hb = (__bf16)v;
        hi[j] = hb;
        lo[j] = (__bf16)(v - (float)hb);
    }
    *reinterpret_cast<bf16x8 *>(planes + r * lda + c0) = hi;
    *reinterpret_cast<bf16x8 *>(planes + plane + r * lda + c0) = lo;
}

}  // namespace

static int dense_x3s_launch(lidar_handle *h, const void *a_planes, int64_t a_plane, int32_t lda, int64_t rows,
                            int32_t k, const void *packed, const float *bias, int32_t cout, int32_t mode,
                            int32_t relu_on, int32_t pool_rows, void *out, int64_t o_plane, int64_t ldo, void *stream)
{
    const bool af32 = a_plane == 0;
    const bool x1 = (mode & 4) != 0;  // the bf16 spec: one ah*bh product (fp32 rows in and out only)
    mode &= 3;
    REQUIRE(!x1 || (af32 && mode == 0), "lidar_dense_x3s_f32: the X1 flag needs fp32 rows in and mode 0");
    REQUIRE(h && a_planes && packed && bias && out, "lidar_dense_x3s_f32: null pointer");
    REQUIRE(rows % SBM == 0 && k > 0 && k <= lda && cout % SBN == 0 && cout > 0,
            "lidar_dense_x3s_f32: rows % 128, k <= lda, cout % 128 must hold");
    // split planes: lda = k rounded up to 32 (zeros past k); fp32 rows: any row stride, k % 4
    REQUIRE(af32 ? (k % 4 == 0 && lda % 4 == 0) : lda == (k + 31) / 32 * 32,
            "lidar_dense_x3s_f32: planes need lda = k rounded up to 32; fp32 rows need k % 4 == 0 and lda % 4 == 0");
    REQUIRE(af32 || (a_plane >= rows * lda && a_plane % 8 == 0),
            "lidar_dense_x3s_f32: a_plane < rows * lda or not 16-B aligned");
    REQUIRE(mode >= 0 && mode <= 2, "lidar_dense_x3s_f32: mode must be 0, 1 or 2");
    REQUIRE(ldo >= cout && ldo % 4 == 0, "lidar_dense_x3s_f32: ldo must be >= cout and a multiple of 4");
    REQUIRE(mode != 1 || (o_plane >= rows * ldo && o_plane % 4 == 0), "lidar_dense_x3s_f32: o_plane < rows * ldo or misaligned");
    REQUIRE(mode != 2 || (relu_on && pool_rows > 0 && pool_rows % SBM == 0 && rows % pool_rows == 0),
            "lidar_dense_x3s_f32: the max-pool needs relu and pool_rows a multiple of 128 dividing rows");
    if (rows == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    const int ks = (k + 31) / 32 * 2;  // the packed image of a (k, cout) layer covers ceil(k/32)*2 k-steps
    const int ntn = cout / SBN;
    const int64_t total = (rows / SBM) * ntn, per_xcd = (total + 7) / 8;
    REQUIRE(per_xcd * 8 <= 0x7fffffff, "lidar_dense_x3s_f32: too many rows");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const __bf16 *a = static_cast<const __bf16 *>(a_planes);
    const __bf16 *w = static_cast<const __bf16 *>(packed);
    const dim3 grid((unsigned)(per_xcd * 8)), block(256);
    auto go = [&](auto kern, int relu, int pool) {
        hipLaunchKernelGGL(kern, grid, block, 0, s, a, a_plane, (int)lda, w, ks, bias, relu, pool, out, o_plane, ldo,
                           (int)cout, ntn, total, per_xcd, (int)k);
    };
    const int rl = relu_on ? 1 : 0;
    if (x1) go(dense_x3s_kernel<0, true, true>, rl, 0);
    else if (mode == 0) af32 ? go(dense_x3s_kernel<0, true>, rl, 0) : go(dense_x3s_kernel<0, false>, rl, 0);
    else if (mode == 1) af32 ? go(dense_x3s_kernel<1, true>, rl, 0) : go(dense_x3s_kernel<1, false>, rl, 0);
    else af32 ? go(dense_x3s_kernel<2, true>, 1, (int)pool_rows) : go(dense_x3s_kernel<2, false>, 1, (int)pool_rows);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

// the GEMM on split planes (see the header comment; mode 0 fp32 rows, 1 split planes, 2 max-pool)
LIDAR_EXPORT int lidar_dense_x3s_f32(lidar_handle *h, const void *a_planes, int64_t a_plane, int32_t lda,
                                     int64_t rows, int32_t k, const void *packed, const float *bias, int32_t cout,
                                     int32_t mode, int32_t relu_on, int32_t pool_rows, void *out, int64_t o_plane,
                                     int64_t ldo, void *stream)
{
    REQUIRE(a_plane > 0, "lidar_dense_x3s_f32: a_plane must be > 0 (fp32 input: lidar_dense_x3f_f32)");
    return dense_x3s_launch(h, a_planes, a_plane, lda, rows, k, packed, bias, cout, mode, relu_on, pool_rows, out,
                            o_plane, ldo, stream);
}

// the same GEMM with A as fp32 rows (rows, lda) (split inside the tile loop; elements k..lda-1
// are read and must be finite — weights there are zero)
LIDAR_EXPORT int lidar_dense_x3f_f32(lidar_handle *h, const float *a, int32_t lda, int64_t rows, int32_t k,
                                     const void *packed, const float *bias, int32_t cout, int32_t mode,
                                     int32_t relu_on, int32_t pool_rows, void *out, int64_t o_plane, int64_t ldo,
                                     void *stream)
{
    return dense_x3s_launch(h, a, 0, lda, rows, k, packed, bias, cout, mode, relu_on, pool_rows, out, o_plane, ldo,
                            stream);
}


// fp32 rows -> split planes for lidar_dense_x3s_f32 (hi = bf16(x), lo = bf16(x - hi), both RNE)
LIDAR_EXPORT int lidar_split_x3_f32(lidar_handle *h, const float *x, int64_t rows, int32_t k, int64_t ldx,
                                    void *planes, int64_t plane, int32_t lda, void *stream)
{
    REQUIRE(h && x && planes, "lidar_split_x3_f32: null pointer");
    REQUIRE(rows >= 0 && k > 0 && ldx >= k && lda >= k && lda % 8 == 0 && plane >= rows * lda,
            "lidar_split_x3_f32: bad sizes");
    if (rows == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    const int64_t n = rows * (lda / 8);
    hipLaunchKernelGGL(split_x3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       x, rows, (int)k, ldx, static_cast<__bf16 *>(planes), plane, (int)lda);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
