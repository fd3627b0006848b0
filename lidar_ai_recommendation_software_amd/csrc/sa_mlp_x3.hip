// sa_mlp_x3.hip — SetAbstraction layers 2-3 in fp32 arithmetic carried by the fp16 matrix cores.
//
// h3 arithmetic (h3.hpp): every fp32 operand x is scaled by a power of two and split exactly as
// hi = fp16(x S), lo = fp16(x S - hi), and a product is accumulated as
//   a*b S_a S_w ~ ah*bh + ah*bl + al*bh    (three v_mfma_f32_16x16x32_f16, fp32 accumulation)
// then unscaled once (exact): <= ~3 2^-22 |a*b| per product, fp32-class, so the features meet
// 1e-4 RELATIVE on every element >= 1e-2 RMS (tests/test_gpu_tier_n.py).  Weights are scaled per
// layer at pack time; activations per 16-row tile: layer 2's input by its tile maximum, layer 3's
// by the tile maximum (fused SA1 kernel) or by the bound colsum(W2) 2^e2 + max|b2| (lean SA2
// kernel, which splits layer 2's output chunk by chunk).  fp16 x fp16 products are exact in fp32.
// The fp16 MFMA issues 16x the fp32 one's flops per cycle, so three of them still run ~5x the
// fp32 rate.  X1 (the bf16 spec, BASELINE configs[4]) runs one bf16 product per MFMA instead.
//
// Same fused design as sa_mlp16.hip (16 grouped rows per wave, weights streamed through LDS in
// chunks of two output tiles shared by the 4 waves, layer 3 transposed so the max-pool is a
// register max).  16x16x32 bf16 maps: lane l holds A[row l&15][k = 8(l>>4) + j] and
// B[k = 8(l>>4) + j][col l&15]; D reg r of lane l is row 4(l>>4) + r, column l&15.  An
// accumulator pair (tiles 2s, 2s+1: channels 16t + 4g + r of point l&15, g = l>>4) is the
// k-step-s fragment of the next layer with element j <-> channel in(s, g, j) = 32s + 16(j>>2) +
// 4g + (j&3); the packed weights (lidar_mlp_pack_x3_f32) follow that k order.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "bq_grid.hpp"
#include "h3.hpp"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
using lidar_h3::f16x8;

__device__ __forceinline__ f32x4 mfma_bf(bf16x8 a, bf16x8 b, f32x4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_bf(f16x8 a, f16x8 b, f32x4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_f(float a, float b, f32x4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }
// ReLU on the bits (signed int max with 0): no canonicalising v_max on MFMA results; equal to
// relu() except that a positive NaN stays NaN
__device__ __forceinline__ float relu_i(float v) { return __int_as_float(max(__float_as_int(v), 0)); }
// max of three, NaN-propagating (v_maximum3_f32: no canonicalising v_max per operand, which
// fmaxf's quiet-NaN rule costs on MFMA results)
__device__ __forceinline__ float maxn(float a, float b, float c)
{
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}

// two accumulator tiles -> the hi / lo fragments of one k-step: h3 (fp16, scaled by s) ...
__device__ __forceinline__ void split_pair(const f32x4 &t0, const f32x4 &t1, f16x8 &hi, f16x8 &lo, float s)
{
    lidar_h3::split8(t0, t1, s, hi, lo);
}
// ... or bf16 (X1: only hi is read)
__device__ __forceinline__ void split_pair(const f32x4 &t0, const f32x4 &t1, bf16x8 &hi, bf16x8 &lo, float)
{
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v = j < 4 ? t0[j] : t1[j - 4];
        const __bf16 h = (__bf16)v;
        hi[j] = h;
        lo[j] = (__bf16)(v - (float)h);
    }
}

// packed image (16-byte units "u4"): [W1 fp32 (T1*64 floats, xyz levels only), padded to 16 B]
// [layer-2 chunks] [layer-3 chunks] [b1 b2 b3 fp32] [tail].  Chunk c = output tiles (2c, 2c+1)
// of a layer with K inputs: u4 at ((s*2 + t)*2 + h)*64 + lane = f16x8 (h = 0 hi, 1 lo) of
// W[in(s, lane>>4, j)][16(2c+t) + (lane&15)] 2^s_layer, j = 0..7, s < K/32.  Tail (x3 image, 16
// bytes): int32 s2, s3 (the layers' scaling exponents), float colsum(W2) (max over output
// channels of sum |W2|), float max |b2| — layer 3's input bound in the lean kernel.
// X1 (the bf16 spec, BASELINE configs[4]): one product ah*bh per MFMA on bf16(x) and bf16(w) —
// the image keeps the hi fragments only: u4 at (s*2 + t)*64 + lane.
template <int C1, int C2, int C3, bool X1 = false>
struct PackX3 {
    static constexpr int T1 = C1 / 16, T2 = C2 / 16, T3 = C3 / 16;
    static constexpr int KS2 = C1 / 32, KS3 = C2 / 32;
    static constexpr int HALVES = X1 ? 1 : 2;
    static constexpr int CH2 = KS2 * 2 * HALVES * 64, CH3 = KS3 * 2 * HALVES * 64;  // chunk sizes in u4
    static constexpr int W1U4 = T1 * 64 / 4;                                       // fp32 W1 in u4
};

// the x3 image's tail (after the biases)
struct X3Tail {
    int32_t s2, s3;
    float colsum2, bmax2;
};
// layer 3's input scaling exponent from layer 2's input exponent e2 (the lean kernel's bound:
// |y2| <= colsum(W2) 2^e2 + max|b2|, widened by 2^-10 for the roundings of y2 and of the bound)
__device__ __forceinline__ int bound_exp3(const X3Tail &t, int e2)
{
    const float b = (t.colsum2 * ldexpf(1.0f, e2) + t.bmax2) * (1.0f + 0x1p-10f);
    return lidar_h3::exp_of_bits(__float_as_uint(b));
}

// layer-1 modes: the grouped row's layer-1 output comes from
//   L1_XYZ  W1 (xyz rows, fp32 in LDS) . (p[k] - c) + b1 on a 16x16x4 fp32 MFMA (levels without features)
//   L1_PRE  relu(P[k] - Q[c]) with P = [f, x] W1 + b1 per point, Q = c W1_xyz per centre (fp32 path)
//   L1_PX   relu(P[k] + W1_xyz . bf16(x_k - c)) with P = bf16(f) bf16(W1_f) + b1 per point: the
//           bf16 spec's layer 1 with the feature part (identical in every group of point k) per point
enum { L1_XYZ = 0, L1_PRE = 1, L1_PX = 2 };
__device__ __forceinline__ float bf16r(float v) { return (float)(__bf16)v; }

// max over the four row groups (lanes col, col+16, col+32, col+48) of every column, in all
// four: v_permlane32_swap / v_permlane16_swap hand each lane its xor-32 / xor-16 partner
__device__ __forceinline__ float max_row_groups(float v)
{
    const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = maxn(v, __uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return maxn(v, __uint_as_float(b[0]), __uint_as_float(b[1]));
}

// R = 16-row tiles per wavefront (R grouped-row tiles of the same centre share every weight
// fragment read from LDS: R = 2 halves the LDS and L2 weight bytes per MFMA)
//
// BQ (xyz levels): the kernel answers its centres' ball queries itself from the frame's grid
// (bq_bin_kernel's output, grid_ws): each wave runs lidar_bq::grid_query_wave for its centre
// into LDS before the MLP, so the (B, M, ns) index tensor never goes through HBM and no separate
// full-chip query launch competes with the pipeline; out_idx (optional) receives the indices.
#ifndef LIDAR_BQ_CAP
#define LIDAR_BQ_CAP 512
#endif
// LIDAR_SA_E3_BOUND: layer 3's input exponent in sa_x3_kernel from the bound colsum(W2) 2^e2 + max|b2|
// (1, round 4: no pass over the tile, 95 VGPRs and no scratch; SA1 1.66 -> 1.62 ms alone per 128
// frames) or a wave maximum over the tile (0)
#ifndef LIDAR_SA_E3_BOUND
#define LIDAR_SA_E3_BOUND 1
#endif
// LIDAR_SA1_W: waves per SIMD the fused SA1 kernel (NS = 32, fp32 contract) is built for (A/B builds only)
#ifndef LIDAR_SA1_W
#define LIDAR_SA1_W 5
#endif
constexpr int kBqCap = LIDAR_BQ_CAP;  // candidates per window a fused wave ranks in LDS (more: index-order scan)
template <int C1, int C2, int C3, int NS, int L1, int R, bool X1, bool BQ = false>
__global__ __launch_bounds__(256, (BQ && !X1 && NS == 32) ? LIDAR_SA1_W : (R == 1 ? 3 : 2)) void sa_x3_kernel(const float *__restrict__ P, int64_t stride,
                                                     const float *__restrict__ Q, const int32_t *__restrict__ idx,
                                                     int n, int m, int64_t total, const uint4 *__restrict__ packed,
                                                     float *__restrict__ out, int64_t out_stride, int64_t out_offset,
                                                     const float *__restrict__ X, const float *__restrict__ Cn,
                                                     const char *__restrict__ grid_ws, float r, float r2,
                                                     int32_t *__restrict__ out_idx)
{
    static_assert(!BQ || L1 == L1_XYZ, "fused ball query: xyz levels only");
    static_assert(NS % (16 * R) == 0 && C1 % 32 == 0 && C2 % 32 == 0 && C3 % 64 == 0, "tile shapes");
    constexpr bool XYZ = L1 == L1_XYZ, HASW1 = L1 != L1_PRE;
    using K = PackX3<C1, C2, C3, X1>;
    using PT = std::conditional_t<X1, bf16x8, f16x8>;  // MFMA operand pieces
    constexpr int HV = K::HALVES;
    constexpr int T1 = K::T1, T2 = K::T2, T3 = K::T3, KS2 = K::KS2, KS3 = K::KS3;
    constexpr int CH2 = K::CH2, CH3 = K::CH3, CHMAX = CH2 > CH3 ? CH2 : CH3;
    constexpr int NCH = T2 / 2 + T3 / 2;
    constexpr int ITERS = NS / (16 * R);
    constexpr int PER = (CHMAX + 255) / 256;

    // SPLIT (the fused SA1 kernel): two LDS variables (distinct alias scopes), so a pass's reads of
    // one buffer need not wait for the weight chunk streaming into the other — with one array the
    // compiler waited for the chunk it had just issued before the pass's first read.  The other
    // instantiations keep one array: there the freed schedule hoists reads and costs registers.
    constexpr bool SPLIT = BQ;
    __shared__ uint4 bufa[SPLIT ? 1 : 2][CHMAX];
    __shared__ uint4 bufb[SPLIT ? CHMAX : 1];
    auto bufp = [&](int p) -> uint4 * {
        if constexpr (SPLIT)
            return p ? bufb : bufa[0];
        else
            return bufa[p];
    };
    __shared__ float bias_s[C1 + C2 + C3];
    __shared__ float w1_s[HASW1 ? T1 * 64 : 1];

    // wave index in an SGPR: the LDS-DMA destinations (M0) and the unit below are wave-uniform
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int q = lane >> 4, col = lane & 15;
    const int64_t unit = lidar::xcd_block() * 4 + wave;
    const bool live = unit < total;  // every wave takes part in the barriers
    const int64_t cc = live ? unit : total - 1;
    const int64_t b = cc / m;

    const uint4 *W2 = packed + (HASW1 ? K::W1U4 : 0);
    const uint4 *W3 = W2 + (int64_t)(T2 / 2) * CH2;
    const float *Bias = reinterpret_cast<const float *>(W3 + (int64_t)(T3 / 2) * CH3);
    // h3: the layers' weight scaling exponents (X1: no scaling)
    int sw2 = 0, sw3 = 0;
    if constexpr (!X1) {
        const X3Tail *tl = reinterpret_cast<const X3Tail *>(Bias + C1 + C2 + C3);
        sw2 = tl->s2;
        sw3 = tl->s3;
    }

    auto fetch = [&](int c, int dst) {
        const uint4 *src = c < T2 / 2 ? W2 + c * CH2 : W3 + (c - T2 / 2) * CH3;
        asm volatile("" : "+s"(src));  // keep each chunk's loads in their own iteration
        const int len = c < T2 / 2 ? CH2 : CH3;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int base = 256 * i + 64 * wave;  // scalar: SGPR base + 32-bit lane offset
            if ((SPLIT && CH2 == CH3 && CH2 % 256 == 0) || base < len)  // equal whole chunks: unconditional
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(src + base + (unsigned)lane),
                                                 (__attribute__((address_space(3))) void *)(&bufp(dst)[base]), 16, 0,
                                                 0);
        }
        if constexpr (SPLIT) __builtin_amdgcn_sched_barrier(0);  // issued before the pass's reads and MFMAs
    };
    fetch(0, 0);
    for (int i = tid; i < C1 + C2 + C3; i += 256) bias_s[i] = Bias[i];
    if constexpr (HASW1)
        for (int i = tid; i < T1 * 64; i += 256) w1_s[i] = reinterpret_cast<const float *>(packed)[i];
    // layer 3's running max-pool of the raw accumulators in registers: mx[j] of row group q
    // holds channel 16 (4j + q) + col (register max, no LDS table: an LDS store here would make
    // the compiler wait for the weight prefetches in flight)
    float mx[T3 / 4];
#pragma unroll
    for (int j = 0; j < T3 / 4; ++j) mx[j] = -INFINITY;
    // windows hold ~NS expected hits, so their candidates (27 cells of side >= r) scale with NS:
    // about 220 at NS = 32 (SSG SA1), about 900 at NS = 128 (MSG's r = 0.4 branch), which past
    // the cap would fall back to an index-order scan of the whole window
    constexpr int QCAP = NS >= 128 ? 2 * kBqCap : kBqCap;
    __shared__ int qidx[BQ ? 4 : 1][BQ ? NS : 1];           // this wave's ball-query result
    __shared__ __attribute__((aligned(8))) int qhits[BQ ? 4 : 1][BQ ? QCAP + 4 : 1];  // its per-window hits / bitmap
    if constexpr (BQ) {
        const float *pf = P + (int64_t)b * n * 3;
        const char *fw = grid_ws + b * lidar_bq::grid_frame_bytes(n);
        lidar_bq::grid_query_wave<QCAP, int, (NS >= 64)>(pf, fw, n, Q[cc * 3], Q[cc * 3 + 1], Q[cc * 3 + 2], r, r2, NS, lane,
                                        qhits[wave], &qidx[wave][0]);
    }
    __syncthreads();
    if constexpr (BQ)
        if (live && out_idx != nullptr)
            for (int i = lane; i < NS; i += 64) out_idx[unit * NS + i] = qidx[wave][i];
    int par = 0;
    // layer 3's max-pool runs on the raw accumulators: x -> relu(x + bias) is monotone in
    // fp32 (round-to-nearest addition never reverses an order), so max_i relu(a_i + b) ==
    // relu(max_i a_i + b) bit for bit — the bias and ReLU are applied once per output
    // channel at the end.

#pragma unroll 1
    for (int it = 0; it < ITERS; ++it) {
        // ---- layer 1 -> the layer-2 operand fragments (hi / lo) of R x 16 grouped rows
        PT xh[R][KS2], xl[R][KS2];
        int e2[R], e3[R];  // h3: the tiles' scaling exponents of layers 2 and 3 (wave-uniform)
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
            const int64_t k = BQ ? qidx[wave][(it * R + rr) * 16 + col] : idx[cc * NS + (it * R + rr) * 16 + col];
            f32x4 y1[T1];
            if constexpr (XYZ) {
                const float *pr = P + ((int64_t)b * n + k) * 3;
                const float *ce = Q + cc * 3;
                float x = q < 3 ? pr[q] - ce[q] : 0.0f;  // lane group q: dx, dy, dz, 0
                if constexpr (X1) x = bf16r(x);  // the bf16 spec rounds the offsets (W1 is pre-rounded)
#pragma unroll
                for (int t = 0; t < T1; ++t) {
                    // the bias is the accumulator's initial value (channel 16t + 4q + r)
                    f32x4 acc = *reinterpret_cast<const f32x4 *>(&bias_s[16 * t + 4 * q]);
                    acc = mfma_f(w1_s[t * 64 + lane], x, acc);
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[r] = relu_i(acc[r]);
                    y1[t] = acc;
                }
            } else if constexpr (L1 == L1_PX) {
                const float *pr = X + ((int64_t)b * n + k) * 3;
                const float *ce = Cn + cc * 3;
                const float x = bf16r(q < 3 ? pr[q] - ce[q] : 0.0f);
                const f32x4 *pp = reinterpret_cast<const f32x4 *>(P + ((int64_t)b * n + k) * stride + 4 * q);
#pragma unroll
                for (int t = 0; t < T1; ++t) {
                    f32x4 acc = mfma_f(w1_s[t * 64 + lane], x, pp[4 * t]);
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[r] = relu_i(acc[r]);
                    y1[t] = acc;
                }
            } else {
                // relu(P[k] - Q[c]); the centre row is re-read per tile (an L1 hit) rather than
                // held in registers across the tiles
                int zero = 0;
                asm volatile("" : "+v"(zero));
                const f32x4 *pp = reinterpret_cast<const f32x4 *>(P + ((int64_t)b * n + k) * stride + 4 * q);
                const f32x4 *qq = reinterpret_cast<const f32x4 *>(Q + cc * stride + 4 * q + zero);
#pragma unroll
                for (int ti = 0; ti < T1; ++ti) {
                    const f32x4 a = pp[4 * ti], c = qq[4 * ti];
#pragma unroll
                    for (int r = 0; r < 4; ++r) y1[ti][r] = relu(a[r] - c[r]);
                }
            }
            float sc = 1.0f;
            if constexpr (!X1) {
                uint32_t mb = 0;
#pragma unroll
                for (int t = 0; t < T1; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) mb = max(mb, __float_as_uint(y1[t][r]));  // ReLU outputs: non-negative bits
                e2[rr] = lidar_h3::wave_exp(mb);
                sc = lidar_h3::scale_of(e2[rr]);
            }
#pragma unroll
            for (int s = 0; s < KS2; ++s) split_pair(y1[2 * s], y1[2 * s + 1], xh[rr][s], xl[rr][s], sc);
        }

        f32x4 y2[R][T2];
        PT zh[R][KS3], zl[R][KS3];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int cn = c + 1 < NCH ? c + 1 : 0;
            const bool more = c + 1 < NCH || it + 1 < ITERS;
            if (more) fetch(cn, par ^ 1);  // lands during this chunk's MFMAs
            const uint4 *wb = bufp(par) + lane;
            f32x4 a0[R], a1[R];
            // layer 2's bias (channel rows: 16t + 4q + r): the accumulators' initial value in X1, added
            // after the unscaling in h3
            const f32x4 b0 = c < T2 / 2 ? *reinterpret_cast<const f32x4 *>(&bias_s[C1 + 16 * (2 * c) + 4 * q]) : f32x4{};
            const f32x4 b1 = c < T2 / 2 ? *reinterpret_cast<const f32x4 *>(&bias_s[C1 + 16 * (2 * c + 1) + 4 * q]) : f32x4{};
            if (X1 && c < T2 / 2) {
#pragma unroll
                for (int rr = 0; rr < R; ++rr) {
                    a0[rr] = b0;
                    a1[rr] = b1;
                }
            } else {
#pragma unroll
                for (int rr = 0; rr < R; ++rr) a0[rr] = a1[rr] = f32x4{};
            }
            if (c < T2 / 2) {  // layer 2: output tiles 2c, 2c+1 (channel rows x point columns)
#pragma unroll
                for (int s = 0; s < KS2; ++s) {
                    const PT h0 = __builtin_bit_cast(PT, wb[((s * 2 + 0) * HV + 0) * 64]);
                    const PT h1 = __builtin_bit_cast(PT, wb[((s * 2 + 1) * HV + 0) * 64]);
                    if constexpr (X1) {
#pragma unroll
                        for (int rr = 0; rr < R; ++rr) {
                            a0[rr] = mfma_bf(h0, xh[rr][s], a0[rr]);
                            a1[rr] = mfma_bf(h1, xh[rr][s], a1[rr]);
                        }
                    } else {
                        const PT l0 = __builtin_bit_cast(PT, wb[((s * 2 + 0) * HV + 1) * 64]);
                        const PT l1 = __builtin_bit_cast(PT, wb[((s * 2 + 1) * HV + 1) * 64]);
#pragma unroll
                        for (int rr = 0; rr < R; ++rr) {
                            a0[rr] = mfma_bf(h0, xh[rr][s], a0[rr]);
                            a1[rr] = mfma_bf(h1, xh[rr][s], a1[rr]);
                            a0[rr] = mfma_bf(h0, xl[rr][s], a0[rr]);
                            a1[rr] = mfma_bf(h1, xl[rr][s], a1[rr]);
                            a0[rr] = mfma_bf(l0, xh[rr][s], a0[rr]);
                            a1[rr] = mfma_bf(l1, xh[rr][s], a1[rr]);
                        }
                    }
                }
#pragma unroll
                for (int rr = 0; rr < R; ++rr) {
                    // unscale by 2^-(s_a + s_w) and add the bias: one fma by an exact power of two
                    const float us = X1 ? 1.0f : ldexpf(1.0f, e2[rr] - 14 - sw2);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if constexpr (!X1) {
                            a0[rr][r] = fmaf(a0[rr][r], us, b0[r]);
                            a1[rr][r] = fmaf(a1[rr][r], us, b1[r]);
                        }
                        a0[rr][r] = relu_i(a0[rr][r]);
                        a1[rr][r] = relu_i(a1[rr][r]);
                    }
                    y2[rr][2 * c < T2 ? 2 * c : 0] = a0[rr];
                    y2[rr][2 * c + 1 < T2 ? 2 * c + 1 : 0] = a1[rr];
                }
                if (c == T2 / 2 - 1) {  // layer 2 complete: its output as layer-3 fragments
#pragma unroll
                    for (int rr = 0; rr < R; ++rr) {
                        float sc = 1.0f;
                        if constexpr (!X1) {
#if LIDAR_SA_E3_BOUND
                            // scaled by the bound colsum(W2) 2^e2 + max|b2| (the lean kernel's rule): no
                            // pass over the tile
                            e3[rr] = bound_exp3(*reinterpret_cast<const X3Tail *>(Bias + C1 + C2 + C3), e2[rr]);
#else
                            uint32_t mb = 0;  // scaled by the tile's maximum
#pragma unroll
                            for (int t = 0; t < T2; ++t)
#pragma unroll
                                for (int r = 0; r < 4; ++r) mb = max(mb, __float_as_uint(y2[rr][t][r]));  // ReLU outputs: non-negative bits
                            e3[rr] = lidar_h3::wave_exp(mb);
#endif
                            sc = lidar_h3::scale_of(e3[rr]);
                        }
#pragma unroll
                        for (int s = 0; s < KS3; ++s)
                            split_pair(y2[rr][2 * s], y2[rr][2 * s + 1], zh[rr][s], zl[rr][s], sc);
                    }
                }
            } else {  // layer 3: output tiles 2tp, 2tp+1, transposed (point rows), + max-pool
                const int tp = c - T2 / 2;
#pragma unroll
                for (int s = 0; s < KS3; ++s) {
                    const PT h0 = __builtin_bit_cast(PT, wb[((s * 2 + 0) * HV + 0) * 64]);
                    const PT h1 = __builtin_bit_cast(PT, wb[((s * 2 + 1) * HV + 0) * 64]);
                    if constexpr (X1) {
#pragma unroll
                        for (int rr = 0; rr < R; ++rr) {
                            a0[rr] = mfma_bf(zh[rr][s], h0, a0[rr]);
                            a1[rr] = mfma_bf(zh[rr][s], h1, a1[rr]);
                        }
                    } else {
                        const PT l0 = __builtin_bit_cast(PT, wb[((s * 2 + 0) * HV + 1) * 64]);
                        const PT l1 = __builtin_bit_cast(PT, wb[((s * 2 + 1) * HV + 1) * 64]);
#pragma unroll
                        for (int rr = 0; rr < R; ++rr) {
                            a0[rr] = mfma_bf(zh[rr][s], h0, a0[rr]);
                            a1[rr] = mfma_bf(zh[rr][s], h1, a1[rr]);
                            a0[rr] = mfma_bf(zh[rr][s], l0, a0[rr]);
                            a1[rr] = mfma_bf(zh[rr][s], l1, a1[rr]);
                            a0[rr] = mfma_bf(zl[rr][s], h0, a0[rr]);
                            a1[rr] = mfma_bf(zl[rr][s], h1, a1[rr]);
                        }
                    }
                }
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const int t = 2 * tp + hh < T3 ? 2 * tp + hh : 0;
                    float v = -INFINITY;
#pragma unroll
                    for (int rr = 0; rr < R; ++rr) {
                        const f32x4 &acc = hh ? a1[rr] : a0[rr];
                        float m4 = maxn(acc[0], acc[1], __builtin_elementwise_maximum(acc[2], acc[3]));
                        // a tile's rows share its scale (2^k x is monotone and exact): its max is
                        // unscaled, before the max over the tiles, whose scales differ
                        if constexpr (!X1) m4 = ldexpf(m4, e3[rr] - 14 - sw3);
                        v = __builtin_elementwise_maximum(v, m4);
                    }
                    v = max_row_groups(v);
                    if (q == (t & 3)) mx[t >> 2] = __builtin_elementwise_maximum(mx[t >> 2], v);
                }
            }
            __syncthreads();  // (vmcnt(0)) chunk c+1 landed for everyone; buf[par] free for c+2
            par ^= 1;
        }
    }
    if (live) {
        float *o = out + unit * out_stride + out_offset;
#pragma unroll
        for (int j = 0; j < T3 / 4; ++j) {
            const int c3 = 16 * (4 * j + q) + col;
            o[c3] = relu(mx[j] + bias_s[C1 + C2 + c3]);
        }
    }
}

// The wide feature levels (SA2): the arithmetic of sa_x3_kernel<.., L1_PRE, R = 2, false> in
// <= 128 VGPRs and 34 KiB of LDS, so that a CU holds three of its workgroups beside a resident
// 512-thread FPS workgroup (two for that form, 160 VGPRs / 50 KiB, which this kernel replaced:
// the two were tested bit-identical in round 2, and only this one ships).  Layer 2 runs one 16-row tile at a time (only that tile's layer-2 operand is live; its
// weight chunks stream through LDS once per tile), layer 3 keeps R = 2 (both tiles share every
// weight fragment), and the max-pool is a register max: per chunk, each lane's max over its rows
// is reduced over the four row groups by two lane swaps and folded into mx[t / 4] of row group
// t % 4 — no LDS table.
//
// PFX: the centre's NS point indices come in one coalesced load at the start (lane l holds rows
// l, 64 + l, ...), and a tile's 16 row indices by ds_bpermute from those registers, so a tile's
// gather of P rows waits on one memory round trip instead of two dependent ones (idx, then P).
//
// LIDAR_SA_ABL (diagnostic builds only, tools/micro/sa2_ablate.py; 0 in the product): bit 1 streams
// layer 2's first chunk for every pass (same instructions, one L2-hot 16 KiB source), bit 2 the per-pass barriers, bit 4 the row gather
// (every tile reads rows 0..15 of its frame) — wrong results, for pricing each part of a pass
#ifndef LIDAR_SA_ABL
#define LIDAR_SA_ABL 0
#endif
// LIDAR_LEAN_R / LIDAR_LEAN_W: A/B builds only (tiles per layer-3 weight fragment; launch-bound waves)
#ifndef LIDAR_LEAN_R
#define LIDAR_LEAN_R 2
#endif
#ifndef LIDAR_LEAN_W
#define LIDAR_LEAN_W 4
#endif
template <int C1, int C2, int C3, int NS, bool PFX>
__global__ __launch_bounds__(256, LIDAR_LEAN_W) void sa_x3_lean_kernel(const float *__restrict__ P, int64_t stride,
                                                            const float *__restrict__ Q,
                                                            const int32_t *__restrict__ idx, int n, int m,
                                                            int64_t total, const uint4 *__restrict__ packed,
                                                            float *__restrict__ out, int64_t out_stride,
                                                            int64_t out_offset)
{
    constexpr int R = LIDAR_LEAN_R;
    static_assert(NS % (16 * R) == 0 && C1 % 32 == 0 && C2 % 32 == 0 && C3 % 64 == 0, "tile shapes");
    using K = PackX3<C1, C2, C3, false>;
    constexpr int T2 = K::T2, T3 = K::T3, KS2 = K::KS2, KS3 = K::KS3;
    constexpr int CH2 = K::CH2, CH3 = K::CH3, CHMAX = CH2 > CH3 ? CH2 : CH3;
    constexpr int NL2 = T2 / 2, NL3 = T3 / 2, NSEQ = R * NL2 + NL3;  // chunk passes per iteration
    constexpr int ITERS = NS / (16 * R);
    constexpr int PER = (CHMAX + 255) / 256;
    static_assert(!PFX || NS % 64 == 0, "PFX: whole 64-row blocks of indices");

    __shared__ uint4 buf0[CHMAX], buf1[CHMAX];  // two variables, as in sa_x3_kernel
    auto bufp = [&](int p) -> uint4 * { return p ? buf1 : buf0; };
    __shared__ float bias_s[C2 + C3];

    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int q = lane >> 4, col = lane & 15;
    const int64_t unit = lidar::xcd_block() * 4 + wave;
    const bool live = unit < total;
    const int64_t cc = live ? unit : total - 1;
    const int64_t b = cc / m;

    const uint4 *W2 = packed;
    const uint4 *W3 = W2 + (int64_t)NL2 * CH2;
    const float *Bias = reinterpret_cast<const float *>(W3 + (int64_t)NL3 * CH3);
    const X3Tail tl = *reinterpret_cast<const X3Tail *>(Bias + C1 + C2 + C3);

    // pass `seq` of an iteration: layer-2 chunk seq % NL2 for tile seq / NL2, then the layer-3 chunks
    auto fetch = [&](int seq, int dst) {
        const int c = (LIDAR_SA_ABL & 1) != 0 ? 0 : seq < R * NL2 ? seq % NL2 : seq - R * NL2 + NL2;
        const uint4 *src = c < NL2 ? W2 + c * CH2 : W3 + (c - NL2) * CH3;
        asm volatile("" : "+s"(src));
        const int len = c < NL2 ? CH2 : CH3;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int base = 256 * i + 64 * wave;
            if ((CH2 == CH3 && CH2 % 256 == 0) || base < len)  // equal whole chunks: unconditional, so the waits can count them
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(src + base + (unsigned)lane),
                                                 (__attribute__((address_space(3))) void *)(&bufp(dst)[base]), 16, 0,
                                                 0);
        }
        __builtin_amdgcn_sched_barrier(0);  // issued before the pass's reads and MFMAs, not sunk to its end
    };
    int32_t kall[PFX ? NS / 64 : 1];
    if constexpr (PFX) {
#pragma unroll
        for (int j = 0; j < NS / 64; ++j) kall[j] = idx[cc * NS + 64 * j + lane];
    }
    fetch(0, 0);
    for (int i = tid; i < C2 + C3; i += 256) bias_s[i] = Bias[C1 + i];
    __syncthreads();
    float mx[T3 / 4];
#pragma unroll
    for (int j = 0; j < T3 / 4; ++j) mx[j] = -INFINITY;
    int par = 0;

#pragma unroll 1
    for (int it = 0; it < ITERS; ++it) {
        f16x8 zh[R][KS3], zl[R][KS3];
        int e3[R];  // the tiles' layer-3 input exponents (wave-uniform)
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
            // layer 1 of this tile's 16 rows: relu(P[k] - Q[c]) as the layer-2 hi / lo fragments,
            // scaled by the tile's maximum
            f16x8 xh[KS2], xl[KS2];
            int e2;
            {
                int zero = 0;
                asm volatile("" : "+v"(zero));
                const int t16 = (it * R + rr) * 16;  // the tile's first row
                int64_t k;
                if constexpr ((LIDAR_SA_ABL & 4) != 0)
                    k = col;
                else if constexpr (PFX)
                    k = __shfl(kall[t16 >> 6], (t16 & 63) + col, 64);
                else
                    k = idx[cc * NS + t16 + col];
                const f32x4 *pp = reinterpret_cast<const f32x4 *>(P + ((int64_t)b * n + k) * stride + 4 * q);
                const f32x4 *qq = reinterpret_cast<const f32x4 *>(Q + cc * stride + 4 * q + zero);
                f32x4 y[KS2][2];
                uint32_t mb = 0;
#pragma unroll
                for (int s = 0; s < KS2; ++s)
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const f32x4 a = pp[4 * (2 * s + h)], c = qq[4 * (2 * s + h)];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            y[s][h][r] = relu(a[r] - c[r]);
                            mb = max(mb, __float_as_uint(y[s][h][r]));  // ReLU outputs: non-negative bits
                        }
                    }
                e2 = lidar_h3::wave_exp(mb);
                const float sc = lidar_h3::scale_of(e2);
#pragma unroll
                for (int s = 0; s < KS2; ++s) split_pair(y[s][0], y[s][1], xh[s], xl[s], sc);
            }
            // layer 2's output is split chunk by chunk (layer-3 k-step c): its scale comes from the
            // bound colsum(W2) 2^e2 + max|b2|, known before any chunk
            e3[rr] = bound_exp3(tl, e2);
            const float sc3 = lidar_h3::scale_of(e3[rr]);
#pragma unroll
            for (int c = 0; c < NL2; ++c) {
                fetch(rr * NL2 + c + 1, par ^ 1);  // a layer-3 pass always follows: lands during these MFMAs
                const uint4 *wb = bufp(par) + lane;
                f32x4 a0 = f32x4{}, a1 = f32x4{};
#pragma unroll
                for (int s = 0; s < KS2; ++s) {
                    const f16x8 h0 = __builtin_bit_cast(f16x8, wb[((s * 2 + 0) * 2 + 0) * 64]);
                    const f16x8 l0 = __builtin_bit_cast(f16x8, wb[((s * 2 + 0) * 2 + 1) * 64]);
                    a0 = mfma_bf(h0, xh[s], a0);
                    a0 = mfma_bf(h0, xl[s], a0);
                    a0 = mfma_bf(l0, xh[s], a0);
                    const f16x8 h1 = __builtin_bit_cast(f16x8, wb[((s * 2 + 1) * 2 + 0) * 64]);
                    const f16x8 l1 = __builtin_bit_cast(f16x8, wb[((s * 2 + 1) * 2 + 1) * 64]);
                    a1 = mfma_bf(h1, xh[s], a1);
                    a1 = mfma_bf(h1, xl[s], a1);
                    a1 = mfma_bf(l1, xh[s], a1);
                }
                const f32x4 b0 = *reinterpret_cast<const f32x4 *>(&bias_s[16 * (2 * c) + 4 * q]);
                const f32x4 b1 = *reinterpret_cast<const f32x4 *>(&bias_s[16 * (2 * c + 1) + 4 * q]);
                const float us = ldexpf(1.0f, e2 - 14 - tl.s2);  // 2^-(s_a + s_w): one exact fma with the bias
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    a0[r] = relu_i(fmaf(a0[r], us, b0[r]));
                    a1[r] = relu_i(fmaf(a1[r], us, b1[r]));
                }
                split_pair(a0, a1, zh[rr][c], zl[rr][c], sc3);  // layer-2 chunk c = layer-3 k-step c
                if constexpr ((LIDAR_SA_ABL & 2) == 0) __syncthreads();
                par ^= 1;
            }
        }
#pragma unroll
        for (int c = 0; c < NL3; ++c) {
            if (c + 1 < NL3 || it + 1 < ITERS) fetch(c + 1 < NL3 ? R * NL2 + c + 1 : 0, par ^ 1);
            const uint4 *wb = bufp(par) + lane;
            f32x4 a0[R], a1[R];
#pragma unroll
            for (int rr = 0; rr < R; ++rr) a0[rr] = a1[rr] = f32x4{};
#pragma unroll
            for (int s = 0; s < KS3; ++s) {
                const f16x8 h0 = __builtin_bit_cast(f16x8, wb[((s * 2 + 0) * 2 + 0) * 64]);
                const f16x8 h1 = __builtin_bit_cast(f16x8, wb[((s * 2 + 1) * 2 + 0) * 64]);
                const f16x8 l0 = __builtin_bit_cast(f16x8, wb[((s * 2 + 0) * 2 + 1) * 64]);
                const f16x8 l1 = __builtin_bit_cast(f16x8, wb[((s * 2 + 1) * 2 + 1) * 64]);
#pragma unroll
                for (int rr = 0; rr < R; ++rr) {
                    a0[rr] = mfma_bf(zh[rr][s], h0, a0[rr]);
                    a1[rr] = mfma_bf(zh[rr][s], h1, a1[rr]);
                    a0[rr] = mfma_bf(zh[rr][s], l0, a0[rr]);
                    a1[rr] = mfma_bf(zh[rr][s], l1, a1[rr]);
                    a0[rr] = mfma_bf(zl[rr][s], h0, a0[rr]);
                    a1[rr] = mfma_bf(zl[rr][s], h1, a1[rr]);
                }
            }
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int t = 2 * c + hh;
                float v = -INFINITY;
#pragma unroll
                for (int rr = 0; rr < R; ++rr) {
                    const f32x4 &acc = hh ? a1[rr] : a0[rr];
                    // the tile's max, unscaled (its rows share the scale) before the max over tiles
                    const float m4 = maxn(acc[0], acc[1], __builtin_elementwise_maximum(acc[2], acc[3]));
                    v = __builtin_elementwise_maximum(v, ldexpf(m4, e3[rr] - 14 - tl.s3));
                }
                v = max_row_groups(v);
                if (q == (t & 3)) mx[t >> 2] = __builtin_elementwise_maximum(mx[t >> 2], v);
            }
            if constexpr ((LIDAR_SA_ABL & 2) == 0) __syncthreads();
            par ^= 1;
        }
    }
    static_assert(NSEQ == R * NL2 + NL3, "pass count");
    if (live) {
        float *o = out + unit * out_stride + out_offset;
#pragma unroll
        for (int j = 0; j < T3 / 4; ++j) {
            const int c3 = 16 * (4 * j + q) + col;
            o[c3] = relu(mx[j] + bias_s[C2 + c3]);
        }
    }
}

// LIDAR_X3_ROWS: 16-row tiles per wavefront (A/B builds; 2 unless NS = 16); LIDAR_X1_ROWS the same for
// the bf16 spec's kernels (X1: half the registers per tile)
#ifndef LIDAR_X3_ROWS
#define LIDAR_X3_ROWS 2
#endif
#ifndef LIDAR_X1_ROWS
#define LIDAR_X1_ROWS 2
#endif
template <int NS, bool X1>
constexpr int rows_for()
{
    return X1 && NS >= 16 * LIDAR_X1_ROWS ? LIDAR_X1_ROWS : (NS >= 16 * LIDAR_X3_ROWS ? LIDAR_X3_ROWS : 1);
}

template <int C1, int C2, int C3, int NS>
int launch_x3_lean(const float *p, int64_t stride, const float *q, const int32_t *idx, int64_t batch, int64_t n,
                   int64_t m, const void *packed, float *out, int64_t os, int64_t oo, hipStream_t s)
{
    const int64_t total = batch * m;
    const int64_t blocks = (total + 3) / 4;
    REQUIRE(blocks <= 0x7fffffff, "sa_group_mlp_x3: too many centres");
    // a centre's row indices in one coalesced load whenever NS is a multiple of the wavefront
    hipLaunchKernelGGL((sa_x3_lean_kernel<C1, C2, C3, NS, NS % 64 == 0>), dim3((unsigned)blocks), dim3(256), 0, s, p,
                       stride, q, idx, (int)n, (int)m, total, static_cast<const uint4 *>(packed), out, os, oo);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

template <int C1, int C2, int C3, int NS, int L1, bool X1 = false>
int launch_x3(const float *p, int64_t stride, const float *q, const int32_t *idx, int64_t batch, int64_t n,
              int64_t m, const void *packed, float *out, int64_t os, int64_t oo, hipStream_t s,
              const float *xyz = nullptr, const float *centres = nullptr)
{
    constexpr int R = rows_for<NS, X1>();
    const int64_t total = batch * m;
    const int64_t blocks = (total + 3) / 4;
    REQUIRE(blocks <= 0x7fffffff, "sa_group_mlp_x3: too many centres");
    hipLaunchKernelGGL((sa_x3_kernel<C1, C2, C3, NS, L1, R, X1>), dim3((unsigned)blocks), dim3(256), 0, s, p, stride,
                       q, idx, (int)n, (int)m, total, static_cast<const uint4 *>(packed), out, os, oo, xyz, centres,
                       nullptr, 0.0f, 0.0f, nullptr);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

template <int C1, int C2, int C3, int NS, bool X1>
int launch_x3_bq(const float *xyz, const char *grid, const float *centres, int64_t batch, int64_t n, int64_t m,
                 float radius, const void *packed, float *out, int64_t os, int64_t oo, int32_t *out_idx,
                 hipStream_t s)
{
    constexpr int R = rows_for<NS, X1>();
    const int64_t total = batch * m;
    const int64_t blocks = (total + 3) / 4;
    REQUIRE(blocks <= 0x7fffffff, "sa_group_mlp_bq: too many centres");
    hipLaunchKernelGGL((sa_x3_kernel<C1, C2, C3, NS, L1_XYZ, R, X1, true>), dim3((unsigned)blocks), dim3(256), 0, s,
                       xyz, (int64_t)3, centres, nullptr, (int)n, (int)m, total, static_cast<const uint4 *>(packed),
                       out, os, oo, nullptr, nullptr, grid, radius, radius * radius, out_idx);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

__host__ uint16_t bf16_rne(float f)
{
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
__host__ float bf16_to_f(uint16_t h)
{
    const uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
// fp16 (RNE) bits of a float, and back (the host side of h3.hpp's split)
__host__ uint16_t f16_bits(float f)
{
    const _Float16 h = (_Float16)f;
    uint16_t u;
    memcpy(&u, &h, 2);
    return u;
}
__host__ float f16_to_f(uint16_t u)
{
    _Float16 h;
    memcpy(&h, &u, 2);
    return (float)h;
}
// a layer's scaling exponent s (max |W| 2^s < 2^14)
__host__ int32_t layer_exp(const float *w, int64_t n)
{
    uint32_t m = 0;
    for (int64_t i = 0; i < n; ++i) {
        uint32_t u;
        memcpy(&u, &w[i], 4);
        m = std::max(m, u & 0x7fffffffu);
    }
    return 14 - lidar_h3::exp_of_bits(m);
}

}  // namespace

// bytes of the x3 packed image
LIDAR_EXPORT int64_t lidar_mlp_packed_size_x3(int32_t xyz_level, int32_t c1, int32_t c2, int32_t c3)
{
    const int64_t w1 = xyz_level ? (int64_t)(c1 / 16) * 64 * 4 : 0;
    return w1 + ((int64_t)(c2 / 32) * (c1 / 32) + (int64_t)(c3 / 32) * (c2 / 32)) * 4 * 64 * 16 +
           (int64_t)(c1 + c2 + c3) * 4 + (int64_t)sizeof(X3Tail);
}

// host packer: w1 (3 + ..., c1) read only for an xyz level (its xyz rows, fp32 as the 16-row
// kernel's layer 1); w2 (c1, c2), w3 (c2, c3) scaled by their layer's power of two and split into
// fp16 hi / lo in the fragment order (h3.hpp); the tail holds the exponents and layer 3's bound
LIDAR_EXPORT int lidar_mlp_pack_x3_f32(int32_t xyz_level, int32_t c1, int32_t c2, int32_t c3, const float *w1,
                                       const float *b1, const float *w2, const float *b2, const float *w3,
                                       const float *b3, void *packed)
{
    REQUIRE(b1 && w2 && b2 && w3 && b3 && packed && (!xyz_level || w1), "lidar_mlp_pack_x3_f32: null pointer");
    REQUIRE(c1 % 32 == 0 && c2 % 32 == 0 && c3 % 32 == 0 && c1 > 0 && c2 > 0 && c3 > 0,
            "lidar_mlp_pack_x3_f32: widths must be positive multiples of 32");
    char *o = static_cast<char *>(packed);
    if (xyz_level) {
        float *f = reinterpret_cast<float *>(o);
        for (int t = 0; t < c1 / 16; ++t)
            for (int l = 0; l < 64; ++l) {
                const int qq = l >> 4;
                *f++ = qq < 3 ? w1[(int64_t)qq * c1 + 16 * t + (l & 15)] : 0.0f;
            }
        o = reinterpret_cast<char *>(f);
    }
    X3Tail tail;
    tail.s2 = layer_exp(w2, (int64_t)c1 * c2);
    tail.s3 = layer_exp(w3, (int64_t)c2 * c3);
    auto layer = [&](const float *w, int cin, int cout, int32_t sexp) {
        const float sc = std::ldexp(1.0f, sexp);
        uint16_t *u = reinterpret_cast<uint16_t *>(o);
        for (int c = 0; c < cout / 32; ++c)
            for (int s = 0; s < cin / 32; ++s)
                for (int t = 0; t < 2; ++t)
                    for (int h = 0; h < 2; ++h)
                        for (int l = 0; l < 64; ++l)
                            for (int j = 0; j < 8; ++j) {
                                const int in = 32 * s + 16 * (j >> 2) + 4 * (l >> 4) + (j & 3);
                                const float v = w[(int64_t)in * cout + 16 * (2 * c + t) + (l & 15)] * sc;
                                const uint16_t hi = f16_bits(v);
                                *u++ = h == 0 ? hi : f16_bits(v - f16_to_f(hi));
                            }
        o = reinterpret_cast<char *>(u);
    };
    layer(w2, c1, c2, tail.s2);
    layer(w3, c2, c3, tail.s3);
    float *f = reinterpret_cast<float *>(o);
    for (int i = 0; i < c1; ++i) *f++ = b1[i];
    for (int i = 0; i < c2; ++i) *f++ = b2[i];
    for (int i = 0; i < c3; ++i) *f++ = b3[i];
    // layer 3's input bound (lean kernel): max over channels of sum_k |W2[k][c]|, and max |b2|,
    // rounded up (float64 sums, then the next float up)
    double cs = 0.0, bm = 0.0;
    for (int c = 0; c < c2; ++c) {
        double a = 0.0;
        for (int k = 0; k < c1; ++k) a += std::fabs((double)w2[(int64_t)k * c2 + c]);
        cs = std::max(cs, a);
        bm = std::max(bm, std::fabs((double)b2[c]));
    }
    tail.colsum2 = std::nextafter((float)cs, INFINITY);
    tail.bmax2 = std::nextafter((float)bm, INFINITY);
    memcpy(f, &tail, sizeof tail);
    return LIDAR_OK;
}

// the x3 fused kernels; arguments as lidar_sa_group_mlp16_f32 (xyz_level: p = xyz, q = centres;
// else p / q = the per-point / per-centre layer-1 rows), packed = lidar_mlp_pack_x3_f32's image
LIDAR_EXPORT int lidar_sa_group_mlp_x3_f32(lidar_handle *h, int32_t xyz_level, const float *p, int64_t p_stride,
                                           const float *q, const int32_t *idx, int64_t batch, int64_t n, int64_t m,
                                           int32_t nsample, int32_t c1, int32_t c2, int32_t c3, const void *packed,
                                           float *out, int64_t out_stride, int64_t out_offset, void *stream)
{
    REQUIRE(h && p && q && idx && packed && out, "lidar_sa_group_mlp_x3_f32: null pointer");
    REQUIRE(batch >= 0 && n >= 1 && m >= 1, "lidar_sa_group_mlp_x3_f32: bad sizes");
    REQUIRE(xyz_level || (p_stride >= c1 && p_stride % 4 == 0), "lidar_sa_group_mlp_x3_f32: bad p_stride");
    REQUIRE(out_offset >= 0 && out_offset + c3 <= out_stride,
            "lidar_sa_group_mlp_x3_f32: output columns exceed out_stride");
    if (batch == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    // the wide feature levels (SA2, MSG's 128-sample branch) run the lean kernel
    if (!xyz_level && c1 == 128 && c2 == 128 && c3 == 256) {
        if (nsample == 64)
            return launch_x3_lean<128, 128, 256, 64>(p, p_stride, q, idx, batch, n, m, packed, out, out_stride,
                                                     out_offset, s);
        if (nsample == 128)
            return launch_x3_lean<128, 128, 256, 128>(p, p_stride, q, idx, batch, n, m, packed, out, out_stride,
                                                      out_offset, s);
    }
#define LIDAR_SAX3(C1_, C2_, C3_, NS_, X_)                                                                   \
    if (!!xyz_level == X_ && c1 == C1_ && c2 == C2_ && c3 == C3_ && nsample == NS_)                           \
        return launch_x3<C1_, C2_, C3_, NS_, X_ ? L1_XYZ : L1_PRE>(p, p_stride, q, idx, batch, n, m, packed, out, \
                                                                out_stride, out_offset, s);
    LIDAR_SAX3(64, 64, 128, 32, true)
    LIDAR_SAX3(32, 32, 64, 16, true)
    LIDAR_SAX3(64, 96, 128, 128, true)
    LIDAR_SAX3(64, 64, 128, 32, false)
#undef LIDAR_SAX3
    return lidar::fail(LIDAR_EINVAL, "lidar_sa_group_mlp_x3_f32: unsupported (widths, nsample) combination");
}

// ------------------------------------------------------------------ X1: the bf16 spec
// bytes of the X1 packed image: [W1 xyz rows fp32 (bf16-rounded), T1*64 floats] [layer-2 / layer-3
// hi fragments] [b1 b2 b3 fp32]
LIDAR_EXPORT int64_t lidar_mlp_packed_size_x1(int32_t c1, int32_t c2, int32_t c3)
{
    return (int64_t)(c1 / 16) * 64 * 4 + ((int64_t)(c2 / 32) * (c1 / 32) + (int64_t)(c3 / 32) * (c2 / 32)) * 2 * 64 * 16 +
           (int64_t)(c1 + c2 + c3) * 4;
}

// host packer of the X1 image: w1 rows 0..2 (the xyz rows of (3 + cfeat, c1)) and w2, w3 rounded
// to bf16 (RNE), the hi fragments of lidar_mlp_pack_x3_f32's order
LIDAR_EXPORT int lidar_mlp_pack_x1_f32(int32_t c1, int32_t c2, int32_t c3, const float *w1, const float *b1,
                                       const float *w2, const float *b2, const float *w3, const float *b3,
                                       void *packed)
{
    REQUIRE(w1 && b1 && w2 && b2 && w3 && b3 && packed, "lidar_mlp_pack_x1_f32: null pointer");
    REQUIRE(c1 % 32 == 0 && c2 % 32 == 0 && c3 % 32 == 0 && c1 > 0 && c2 > 0 && c3 > 0,
            "lidar_mlp_pack_x1_f32: widths must be positive multiples of 32");
    char *o = static_cast<char *>(packed);
    float *f = reinterpret_cast<float *>(o);
    for (int t = 0; t < c1 / 16; ++t)
        for (int l = 0; l < 64; ++l) {
            const int qq = l >> 4;
            *f++ = qq < 3 ? bf16_to_f(bf16_rne(w1[(int64_t)qq * c1 + 16 * t + (l & 15)])) : 0.0f;
        }
    o = reinterpret_cast<char *>(f);
    auto layer = [&](const float *w, int cin, int cout) {
        uint16_t *u = reinterpret_cast<uint16_t *>(o);
        for (int c = 0; c < cout / 32; ++c)
            for (int s = 0; s < cin / 32; ++s)
                for (int t = 0; t < 2; ++t)
                    for (int l = 0; l < 64; ++l)
                        for (int j = 0; j < 8; ++j) {
                            const int in = 32 * s + 16 * (j >> 2) + 4 * (l >> 4) + (j & 3);
                            *u++ = bf16_rne(w[(int64_t)in * cout + 16 * (2 * c + t) + (l & 15)]);
                        }
        o = reinterpret_cast<char *>(u);
    };
    layer(w2, c1, c2);
    layer(w3, c2, c3);
    f = reinterpret_cast<float *>(o);
    for (int i = 0; i < c1; ++i) *f++ = b1[i];
    for (int i = 0; i < c2; ++i) *f++ = b2[i];
    for (int i = 0; i < c3; ++i) *f++ = b3[i];
    return LIDAR_OK;
}

// SA branch in the bf16 spec (BASELINE configs[4]): layer inputs and weights
// rounded to bf16, fp32 accumulation, bias / ReLU / max-pool in fp32.  layer1_mode 0 (xyz
// level): p = the level's points (batch, n, 3), q = centres (batch, m, 3).  layer1_mode 2
// (feature level): p (batch*n, p_stride) = bf16(f) bf16(W1_f) + b1 per point (lidar_dense_x3f_f32
// with the X1 flag), xyz = the level's points, centres; a grouped row's layer 1 is
// relu(p[k] + bf16(W1_xyz) . bf16(x_k - c)).  packed = lidar_mlp_pack_x1_f32's image.
LIDAR_EXPORT int lidar_sa_group_mlp_x1_f32(lidar_handle *h, int32_t layer1_mode, const float *p, int64_t p_stride,
                                           const float *q, const float *xyz, const float *centres,
                                           const int32_t *idx, int64_t batch, int64_t n, int64_t m, int32_t nsample,
                                           int32_t c1, int32_t c2, int32_t c3, const void *packed, float *out,
                                           int64_t out_stride, int64_t out_offset, void *stream)
{
    REQUIRE(h && p && idx && packed && out, "lidar_sa_group_mlp_x1_f32: null pointer");
    REQUIRE(layer1_mode == 0 || layer1_mode == 2, "lidar_sa_group_mlp_x1_f32: layer1_mode must be 0 or 2");
    REQUIRE(layer1_mode == 2 ? (xyz && centres && p_stride >= c1 && p_stride % 4 == 0) : q != nullptr,
            "lidar_sa_group_mlp_x1_f32: mode 0 needs q = centres; mode 2 needs xyz, centres, p_stride >= c1");
    REQUIRE(batch >= 0 && n >= 1 && m >= 1, "lidar_sa_group_mlp_x1_f32: bad sizes");
    REQUIRE(out_offset >= 0 && out_offset + c3 <= out_stride,
            "lidar_sa_group_mlp_x1_f32: output columns exceed out_stride");
    if (batch == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
#define LIDAR_SAX1(C1_, C2_, C3_, NS_, M_)                                                                    \
    if (layer1_mode == M_ && c1 == C1_ && c2 == C2_ && c3 == C3_ && nsample == NS_)                           \
        return launch_x3<C1_, C2_, C3_, NS_, M_, true>(p, p_stride, M_ == 0 ? q : nullptr, idx, batch, n, m,   \
                                                       packed, out, out_stride, out_offset, s, xyz, centres);
    LIDAR_SAX1(32, 32, 64, 16, 0)
    LIDAR_SAX1(64, 64, 128, 32, 0)
    LIDAR_SAX1(64, 96, 128, 128, 0)
    LIDAR_SAX1(64, 64, 128, 32, 2)
    LIDAR_SAX1(128, 128, 256, 64, 2)
    LIDAR_SAX1(128, 128, 256, 128, 2)
#undef LIDAR_SAX1
    return lidar::fail(LIDAR_EINVAL, "lidar_sa_group_mlp_x1_f32: unsupported (widths, nsample) combination");
}

// SA branch of an xyz level with its ball queries answered inside the kernel (sa_x3_kernel with
// BQ) from grid = lidar_ball_query_bin_f32(xyz, radius, nsample)'s output for these frames:
// the same result as lidar_ball_query_binned_f32 followed by lidar_sa_group_mlp_x3_f32 (x1 = 0)
// or lidar_sa_group_mlp_x1_f32 mode 0 (x1 = 1), bit for bit.  out_idx (batch, m, nsample) int32,
// optional, receives the ball-query indices.  packed: the x3 / x1 image of the branch.
LIDAR_EXPORT int lidar_sa_group_mlp_bq_f32(lidar_handle *h, int32_t x1, const float *xyz, const void *grid,
                                           const float *centres, int64_t batch, int64_t n, int64_t m, float radius,
                                           int32_t nsample, int32_t c1, int32_t c2, int32_t c3, const void *packed,
                                           float *out, int64_t out_stride, int64_t out_offset, int32_t *out_idx,
                                           void *stream)
{
    REQUIRE(h && xyz && grid && centres && packed && out, "lidar_sa_group_mlp_bq_f32: null pointer");
    REQUIRE(batch >= 0 && n >= 1 && n < 0x3fffffff && m >= 1 && m < 0x7fffffff,
            "lidar_sa_group_mlp_bq_f32: bad sizes");
    REQUIRE(radius >= 0.0f, "lidar_sa_group_mlp_bq_f32: negative radius");
    REQUIRE(out_offset >= 0 && out_offset + c3 <= out_stride,
            "lidar_sa_group_mlp_bq_f32: output columns exceed out_stride");
    if (batch == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const char *g = static_cast<const char *>(grid);
#define LIDAR_SABQ(C1_, C2_, C3_, NS_)                                                                          \
    if (c1 == C1_ && c2 == C2_ && c3 == C3_ && nsample == NS_)                                                  \
        return x1 ? launch_x3_bq<C1_, C2_, C3_, NS_, true>(xyz, g, centres, batch, n, m, radius, packed, out,    \
                                                           out_stride, out_offset, out_idx, s)                   \
                  : launch_x3_bq<C1_, C2_, C3_, NS_, false>(xyz, g, centres, batch, n, m, radius, packed, out,   \
                                                            out_stride, out_offset, out_idx, s);
    LIDAR_SABQ(64, 64, 128, 32)
    LIDAR_SABQ(32, 32, 64, 16)
    LIDAR_SABQ(64, 96, 128, 128)
#undef LIDAR_SABQ
    return lidar::fail(LIDAR_EINVAL, "lidar_sa_group_mlp_bq_f32: unsupported (widths, nsample) combination");
}
