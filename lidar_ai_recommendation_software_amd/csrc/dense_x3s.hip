// dense_x3s.hip — the dense GEMM of the fp32 contract (SA2's per-point layer 1, group_all's three
// layers) in h3 arithmetic (h3.hpp): y = x W + b [ReLU] [max-pool] with every product carried as
// ah*bh + ah*bl + al*bh on v_mfma_f32_32x32x16_f16 (fp32 accumulation), x scaled per wavefront
// and W per layer by powers of two, unscaled once before the bias.
//
// A is fp32 rows (rows, lda); each wave splits the fragments it reads, every row by its own power
// of two (rows stay independent, as in fp32: a padding row of garbage or a huge row cannot cost
// another row its precision).  The scale is a running one: a K stage whose |x| maximum in a row
// outgrows the row's current scale raises it and rescales that row's accumulators by the (exact)
// power of two, so no scaled value reaches 2^14 (a NaN or inf sets its own row's scale, whose
// products are NaN / inf anyway, as in fp32).
// X1 (the bf16 spec, BASELINE configs[4]): one product bf16(x) bf16(w) per MFMA on
// v_mfma_f32_32x32x16_bf16, no scaling (lidar_dense_x1_pack_f32's image).
//
// Tile: 128 rows x 128 output channels per 4-wave workgroup, a wave's 32 rows x all 128 channels
// (1 x 4 MFMA tiles: each A row is split by the one wave that owns it, not by two), K in stages of
// 32 double-buffered in LDS by global_load_lds:
//   A stage: 128 rows x 32 fp32; row r's 16-byte chunk q at slot q ^ ((r >> 1) & 7);
//   B stage: x3_pack.hip's packed weight fragments, read lane-linear.
// Every output mode computes D = W^T X^T (a lane holds one row: its row's scale is its own):
//   0 fp32 rows (rows, ldo) [+ ReLU]             — a lane stores 4 consecutive channels of its row
//   1 h3 planes (rows, ldo) x 2 [+ ReLU]         — the next layer's A operand already scaled and split
//                                                   (fp16 hi plane, then lo plane), with the row's
//                                                   exponent e (|y| < 2^e) in out_exp[row]
//   2 fp32 max-pool over runs of pool_rows rows  — the max over the 32 rows of a tile by lane
//     (rows / pool_rows, ldo), ReLU, out zeroed     swaps, then an atomic max on the bits (exact,
//     by the caller                                 order-free) across waves and workgroups
// PL (A as h3 planes, lidar_dense_h3p_f32): the producing layer (mode 1) split every element once,
// scaled by its row's exponent, so the GEMM loop does no max pass, no rescale and no split (an
// fp32 row is re-split by every column tile's workgroup: 8 times for group_all's third layer).  A
// row's exponent must hold in every column tile of the producer, so it is a bound, not the row's
// maximum: |y_c| <= sum_k |x_k| |W_kc| + |b_c| < 2^e_in colsum(W) + max|b| (the lean SA2 kernel's
// layer-3 rule, sa_mlp_x3.hip), from the input row's own exponent (PL) or its running one (fp32 A).
#include "h3.hpp"

namespace {

using lidar_h3::f16x8;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef DENSE_SBK
#define DENSE_SBK 32
#endif
constexpr int SBM = 128, SBN = 128, SBK = DENSE_SBK;  // K per LDS stage: 32 (64 KiB of LDS) or 16 (32 KiB)
constexpr int NSS = SBK / 16;                        // MFMA k-steps per stage
constexpr int CPR = SBK / 8;                         // 16-byte chunks per A row (bf16 units)
constexpr int kStageA = SBM * SBK;                   // fp32 per A stage
constexpr int kStageB = 4 * 2 * NSS * 512;           // 16-bit B elements per stage
static_assert(SBK == 16 || SBK == 32, "DENSE_SBK must be 16 or 32");
__device__ __forceinline__ int swzf(int r) { return CPR == 4 ? (r >> 1) & 7 : (r >> 2) & 3; }


__device__ __forceinline__ f32x16 mfma_bf(bf16x8 a, bf16x8 b, f32x16 c)
{
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma_h(f16x8 a, f16x8 b, f32x16 c)
{
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void lds_dma16(const void *g, void *l)
{
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)l, 16, 0, 0);
}

__device__ __forceinline__ float relu_i(float v) { return __int_as_float(max(__float_as_int(v), 0)); }

// NaN-propagating max over the 32 lanes of each half-wave, in every lane of it: four DPP steps
// within each 16-lane row, then v_permlane16_swap's xor-16 partner
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float max_half_wave(float v)
{
    v = __builtin_elementwise_maximum(v, dpp_f<0xB1>(v));   // quad_perm [1,0,3,2]
    v = __builtin_elementwise_maximum(v, dpp_f<0x4E>(v));   // quad_perm [2,3,0,1]
    v = __builtin_elementwise_maximum(v, dpp_f<0x141>(v));  // row_half_mirror
    v = __builtin_elementwise_maximum(v, dpp_f<0x140>(v));  // row_mirror
    const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __builtin_elementwise_maximum(v, __builtin_elementwise_maximum(__uint_as_float(b[0]), __uint_as_float(b[1])));
}

__device__ __forceinline__ bf16x8 round8_bf(const f32x4 &a0, const f32x4 &a1)
{
    bf16x8 hi;
#pragma unroll
    for (int j = 0; j < 8; ++j) hi[j] = (__bf16)(j < 4 ? a0[j] : a1[j - 4]);
    return hi;
}

// r's 16-byte chunk q of a planes stage (CPR per row and plane) sits at slot q ^ swzp(r): a fragment
// read (32 consecutive rows, one chunk) spreads over the banks
__device__ __forceinline__ int swzp(int r) { return CPR == 4 ? (r >> 2) & 3 : (r >> 3) & 1; }

// the h3 output exponent of a row whose inputs are below 2^e_in: |y| < 2^e_in colsum + bmax,
// widened by 2^-10 for the roundings of y and of the bound (sa_mlp_x3.hip's bound_exp3)
__device__ __forceinline__ int out_bound_exp(float colsum, float bmax, int e_in)
{
    const float b = (colsum * ldexpf(1.0f, e_in) + bmax) * (1.0f + 0x1p-10f);
    return lidar_h3::exp_of_bits(__float_as_uint(b));
}

// MODE 0 / 1 / 2 as in the header; X1: the bf16 spec (one ah*bh product, no scaling); PL: A as h3
// planes (hi at a, lo at a + a_plane halves, row exponents a_exp)
// Launch bounds (256, 2): the 64 KiB LDS stage already limits this kernel to 2 workgroups per
// CU. At (256, 4) the compiler capped VGPRs at 64+64 AGPRs and copied the 64 accumulators
// AGPR<->VGPR around every K-stage pair (128 extra VALU per iteration); at (256, 2) they stay
// in VGPRs (102-126 total, 0 AGPRs, no copies).
template <int MODE, bool X1, bool PL = false>
__global__ __launch_bounds__(256, 2) void dense_x3_kernel(const float *__restrict__ af, int lda,
                                                          const uint16_t *__restrict__ wp, int ks,
                                                          const int32_t *__restrict__ wexp,
                                                          const float *__restrict__ bias, int relu_on,
                                                          int pool_rows, float *__restrict__ out, int64_t ldo,
                                                          int cout, int ntn, int64_t total, int64_t per_xcd, int kdim,
                                                          const int32_t *__restrict__ a_exp = nullptr,
                                                          int64_t a_plane = 0, int32_t *__restrict__ out_exp = nullptr,
                                                          float w_colsum = 0.0f, float b_max = 0.0f)
{
    static_assert(!PL || !X1, "h3 planes carry the fp32 contract only");
    static_assert(MODE != 1 || !X1, "mode 1 writes h3 planes");
    // the two stage buffers are separate LDS variables (distinct alias scopes) and the stage loop is
    // unrolled by two, so a stage's reads need not wait for the next stage streaming into the other
    // buffer (with one array indexed by st & 1 the compiler waited for the stage it had just issued)
    __shared__ __attribute__((aligned(16))) float As0[kStageA], As1[kStageA];
    __shared__ __attribute__((aligned(16))) uint16_t Bs0[kStageB], Bs1[kStageB];
    auto Asb = [&](int buf) { return buf ? As1 : As0; };
    auto Bsb = [&](int buf) { return buf ? Bs1 : Bs0; };
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5, col = lane & 31;
    const int64_t L = blockIdx.x;
    const int64_t logical = (L & 7) * per_xcd + (L >> 3);  // a row tile's column tiles share an XCD
    if (logical >= total) return;                           // whole workgroup
    const int64_t row0 = logical / ntn * SBM;
    const int tn = (int)(logical % ntn);
    // stages that hold k < kdim (a 16-deep stage past kdim would be all padding: zero weights, and
    // a read past the row)
    const int nst = (kdim + SBK - 1) / SBK;

    auto load_stage = [&](int st, int buf) {
        const int k0 = st * SBK;
        if constexpr (PL) {
            // wave w: plane w >> 1 (hi, lo), rows 64 (w & 1) .. + 63, CPR instructions of 64 / CPR rows;
            // lane i fills slot i % CPR of its row with chunk slot ^ swzp(row); planes are zero past k
            constexpr int RPI = 64 / CPR;
            const int pl = wave >> 1, rbase = 64 * (wave & 1);
            const uint16_t *ap = reinterpret_cast<const uint16_t *>(af) + pl * a_plane;
            uint16_t *dst = reinterpret_cast<uint16_t *>(Asb(buf)) + pl * (SBM * SBK);
#pragma unroll
            for (int t = 0; t < CPR; ++t) {
                const int r = rbase + RPI * t + lane / CPR;
                const int q = (lane % CPR) ^ swzp(r);
                lds_dma16(ap + (row0 + r) * lda + k0 + 8 * q, dst + (rbase + RPI * t) * SBK);
            }
        } else {
        // wave w: rows 32 w .. 32 w + 31 of 2 CPR 16-byte chunks, CPR instructions
        constexpr int CF = 2 * CPR, RPI = 64 / CF;
        float *dst = Asb(buf);
#pragma unroll
        for (int i = 0; i < CPR; ++i) {
            const int r = 32 * wave + RPI * i + lane / CF;
            const int kq = (lane % CF) ^ swzf(r);
            // chunks at or past k (the weights there are zero) re-read the stage's first chunk:
            // finite, in bounds, and no stale LDS in the products
            const int kc = k0 + 4 * kq < kdim ? k0 + 4 * kq : k0;
            lds_dma16(af + (row0 + r) * lda + kc, dst + (32 * wave + RPI * i) * SBK);
        }
        }
        // B: wave w loads column tile 4 tn + w, k-steps NSS st .. NSS st + NSS - 1, hi / lo (contiguous)
        const uint16_t *src = wp + (((int64_t)(4 * tn + wave) * ks + NSS * st) * 2) * 512;
#pragma unroll
        for (int i = 0; i < 2 * NSS; ++i) lds_dma16(src + i * 512 + lane * 8, &Bsb(buf)[(wave * 2 * NSS + i) * 512]);
        __builtin_amdgcn_sched_barrier(0);  // issued before the stage's reads and MFMAs
    };

    f32x16 acc[4] = {};
    // h3: the running scaling exponent of the lane's row (its values so far are below 2^(E - 3):
    // three bits of headroom, so a later stage rarely needs a rescale); kEmin - 1 = unset
    int E = lidar_h3::kEmin - 1;
    if constexpr (PL) E = a_exp[row0 + 32 * wave + col];  // the row's exponent, fixed
    // the lane's row r = 32 wave + col, k = 8 h .. 8 h + 7 of k-step ss: A fragment of the MFMA
    auto frag = [&](const float *as, int ss, f32x4 &a0, f32x4 &a1) {
        const int r = 32 * wave + col;
        const int kq = 4 * ss + 2 * h;
        const int sl = kq ^ swzf(r);  // kq even: the pair (sl, sl ^ 1)
        a0 = *reinterpret_cast<const f32x4 *>(as + r * SBK + 4 * sl);
        a1 = *reinterpret_cast<const f32x4 *>(as + r * SBK + 4 * (sl ^ 1));
    };
    auto compute = [&](int buf) {
        if constexpr (PL) {
            const uint16_t *ah = reinterpret_cast<const uint16_t *>(Asb(buf));
            const int r = 32 * wave + col;
#pragma unroll
            for (int ss = 0; ss < NSS; ++ss) {
                const int slot = (2 * ss + h) ^ swzp(r);
                const f16x8 xh = *reinterpret_cast<const f16x8 *>(ah + (r * CPR + slot) * 8);
                const f16x8 xl = *reinterpret_cast<const f16x8 *>(ah + SBM * SBK + (r * CPR + slot) * 8);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f16x8 wh = *reinterpret_cast<const f16x8 *>(&Bsb(buf)[((j * NSS + ss) * 2 + 0) * 512 + lane * 8]);
                    const f16x8 wl = *reinterpret_cast<const f16x8 *>(&Bsb(buf)[((j * NSS + ss) * 2 + 1) * 512 + lane * 8]);
                    acc[j] = mfma_h(wh, xh, acc[j]);
                    acc[j] = mfma_h(wl, xh, acc[j]);
                    acc[j] = mfma_h(wh, xl, acc[j]);
                }
            }
            return;
        }
        const float *as = Asb(buf);
        float S = 1.0f;
        if constexpr (!X1) {
            // the stage's |x| maximum of the row, in a pass of its own (the fragments are read again
            // below); a row's values of a stage sit in lanes col and col + 32
            float m = 0.0f;
#pragma unroll
            for (int ss = 0; ss < NSS; ++ss) {
                f32x4 a0, a1;
                frag(as, ss, a0, a1);
#pragma unroll
                for (int t = 0; t < 4; ++t) m = lidar_h3::absmax3(m, a0[t], a1[t]);
            }
            const auto sw32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
            m = lidar_h3::absmax3(m, __uint_as_float(sw32[0]), __uint_as_float(sw32[1]));
            const int e = lidar_h3::exp_of_bits(__float_as_uint(m)) + 3;
            if (__ballot(e > E)) {  // the first stage, then rarely: rescale the rows that grew
                const int d = e > E ? E - e : 0;
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[j][r] = ldexpf(acc[j][r], d);
                E = e > E ? e : E;
            }
            S = lidar_h3::scale_of(E);
            asm volatile("" ::: "memory");  // re-read the fragments below
        }
#pragma unroll
        for (int ss = 0; ss < NSS; ++ss) {
            f32x4 a0, a1;
            frag(as, ss, a0, a1);
            if constexpr (X1) {
                const bf16x8 xh = round8_bf(a0, a1);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const bf16x8 wh = *reinterpret_cast<const bf16x8 *>(&Bsb(buf)[((j * NSS + ss) * 2 + 0) * 512 + lane * 8]);
                    acc[j] = mfma_bf(wh, xh, acc[j]);
                }
            } else {
                f16x8 xh, xl;
                lidar_h3::split8(a0, a1, S, xh, xl);
#pragma unroll
                for (int j = 0; j < 4; ++j) {  // D[channel][row]
                    const f16x8 wh = *reinterpret_cast<const f16x8 *>(&Bsb(buf)[((j * NSS + ss) * 2 + 0) * 512 + lane * 8]);
                    const f16x8 wl = *reinterpret_cast<const f16x8 *>(&Bsb(buf)[((j * NSS + ss) * 2 + 1) * 512 + lane * 8]);
                    acc[j] = mfma_h(wh, xh, acc[j]);
                    acc[j] = mfma_h(wl, xh, acc[j]);
                    acc[j] = mfma_h(wh, xl, acc[j]);
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
    // an image of the other kind (h3 vs bf16) is never reinterpreted: NaN outputs instead
    if (wexp[1] != (X1 ? lidar_h3::kTagX1 : lidar_h3::kTagH3)) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[j][r] = __builtin_nanf("");
    }
    // unscaled by 2^-(s_a + s_w) per row: s_a = 14 - E, s_w from the packed image (X1: none); lane
    // (col, h) holds row row0 + 32 wave + col, channels tn 128 + 32 j + 8 g + 4 h + t (tile j,
    // register 4 g + t)
    if constexpr (!X1) {
        const int us = E - 14 - *wexp;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[j][r] = ldexpf(acc[j][r], us);
    }
    const int cbase = tn * SBN;
    if constexpr (MODE == 1) {
        // h3 planes of y = relu?(acc + b): every column tile's workgroup takes the same exponent for a
        // row (a bound from the row's input exponent E), so the next layer reads one scale per row
        const int64_t row = row0 + 32 * wave + col;
        // |x| < 2^E for planes; the running exponent of fp32 rows keeps three bits of headroom
        const int eo = out_bound_exp(w_colsum, b_max, PL ? E : E - 3);
        const float so = lidar_h3::scale_of(eo);
        uint16_t *oh = reinterpret_cast<uint16_t *>(out);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int c = cbase + 32 * j + 8 * g + 4 * h;
                const f32x4 b4 = *reinterpret_cast<const f32x4 *>(bias + c);
                float v[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const float y = acc[j][4 * g + t] + b4[t];
                    v[t] = (relu_on ? relu_i(y) : y) * so;
                }
                uint32_t hi[2], lo[2];
                lidar_h3::split2(v[0], v[1], hi[0], lo[0]);
                lidar_h3::split2(v[2], v[3], hi[1], lo[1]);
                *reinterpret_cast<uint2 *>(oh + row * ldo + c) = make_uint2(hi[0], hi[1]);
                *reinterpret_cast<uint2 *>(oh + row * ldo + c + (int64_t)total / ntn * SBM * ldo) = make_uint2(lo[0], lo[1]);
            }
        if (h == 0 && tn == 0) out_exp[row] = eo;
    } else if constexpr (MODE == 0) {
        const int64_t row = row0 + 32 * wave + col;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int c = cbase + 32 * j + 8 * g + 4 * h;
                const f32x4 b4 = *reinterpret_cast<const f32x4 *>(bias + c);
                f32x4 v;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const float y = acc[j][4 * g + t] + b4[t];
                    v[t] = relu_on ? relu_i(y) : y;
                }
                *reinterpret_cast<f32x4 *>(out + row * ldo + c) = v;
            }
    } else {
        unsigned *orow = reinterpret_cast<unsigned *>(out + (row0 / pool_rows) * ldo);
        // the max over the wave's 32 rows per channel, over the 32 lanes of each h; then an atomic
        // max across waves and workgroups.  relu(max + b) == max relu(x + b) (x -> relu(x + b) is
        // monotone); non-negative floats order as their bits: exact, order-free
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float mine = 0.0f;  // lane col < 16 of each half-wave takes register col's max
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float v = max_half_wave(acc[j][r]);
                mine = col == r ? v : mine;
            }
            if (col < 16) {  // one 32-lane atomic per tile (not one per register)
                const int c = cbase + 32 * j + 8 * (col >> 2) + 4 * h + (col & 3);
                atomicMax(orow + c, __float_as_uint(relu_i(mine + bias[c])));
            }
        }
    }
}

}  // namespace

int lidar_dense_x3_packed_image(int32_t k, int32_t cout, int64_t *bytes);  // x3_pack.hip

// the GEMM with A as fp32 rows (rows, lda) (split inside the tile loop; elements k..lda-1 are
// read and must be finite — weights there are zero).  mode 0: fp32 rows out (rows, ldo);
// mode 2: fp32 max over runs of pool_rows rows (ReLU; out zeroed by the caller).  mode | 4: the
// bf16 spec (X1) on lidar_dense_x1_pack_f32's image (mode 0 only); otherwise packed =
// lidar_dense_x3_pack_f32's h3 image.
LIDAR_EXPORT int lidar_dense_x3f_f32(lidar_handle *h, const float *a, int32_t lda, int64_t rows, int32_t k,
                                     const void *packed, const float *bias, int32_t cout, int32_t mode,
                                     int32_t relu_on, int32_t pool_rows, void *out, int64_t o_plane, int64_t ldo,
                                     void *stream)
{
    const bool x1 = (mode & 4) != 0;
    mode &= 3;
    (void)o_plane;
    REQUIRE(!x1 || mode == 0, "lidar_dense_x3f_f32: the X1 flag needs mode 0");
    REQUIRE(h && a && packed && bias && out, "lidar_dense_x3f_f32: null pointer");
    REQUIRE(rows % SBM == 0 && k > 0 && k <= lda && cout % SBN == 0 && cout > 0,
            "lidar_dense_x3f_f32: rows % 128, k <= lda, cout % 128 must hold");
    REQUIRE(k % 4 == 0 && lda % 4 == 0, "lidar_dense_x3f_f32: k % 4 == 0 and lda % 4 == 0 (fp32 rows)");
    REQUIRE(mode == 0 || mode == 2, "lidar_dense_x3f_f32: mode must be 0 or 2");
    REQUIRE(ldo >= cout && ldo % 4 == 0, "lidar_dense_x3f_f32: ldo must be >= cout and a multiple of 4");
    REQUIRE(mode != 2 || (relu_on && pool_rows > 0 && pool_rows % SBM == 0 && rows % pool_rows == 0),
            "lidar_dense_x3f_f32: the max-pool needs relu and pool_rows a multiple of 128 dividing rows");
    if (rows == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    const int ks = (k + 31) / 32 * 2;  // the packed image of a (k, cout) layer covers ceil(k/32)*2 k-steps
    const int ntn = cout / SBN;
    const int64_t total = (rows / SBM) * ntn, per_xcd = (total + 7) / 8;
    REQUIRE(per_xcd * 8 <= 0x7fffffff, "lidar_dense_x3f_f32: too many rows");
    int64_t wbytes = 0;
    if (lidar_dense_x3_packed_image(k, cout, &wbytes) != LIDAR_OK) return LIDAR_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint16_t *w = static_cast<const uint16_t *>(packed);
    // the h3 image ends in its layer scaling exponent (x3_pack.hip)
    const int32_t *wexp = reinterpret_cast<const int32_t *>(static_cast<const char *>(packed) + wbytes);
    const dim3 grid((unsigned)(per_xcd * 8)), block(256);
    auto go = [&](auto kern, int relu, int pool) {
        hipLaunchKernelGGL(kern, grid, block, 0, s, a, (int)lda, w, ks, wexp, bias, relu, pool,
                           static_cast<float *>(out), ldo, (int)cout, ntn, total, per_xcd, (int)k,
                           (const int32_t *)nullptr, (int64_t)0, (int32_t *)nullptr, 0.0f, 0.0f);
    };
    const int rl = relu_on ? 1 : 0;
    if (x1) go(dense_x3_kernel<0, true>, rl, 0);
    else if (mode == 0) go(dense_x3_kernel<0, false>, rl, 0);
    else go(dense_x3_kernel<2, false>, 1, (int)pool_rows);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

// The h3 chain of group_all: A as fp32 rows (a_exp NULL; lda % 4 == 0, elements k..lda-1 read and
// finite) or as h3 planes (a_exp (rows,) int32 the rows' exponents, |x| < 2^e: hi plane (rows, lda)
// fp16 at a, lo plane at a + rows * lda halves; lda = k rounded up to 32, zeros past k — what mode 1
// writes).  mode 0: fp32 rows (rows, ldo) [+ ReLU]; 1: h3 planes of y [+ ReLU] (hi at out, lo at
// out + rows * ldo halves, ldo % 8 == 0) and out_exp (rows,) — their exponent, from the bound
// 2^e_in w_colsum + b_max (w_colsum >= max over columns of sum_k |W_kc|, b_max >= max |b|: the
// caller's, rounded up); 2: ReLU + max over runs of pool_rows rows (out zeroed by the caller).
LIDAR_EXPORT int lidar_dense_h3p_f32(lidar_handle *h, const void *a, int32_t lda, int64_t rows, int32_t k,
                                     const int32_t *a_exp, const void *packed, const float *bias, int32_t cout,
                                     int32_t mode, int32_t relu_on, int32_t pool_rows, void *out, int32_t *out_exp,
                                     int64_t ldo, float w_colsum, float b_max, void *stream)
{
    const bool pl = a_exp != nullptr;
    REQUIRE(h && a && packed && bias && out, "lidar_dense_h3p_f32: null pointer");
    REQUIRE(rows % SBM == 0 && k > 0 && k <= lda && cout % SBN == 0 && cout > 0,
            "lidar_dense_h3p_f32: rows % 128, k <= lda, cout % 128 must hold");
    REQUIRE(pl ? lda == (k + 31) / 32 * 32 : (k % 4 == 0 && lda % 4 == 0),
            "lidar_dense_h3p_f32: planes need lda = k rounded up to 32; fp32 rows k % 4 == 0 and lda % 4 == 0");
    REQUIRE(mode >= 0 && mode <= 2, "lidar_dense_h3p_f32: mode must be 0, 1 or 2");
    REQUIRE(mode != 1 || (out_exp != nullptr && ldo == cout && w_colsum >= 0.0f && b_max >= 0.0f),
            "lidar_dense_h3p_f32: mode 1 needs out_exp, ldo == cout and the bounds w_colsum, b_max >= 0");
    REQUIRE(ldo >= cout && ldo % 4 == 0, "lidar_dense_h3p_f32: ldo must be >= cout and a multiple of 4");
    REQUIRE(mode != 2 || (relu_on && pool_rows > 0 && pool_rows % SBM == 0 && rows % pool_rows == 0),
            "lidar_dense_h3p_f32: the max-pool needs relu and pool_rows a multiple of 128 dividing rows");
    if (rows == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    const int ks = (k + 31) / 32 * 2;
    const int ntn = cout / SBN;
    const int64_t total = (rows / SBM) * ntn, per_xcd = (total + 7) / 8;
    REQUIRE(per_xcd * 8 <= 0x7fffffff, "lidar_dense_h3p_f32: too many rows");
    int64_t wbytes = 0;
    if (lidar_dense_x3_packed_image(k, cout, &wbytes) != LIDAR_OK) return LIDAR_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint16_t *w = static_cast<const uint16_t *>(packed);
    const int32_t *wexp = reinterpret_cast<const int32_t *>(static_cast<const char *>(packed) + wbytes);
    const dim3 grid((unsigned)(per_xcd * 8)), block(256);
    const float *af = static_cast<const float *>(a);
    float *o = static_cast<float *>(out);
    const int rl = relu_on ? 1 : 0;
    auto go = [&](auto kern, int relu, int pool) {
        hipLaunchKernelGGL(kern, grid, block, 0, s, af, (int)lda, w, ks, wexp, bias, relu, pool, o, ldo, (int)cout, ntn,
                           total, per_xcd, (int)k, a_exp, rows * lda, out_exp, w_colsum, b_max);
    };
    if (pl) {
        if (mode == 0) go(dense_x3_kernel<0, false, true>, rl, 0);
        else if (mode == 1) go(dense_x3_kernel<1, false, true>, rl, 0);
        else go(dense_x3_kernel<2, false, true>, 1, (int)pool_rows);
    } else {
        if (mode == 0) go(dense_x3_kernel<0, false>, rl, 0);
        else if (mode == 1) go(dense_x3_kernel<1, false>, rl, 0);
        else go(dense_x3_kernel<2, false>, 1, (int)pool_rows);
    }
    LAUNCH_CHECK();
    return LIDAR_OK;
}
