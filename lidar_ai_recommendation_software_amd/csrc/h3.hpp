// h3.hpp — fp32 products carried by the fp16 matrix cores ("h3" arithmetic).
//
// An fp32 operand x is scaled by a power of two S (exact) and split as
//   hi = fp16(x S),  lo = fp16(x S - hi)          (RNE both; x S - hi is exact in fp32)
// and a product as  a b S_a S_w ~ ah bh + ah bl + al bh   (three fp16 MFMAs, fp32 accumulation;
// fp16 x fp16 products are exact in fp32), unscaled once at the end by 2^-(s_a + s_w) (exact).
// With 11-bit pieces (unit roundoff 2^-11) x S = hi + lo + r with |r| <= 2^-22 |x S|, and the
// dropped al bl, ah br, ar bh are <= 3 2^-22 (1 + 2^-10) |a b| for every element within 2^14 of
// its scaling group's maximum (below that, 2^-38 of the maximum absolute): the size of an fp32
// accumulation's own rounding, at the bf16 MFMA rate.  (The bf16 pieces of rounds 1-3 left
// 3 2^-16 per product, which failed 1e-4 relative on the small elements of the features:
// tools/x3_error_model.py.)
//
// Scaling groups: weights per layer (at pack time), activations per row (the dense GEMM, a running
// maximum over the K stages) or per 16-row tile of one centre's neighbourhood (the SA kernels).
// The scale keeps the group's maximum below 2^14 (fp16 holds up to 65504), so no value can
// overflow; elements below 2^-14 of the maximum keep an absolute precision of 2^-38 of it.  A NaN
// or inf sets its own group's scale (its fp32 products would be NaN / inf anyway).
//
// Non-finite operands: an inf splits into hi = inf, lo = inf - inf = NaN, and a 0 piece times an
// inf one is NaN, so every output an inf or NaN operand reaches is NaN in h3 where fp32 would give
// +-inf or NaN: non-finite outputs stay non-finite (tests/test_gpu_tier_n.py::test_dense_x3s_nonfinite),
// only the class (inf vs NaN) may differ.  Finite rows are unaffected (scaling groups are per row / tile).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.hpp"

namespace lidar_h3 {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// image-kind tags in the second int32 of a dense weight image's tail (x3_pack.hip): the GEMM
// checks that the image matches its mode and writes NaN outputs otherwise (never a silent mix-up)
constexpr int32_t kTagH3 = 0x33484d47;  // "GMH3": fp16 hi / lo of W 2^s, s in tail[0]
constexpr int32_t kTagX1 = 0x31584d47;  // "GMX1": bf16(W) for the bf16 spec
constexpr int kEmin = -100;  // exponent floor: groups whose maximum is 0 or below 2^-100
constexpr int kEmax = 128;   // inf / NaN maxima (their products are inf / NaN anyway)

// e with max < 2^e (max given as the bits of a non-negative float), clamped to [kEmin, kEmax]
__host__ __device__ inline int exp_of_bits(uint32_t mbits)
{
    const int e8 = (int)(mbits >> 23);
    int e = e8 == 0 ? kEmin : e8 - 126;
    e = e < kEmin ? kEmin : e;
    return e > kEmax ? kEmax : e;
}

// the scale 2^(14 - e) (a normal float for every e in [kEmin, kEmax])
__host__ __device__ inline float scale_of(int e)
{
    const uint32_t b = (uint32_t)(14 - e + 127) << 23;
    float f;
    __builtin_memcpy(&f, &b, 4);
    return f;
}

// hi = fp16(v), lo = fp16(v - hi) of already-scaled values, two at a time: one v_cvt_pk_f16_f32
// for the his, one v_fma_mix{lo,hi}_f16 per lo (fma(hi, -1, v) is v - hi exactly, rounded once to
// fp16, RNE) — 1.5 VALU per element instead of 3 (convert hi back, subtract, convert)
__device__ __forceinline__ void split2(float v0, float v1, uint32_t &hi, uint32_t &lo)
{
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    const f16x2 h = {(_Float16)v0, (_Float16)v1};
    hi = __builtin_bit_cast(uint32_t, h);
    // mixlo writes the low half (its high half is whatever the register held: mixhi overwrites it)
    uint32_t l;
    asm volatile("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(hi), "v"(v0));
    asm volatile("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l) : "v"(hi), "v"(v1));
    lo = l;
}

// eight values (two accumulator quads) scaled by s, split into the hi / lo fragments
__device__ __forceinline__ void split8(const f32x4 &a0, const f32x4 &a1, float s, f16x8 &hi, f16x8 &lo)
{
    uint32_t h[4], l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float v0 = (j < 2 ? a0[2 * j] : a1[2 * j - 4]) * s, v1 = (j < 2 ? a0[2 * j + 1] : a1[2 * j - 3]) * s;
        split2(v0, v1, h[j], l[j]);
    }
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    hi = __builtin_bit_cast(f16x8, u32x4{h[0], h[1], h[2], h[3]});
    lo = __builtin_bit_cast(f16x8, u32x4{l[0], l[1], l[2], l[3]});
}

// max |v| of a group's values: NaN-propagating (v_maximum3 with abs modifiers; a NaN or inf sets
// its own group's scale, whose fp32 products would be NaN / inf anyway)
__device__ __forceinline__ float absmax3(float m, float a, float b)
{
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(m, __builtin_fabsf(a)), __builtin_fabsf(b));
}

// |v| as bits (a non-negative float orders as its bits; NaN above inf)
__device__ __forceinline__ uint32_t abs_bits(float v) { return __float_as_uint(v) & 0x7fffffffu; }
// the wave's scaling exponent from every lane's max |v| bits (wave-uniform result)
__device__ __forceinline__ int wave_exp(uint32_t lane_bits)
{
    return exp_of_bits((uint32_t)lidar::wave_max_i32_dpp((int)lane_bits));
}

}  // namespace lidar_h3
