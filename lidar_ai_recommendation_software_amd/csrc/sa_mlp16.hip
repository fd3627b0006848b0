// sa_mlp16.hip — SetAbstraction layers on v_mfma_f32_16x16x4_f32, 16 grouped rows per wave.
//
// The fused SetAbstraction branch (gather -> MFMA chain -> max-pool, weights streamed
// through LDS in 16 KiB chunks shared by the 4 waves of a workgroup), with 16-row tiles:
//   16x16x4 f32: lane l holds A[l&15][k = l>>4], B[k = l>>4][l&15]; D reg r of lane l is row
//   4*(l>>4) + r, column l&15.
// Layer l's accumulators (channel rows x point columns: reg r of lane l = channel
// 16t + 4(l>>4) + r of point l&15) are directly the next layer's B operand — MFMA step
// (ti, r) feeds channels 16ti + 4q + r from lane group q; that k order is folded into the
// packed weights (lidar_mlp_pack16_f32).  The last layer is computed transposed (point rows x
// channel columns) so the max over the 16 points is 4 register maxes + 2 xor swaps.  Layer 1
// of a level without features is ONE MFMA per 16-channel tile: lane group q supplies
// (dx, dy, dz, 0)[q].  Two output tiles are accumulated in alternation (a 16x16x4 f32 MFMA
// issues every 32 cycles but its result is ready after 40).
//
// Why 16 rows: the activations of 16 rows take half the registers of 32 (y1 + y2 = 64 VGPRs
// for 128-wide layers), so the kernel fits ~128 VGPRs: 4 waves per SIMD, and 2 still fit on a
// CU that also hosts an FPS workgroup (32-row tiles need ~256 and drop to 1 there).
#include <vector>

#include "common.hpp"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c)
{
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }

// packed image (floats): [W1: T1*64 (XYZ levels only, see below)] [chunks of layer 2]
// [chunks of layer 3] [b1 C1] [b2 C2] [b3 C3].  A chunk covers output tiles (2c, 2c+1) of a
// layer with K input channels: K/8 float4 per lane, element (2 sp + e) of tile (2c + t) at
// [sp][lane][2t + e] = W[in(2sp+e, l>>4)][16(2c+t) + (l&15)], in(s, q) = 16(s/4) + 4q + s%4.
template <int C1, int C2, int C3>
struct Pack16 {
    static constexpr int T1 = C1 / 16, T2 = C2 / 16, T3 = C3 / 16;
    static constexpr int CH2 = C1 / 8 * 64, CH3 = C2 / 8 * 64;  // chunk sizes in float4
    static constexpr int64_t W1 = (int64_t)T1 * 64;             // floats
};

template <int C1, int C2, int C3, int NS, bool XYZ, int WPG>
__global__ __launch_bounds__(64 * WPG, 4) void sa16_kernel(const float *__restrict__ P, int64_t stride,
                                                   const float *__restrict__ Q, const int32_t *__restrict__ idx,
                                                   int n, int m, int64_t total, const float *__restrict__ packed,
                                                   float *__restrict__ out, int64_t out_stride, int64_t out_offset)
{
    static_assert(NS % 16 == 0, "16-row tiles");
    using K = Pack16<C1, C2, C3>;
    constexpr int T1 = K::T1, T2 = K::T2, T3 = K::T3;
    constexpr int CH2 = K::CH2, CH3 = K::CH3, CHMAX = CH2 > CH3 ? CH2 : CH3;
    constexpr int NCH = T2 / 2 + T3 / 2;  // chunks per row tile
    constexpr int TILES = NS / 16;
    constexpr int NT = 64 * WPG;  // threads per workgroup: WPG waves share every weight chunk
    constexpr int PER = (CHMAX + NT - 1) / NT;
    static_assert(CH2 % 64 == 0 && CH3 % 64 == 0, "chunks copied in 64-float4 slabs, one per wave");
    static_assert(T2 % 2 == 0 && T3 % 2 == 0, "output tiles come in pairs");

    // two LDS variables (distinct alias scopes) when the chunk count per tile is even, so the buffer of a
    // pass is a compile-time choice: a pass's reads (and its max-pool stores) then need not wait for the
    // chunk streaming into the other buffer (as sa_x3_kernel's SPLIT, sa_mlp_x3.hip)
    constexpr bool SPLIT = NCH % 2 == 0;
    __shared__ f32x4 bufa[SPLIT ? 1 : 2][CHMAX];
    __shared__ f32x4 bufb[SPLIT ? CHMAX : 1];
    auto bufp = [&](int p) -> f32x4 * {
        if constexpr (SPLIT)
            return p ? bufb : bufa[0];
        else
            return bufa[p];
    };
    __shared__ float bias_s[C1 + C2 + C3];
    __shared__ float w1_s[XYZ ? T1 * 64 : 1];
    __shared__ float mx_s[WPG][C3];  // running max-pool per wave: kept out of the registers

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int q = lane >> 4, col = lane & 15;
    const int64_t unit = (int64_t)blockIdx.x * WPG + wave;
    const bool live = unit < total;  // every wave takes part in the barriers
    const int64_t cc = live ? unit : total - 1;
    const int64_t b = cc / m;

    const float *W1 = packed;
    const f32x4 *W2 = reinterpret_cast<const f32x4 *>(packed + (XYZ ? K::W1 : 0));
    const f32x4 *W3 = W2 + (int64_t)(T2 / 2) * CH2;
    const float *Bias = reinterpret_cast<const float *>(W3 + (int64_t)(T3 / 2) * CH3);

    auto chunk_src = [&](int c) -> const f32x4 * { return c < T2 / 2 ? W2 + c * CH2 : W3 + (c - T2 / 2) * CH3; };
    auto chunk_len = [&](int c) -> int { return c < T2 / 2 ? CH2 : CH3; };
    auto fetch = [&](int c, int dst) {
        const f32x4 *src = chunk_src(c);
        asm volatile("" : "+s"(src));  // keep each chunk's loads in their own iteration
        const int len = chunk_len(c);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int base = NT * i + 64 * wave;
            if ((SPLIT && CH2 == CH3 && CH2 % NT == 0) || base < len)  // equal whole chunks: unconditional
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(src + base + lane),
                                                 (__attribute__((address_space(3))) void *)(&bufp(dst)[base]), 16, 0,
                                                 0);
        }
        if constexpr (SPLIT) __builtin_amdgcn_sched_barrier(0);  // issued before the pass's reads and MFMAs
    };
    fetch(0, 0);
    for (int i = tid; i < C1 + C2 + C3; i += NT) bias_s[i] = Bias[i];
    if constexpr (XYZ)
        for (int i = tid; i < T1 * 64; i += NT) w1_s[i] = W1[i];
    __syncthreads();

    for (int i = lane; i < C3; i += 64) mx_s[wave][i] = 0.0f;  // post-ReLU values are >= 0
    int par = 0;

#pragma unroll 1
    for (int tile = 0; tile < TILES; ++tile) {
        const int64_t k = idx[cc * NS + tile * 16 + col];
        f32x4 y1[T1];
        if constexpr (XYZ) {
            const float *pr = P + ((int64_t)b * n + k) * 3;
            const float *ce = Q + cc * 3;
            const float x = q < 3 ? pr[q] - ce[q] : 0.0f;  // lane group q: dx, dy, dz, 0
#pragma unroll
            for (int t = 0; t < T1; ++t) {
                f32x4 acc = {};
                acc = mfma16(w1_s[t * 64 + lane], x, acc);
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[r] = relu(acc[r] + bias_s[16 * t + 4 * q + r]);
                y1[t] = acc;
            }
        } else {
            // relu(P[k] - Q[c]): channel 16ti + 4q + r of point k
            const f32x4 *pp = reinterpret_cast<const f32x4 *>(P + ((int64_t)b * n + k) * stride + 4 * q);
            // the centre row is re-read per tile (an L1 hit): hoisted out of the loop it would
            // pin C1 / 2 VGPRs for the whole kernel and cost a wave per SIMD beside FPS work
            int zero = 0;
            asm volatile("" : "+v"(zero));
            const f32x4 *qq = reinterpret_cast<const f32x4 *>(Q + cc * stride + 4 * q + zero);
#pragma unroll
            for (int ti = 0; ti < T1; ++ti) {
                const f32x4 a = pp[4 * ti], c = qq[4 * ti];
#pragma unroll
                for (int r = 0; r < 4; ++r) y1[ti][r] = relu(a[r] - c[r]);
            }
        }

        f32x4 y2[T2];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int cn = c + 1 < NCH ? c + 1 : 0;
            const bool more = c + 1 < NCH || tile + 1 < TILES;
            if (more) fetch(cn, par ^ 1);  // lands during this chunk's MFMAs
            const f32x4 *wb = bufp(par) + lane;
            f32x4 a0 = {}, a1 = {};
            if (c < T2 / 2) {  // layer 2: output tiles 2c, 2c+1 (channel rows x point columns)
                constexpr int S = C1 / 4;  // k-steps
#pragma unroll
                for (int sp = 0; sp < S / 2; ++sp) {
                    const f32x4 w = wb[sp * 64];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int s = 2 * sp + e;
                        const float act = y1[s / 4][s % 4];
                        a0 = mfma16(w[e], act, a0);
                        a1 = mfma16(w[2 + e], act, a1);
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    a0[r] = relu(a0[r] + bias_s[C1 + 16 * (2 * c) + 4 * q + r]);
                    a1[r] = relu(a1[r] + bias_s[C1 + 16 * (2 * c + 1) + 4 * q + r]);
                }
                y2[2 * c < T2 ? 2 * c : 0] = a0;
                y2[2 * c + 1 < T2 ? 2 * c + 1 : 0] = a1;
            } else {  // layer 3: output tiles 2t', 2t'+1, transposed, + max over the 16 rows
                const int tp = c - T2 / 2;
                constexpr int S = C2 / 4;
#pragma unroll
                for (int sp = 0; sp < S / 2; ++sp) {
                    const f32x4 w = wb[sp * 64];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int s = 2 * sp + e;
                        const float act = y2[s / 4][s % 4];
                        a0 = mfma16(act, w[e], a0);
                        a1 = mfma16(act, w[2 + e], a1);
                    }
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const f32x4 &acc = h ? a1 : a0;
                    const int t = 2 * tp + h;
                    const float bias = bias_s[C1 + C2 + 16 * t + col];
                    float v = 0.0f;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v = fmaxf(v, relu(acc[r] + bias));
                    v = fmaxf(v, __shfl_xor(v, 16, 64));
                    v = fmaxf(v, __shfl_xor(v, 32, 64));
                    if (q == 0) {
                        float &m = mx_s[wave][(t < T3 ? 16 * t : 0) + col];
                        m = fmaxf(m, v);
                    }
                }
            }
            __syncthreads();  // (vmcnt(0)) chunk c+1 landed for everyone; buf[par] free for c+2
            par ^= 1;
        }
    }
    if (live && q == 0) {
        float *o = out + unit * out_stride + out_offset;
#pragma unroll
        for (int t = 0; t < T3; ++t) o[16 * t + col] = mx_s[wave][16 * t + col];
    }
}

template <int C1, int C2, int C3, int NS, bool XYZ, int WPG>
int launch16w(const float *p, int64_t stride, const float *q, const int32_t *idx, int64_t batch, int64_t n,
              int64_t m, const float *packed, float *out, int64_t os, int64_t oo, hipStream_t s)
{
    const int64_t total = batch * m;
    const int64_t blocks = (total + WPG - 1) / WPG;
    REQUIRE(blocks <= 0x7fffffff, "sa_group_mlp16: too many centres");
    hipLaunchKernelGGL((sa16_kernel<C1, C2, C3, NS, XYZ, WPG>), dim3((unsigned)blocks), dim3(64 * WPG), 0, s, p,
                       stride, q, idx, (int)n, (int)m, total, packed, out, os, oo);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

template <int C1, int C2, int C3, int NS, bool XYZ>
int launch16(const float *p, int64_t stride, const float *q, const int32_t *idx, int64_t batch, int64_t n,
             int64_t m, const float *packed, float *out, int64_t os, int64_t oo, hipStream_t s)
{
    // 4 waves per workgroup: 8 (half the weight-chunk traffic per MFMA) measured slower in
    // the pipeline (425 vs 450 M pts/s), occupancy matters more than L2 -> LDS bytes here
    return launch16w<C1, C2, C3, NS, XYZ, 4>(p, stride, q, idx, batch, n, m, packed, out, os, oo, s);
}

}  // namespace

LIDAR_EXPORT int64_t lidar_mlp_packed_size16(int32_t xyz_level, int32_t c1, int32_t c2, int32_t c3)
{
    return (xyz_level ? (int64_t)(c1 / 16) * 64 : 0) + (int64_t)(c2 / 16) * (c1 / 4) * 64 +
           (int64_t)(c3 / 16) * (c2 / 4) * 64 + c1 + c2 + c3;
}

// host packer for the 16-row kernels: w1 (3 or 3 + cfeat rows, c1) is only read for an xyz
// level (its first 3 rows: dx, dy, dz); w2 (c1, c2), w3 (c2, c3); biases b1, b2, b3
LIDAR_EXPORT int lidar_mlp_pack16_f32(int32_t xyz_level, int32_t c1, int32_t c2, int32_t c3, const float *w1,
                                      const float *b1, const float *w2, const float *b2, const float *w3,
                                      const float *b3, float *packed)
{
    REQUIRE(b1 && w2 && b2 && w3 && b3 && packed && (!xyz_level || w1), "lidar_mlp_pack16_f32: null pointer");
    REQUIRE(c1 % 32 == 0 && c2 % 32 == 0 && c3 % 32 == 0 && c1 > 0 && c2 > 0 && c3 > 0,
            "lidar_mlp_pack16_f32: widths must be positive multiples of 32");
    float *o = packed;
    if (xyz_level) {
        for (int t = 0; t < c1 / 16; ++t)
            for (int l = 0; l < 64; ++l) {
                const int qq = l >> 4;
                *o++ = qq < 3 ? w1[(int64_t)qq * c1 + 16 * t + (l & 15)] : 0.0f;
            }
    }
    auto layer = [&](const float *w, int cin, int cout) {
        const int steps = cin / 4;
        for (int c = 0; c < cout / 32; ++c)
            for (int sp = 0; sp < steps / 2; ++sp)
                for (int l = 0; l < 64; ++l)
                    for (int t = 0; t < 2; ++t)
                        for (int e = 0; e < 2; ++e) {
                            const int s = 2 * sp + e;
                            const int in = 16 * (s / 4) + 4 * (l >> 4) + s % 4;
                            *o++ = w[(int64_t)in * cout + 16 * (2 * c + t) + (l & 15)];
                        }
    };
    layer(w2, c1, c2);
    layer(w3, c2, c3);
    for (int i = 0; i < c1; ++i) *o++ = b1[i];
    for (int i = 0; i < c2; ++i) *o++ = b2[i];
    for (int i = 0; i < c3; ++i) *o++ = b3[i];
    return LIDAR_OK;
}

// the 16-row fused kernels.  xyz_level: p = xyz (B*n, 3), q = centres (B*m, 3) and layer 1 runs
// here; else p / q are the per-point / per-centre layer-1 rows (layer1_per_point's
// P and Q, row stride p_stride).  packed: lidar_mlp_pack16_f32's image.
LIDAR_EXPORT int lidar_sa_group_mlp16_f32(lidar_handle *h, int32_t xyz_level, const float *p, int64_t p_stride,
                                          const float *q, const int32_t *idx, int64_t batch, int64_t n, int64_t m,
                                          int32_t nsample, int32_t c1, int32_t c2, int32_t c3, const float *packed,
                                          float *out, int64_t out_stride, int64_t out_offset, void *stream)
{
    REQUIRE(h && p && q && idx && packed && out, "lidar_sa_group_mlp16_f32: null pointer");
    REQUIRE(batch >= 0 && n >= 1 && m >= 1, "lidar_sa_group_mlp16_f32: bad sizes");
    REQUIRE(xyz_level || (p_stride >= c1 && p_stride % 4 == 0), "lidar_sa_group_mlp16_f32: bad p_stride");
    REQUIRE(out_offset >= 0 && out_offset + c3 <= out_stride, "lidar_sa_group_mlp16_f32: output columns exceed out_stride");
    if (batch == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
#define LIDAR_SA16(C1_, C2_, C3_, NS_, X_)                                                                 \
    if (!!xyz_level == X_ && c1 == C1_ && c2 == C2_ && c3 == C3_ && nsample == NS_)                         \
        return launch16<C1_, C2_, C3_, NS_, X_>(p, p_stride, q, idx, batch, n, m, packed, out, out_stride, \
                                                out_offset, s);
    LIDAR_SA16(64, 64, 128, 32, true)
    LIDAR_SA16(32, 32, 64, 16, true)
    LIDAR_SA16(128, 128, 256, 64, false)
    LIDAR_SA16(128, 128, 256, 128, false)
    LIDAR_SA16(64, 64, 128, 32, false)
    LIDAR_SA16(64, 96, 128, 128, true)
#undef LIDAR_SA16
    return lidar::fail(LIDAR_EINVAL, "lidar_sa_group_mlp16_f32: unsupported (widths, nsample) combination");
}
