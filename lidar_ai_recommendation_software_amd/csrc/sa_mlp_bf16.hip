// sa_mlp_bf16.hip — the SetAbstraction shared MLP in bf16 on gfx950 MFMA
// (v_mfma_f32_32x32x16_bf16, fp32 accumulation): BASELINE.json configs[4] (MSG + bf16).
//
// Same fused structure as sa_mlp.hip (gather + 3 layers + max-pool per 32-row tile, layer
// chaining in registers, last layer transposed so the pool is a register max), with the
// bf16 fragment maps: lane l holds A[row l&31][k = 8h + j] and B[k = 8h + j][col l&31]
// (h = l >> 5, j = 0..7); the fp32 accumulator of one layer becomes the next layer's
// operand by converting registers 8s..8s+7 to bf16 (v_cvt_pk_bf16_f32, RNE) — element j
// of lane half h is channel 16s + 8(j>>2) + 4h + (j&3) of the tile, and that order is
// folded into the packed weight image (lidar_mlp_pack_bf16).
//
// Numerics (the bf16 spec): every layer's inputs (grouped xyz offsets,
// features, hidden activations) and weights are rounded to bf16 (RNE); products are
// accumulated in fp32; bias and ReLU in fp32; the pooled output is fp32.
#include <cstring>

#include "common.hpp"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int rho(int r) { return (r & 3) + 8 * (r >> 2); }

__device__ __forceinline__ f32x16 mfma16(bf16x8 a, bf16x8 b, f32x16 c)
{
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }

template <int CF, int C1, int C2, int C3>
struct Shape16 {
    static constexpr int K1 = (CF + 3 + 15) / 16 * 16;  // [features, dx, dy, dz, 0-pad]
    static constexpr int S1 = K1 / 16;
    static constexpr int T1 = C1 / 32, T2 = C2 / 32, T3 = C3 / 32;
    static constexpr int64_t W1 = (int64_t)T1 * S1 * 64;  // bf16x8 units
    static constexpr int64_t W2 = (int64_t)T2 * T1 * 2 * 64;
    static constexpr int64_t W3 = (int64_t)T3 * T2 * 2 * 64;
    static constexpr int64_t wunits = W1 + W2 + W3;
};

// accumulator tile (fp32, after bias+ReLU) -> two bf16x8 K-fragments
__device__ __forceinline__ void to_frag(const f32x16 &y, bf16x8 &f0, bf16x8 &f1)
{
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        f0[j] = (__bf16)y[j];
        f1[j] = (__bf16)y[8 + j];
    }
}

template <int CF, int C1, int C2, int C3, int NS>
__global__ __launch_bounds__(256) void sa_group_mlp_bf16_kernel(
    const float *__restrict__ xyz, const float *__restrict__ feats, int64_t feat_stride,
    const float *__restrict__ centres, const int32_t *__restrict__ idx, int n, int m, int64_t total,
    int64_t units, const bf16x8 *__restrict__ packed, float *__restrict__ out, int64_t out_stride,
    int64_t out_offset)
{
    using S = Shape16<CF, C1, C2, C3>;
    constexpr int TILES = NS >= 32 ? NS / 32 : 1;
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5, col = lane & 31;
    const int64_t unit = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (unit >= units) return;  // wave-uniform

    float mx[S::T3];
#pragma unroll
    for (int t = 0; t < S::T3; ++t) mx[t] = 0.0f;

#pragma unroll 1
    for (int tile = 0; tile < TILES; ++tile) {
        const bf16x8 *pk = packed;
        asm volatile("" : "+s"(pk));  // keep the loop-invariant weight loads inside the loop
        const bf16x8 *W1 = pk, *W2 = W1 + S::W1, *W3 = W2 + S::W2;
        const float *B1 = reinterpret_cast<const float *>(W3 + S::W3);
        const float *B2 = B1 + C1, *B3 = B2 + C2;

        int64_t c;
        int s;
        if constexpr (NS >= 32) {
            c = unit;
            s = tile * 32 + col;
        } else {
            c = unit * 2 + (col >> 4);
            s = col & 15;
        }
        const int64_t cc = c < total ? c : total - 1;
        const int64_t b = cc / m;
        const int64_t k = idx[cc * NS + s];
        const float *pr = xyz + (b * n + k) * 3;
        const float *ce = centres + cc * 3;
        const float d3[3] = {pr[0] - ce[0], pr[1] - ce[1], pr[2] - ce[2]};

        // ---- layer-1 B fragments: step s2, half h = physical channels [16 s2 + 8h, +8)
        bf16x8 x1[S::S1];
        const float *fr = feats + (b * n + k) * feat_stride;
#pragma unroll
        for (int s2 = 0; s2 < S::S1; ++s2) {
            const int p0 = 16 * s2 + 8 * h;  // runtime in h only
            bf16x8 v;
            if (16 * s2 + 16 <= CF) {  // whole step inside the features (wave-uniform)
                const f32x4 a = *reinterpret_cast<const f32x4 *>(fr + p0);
                const f32x4 bq = *reinterpret_cast<const f32x4 *>(fr + p0 + 4);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    v[j] = (__bf16)a[j];
                    v[4 + j] = (__bf16)bq[j];
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int ch = p0 + j;
                    float f = 0.0f;
                    if (ch < CF) f = fr[ch];
                    else if (ch < CF + 3) f = d3[ch - CF];
                    v[j] = (__bf16)f;
                }
            }
            x1[s2] = v;
        }

        // ---- layer 1 (channel rows x point columns)
        bf16x8 y1[S::T1][2];
#pragma unroll
        for (int t = 0; t < S::T1; ++t) {
            f32x16 acc = {};
            const bf16x8 *w = W1 + (int64_t)t * S::S1 * 64 + lane;
#pragma unroll
            for (int s2 = 0; s2 < S::S1; ++s2) acc = mfma16(w[s2 * 64], x1[s2], acc);
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = relu(acc[r] + B1[32 * t + rho(r) + 4 * h]);
            to_frag(acc, y1[t][0], y1[t][1]);
        }
        // ---- layer 2
        bf16x8 y2[S::T2][2];
#pragma unroll
        for (int t = 0; t < S::T2; ++t) {
            f32x16 acc = {};
            const bf16x8 *w = W2 + (int64_t)t * S::T1 * 2 * 64 + lane;
#pragma unroll
            for (int ti = 0; ti < S::T1; ++ti)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) acc = mfma16(w[(ti * 2 + s2) * 64], y1[ti][s2], acc);
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = relu(acc[r] + B2[32 * t + rho(r) + 4 * h]);
            to_frag(acc, y2[t][0], y2[t][1]);
        }
        // ---- layer 3, transposed (point rows x channel columns) + max over points
#pragma unroll
        for (int t = 0; t < S::T3; ++t) {
            f32x16 acc = {};
            const bf16x8 *w = W3 + (int64_t)t * S::T2 * 2 * 64 + lane;
#pragma unroll
            for (int ti = 0; ti < S::T2; ++ti)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) acc = mfma16(y2[ti][s2], w[(ti * 2 + s2) * 64], acc);
            const float bias = B3[32 * t + col];
            if constexpr (NS >= 32) {
                float v = 0.0f;
#pragma unroll
                for (int r = 0; r < 16; ++r) v = fmaxf(v, relu(acc[r] + bias));
                v = fmaxf(v, __shfl_xor(v, 32, 64));
                mx[t] = fmaxf(mx[t], v);
            } else {
                float va = 0.0f, vb = 0.0f;
#pragma unroll
                for (int r = 0; r < 8; ++r) va = fmaxf(va, relu(acc[r] + bias));
#pragma unroll
                for (int r = 8; r < 16; ++r) vb = fmaxf(vb, relu(acc[r] + bias));
                va = fmaxf(va, __shfl_xor(va, 32, 64));
                vb = fmaxf(vb, __shfl_xor(vb, 32, 64));
                mx[t] = h ? vb : va;
            }
        }
    }
    if constexpr (NS >= 32) {
        if (h == 0) {
            float *o = out + unit * out_stride + out_offset;
#pragma unroll
            for (int t = 0; t < S::T3; ++t) o[32 * t + col] = mx[t];
        }
    } else {
        const int64_t c = unit * 2 + h;
        if (c < total) {
            float *o = out + c * out_stride + out_offset;
#pragma unroll
            for (int t = 0; t < S::T3; ++t) o[32 * t + col] = mx[t];
        }
    }
}

typedef int (*launch16_fn)(const float *, const float *, int64_t, const float *, const int32_t *, int64_t,
                           int64_t, int64_t, const void *, float *, int64_t, int64_t, hipStream_t);

template <int CF, int C1, int C2, int C3, int NS>
int launch16(const float *xyz, const float *feats, int64_t fs, const float *centres, const int32_t *idx,
             int64_t batch, int64_t n, int64_t m, const void *packed, float *out, int64_t os, int64_t oo,
             hipStream_t s)
{
    const int64_t total = batch * m;
    const int64_t units = NS >= 32 ? total : (total + 1) / 2;
    const int64_t blocks = (units + 3) / 4;
    REQUIRE(blocks <= 0x7fffffff, "sa_group_mlp_bf16: too many centres");
    hipLaunchKernelGGL((sa_group_mlp_bf16_kernel<CF, C1, C2, C3, NS>), dim3((unsigned)blocks), dim3(256), 0, s,
                       xyz, feats, fs, centres, idx, (int)n, (int)m, total, units,
                       static_cast<const bf16x8 *>(packed), out, os, oo);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

struct Variant16 {
    int cf, c1, c2, c3, ns;
    launch16_fn fn;
};

// MSG SA1 / SA2 branches (configs[4]) plus the SSG levels in bf16
const Variant16 kVariants16[] = {
    {0, 32, 32, 64, 16, launch16<0, 32, 32, 64, 16>},
    {0, 64, 64, 128, 32, launch16<0, 64, 64, 128, 32>},
    {0, 64, 96, 128, 128, launch16<0, 64, 96, 128, 128>},
    {320, 64, 64, 128, 32, launch16<320, 64, 64, 128, 32>},
    {320, 128, 128, 256, 64, launch16<320, 128, 128, 256, 64>},
    {320, 128, 128, 256, 128, launch16<320, 128, 128, 256, 128>},
    {128, 128, 128, 256, 64, launch16<128, 128, 128, 256, 64>},
};

uint16_t bf16_bits(float f)
{
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

}  // namespace

LIDAR_EXPORT int64_t lidar_mlp_packed_size_bf16(int32_t cf, int32_t c1, int32_t c2, int32_t c3)
{
    // bytes: bf16x8 weight fragments + fp32 biases
    const int64_t k1 = ((int64_t)cf + 3 + 15) / 16 * 16;
    const int64_t units = (c1 / 32) * (k1 / 16) * 64 + (int64_t)(c2 / 32) * (c1 / 32) * 2 * 64 +
                          (int64_t)(c3 / 32) * (c2 / 32) * 2 * 64;
    return units * 16 + 4 * ((int64_t)c1 + c2 + c3);
}

LIDAR_EXPORT int lidar_mlp_pack_bf16(int32_t cf, int32_t c1, int32_t c2, int32_t c3, const float *w1,
                                     const float *b1, const float *w2, const float *b2, const float *w3,
                                     const float *b3, void *packed)
{
    REQUIRE(w1 && b1 && w2 && b2 && w3 && b3 && packed, "lidar_mlp_pack_bf16: null pointer");
    REQUIRE(cf >= 0 && cf % 16 == 0, "lidar_mlp_pack_bf16: cfeat must be a multiple of 16");
    REQUIRE(c1 % 32 == 0 && c2 % 32 == 0 && c3 % 32 == 0 && c1 > 0 && c2 > 0 && c3 > 0,
            "lidar_mlp_pack_bf16: widths must be positive multiples of 32");
    const int k1 = (cf + 3 + 15) / 16 * 16, s1 = k1 / 16;
    uint16_t *o = static_cast<uint16_t *>(packed);
    // layer 1: physical channel P = 16 s + 8 h + j -> canonical row (features after dx,dy,dz)
    for (int t = 0; t < c1 / 32; ++t)
        for (int s = 0; s < s1; ++s)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 8; ++j) {
                    const int P = 16 * s + 8 * (l >> 5) + j;
                    const int row = P < cf ? 3 + P : (P < cf + 3 ? P - cf : -1);
                    const float v = row >= 0 ? w1[(int64_t)row * c1 + 32 * t + (l & 31)] : 0.0f;
                    o[((((int64_t)t * s1 + s) * 64) + l) * 8 + j] = bf16_bits(v);
                }
    o += (int64_t)(c1 / 32) * s1 * 64 * 8;
    auto hidden = [&](const float *w, int cin, int cout) {
        const int tin = cin / 32;
        for (int t = 0; t < cout / 32; ++t)
            for (int ti = 0; ti < tin; ++ti)
                for (int s = 0; s < 2; ++s)
                    for (int l = 0; l < 64; ++l)
                        for (int j = 0; j < 8; ++j) {
                            const int kk = 32 * ti + 16 * s + 8 * (j >> 2) + 4 * (l >> 5) + (j & 3);
                            o[((((int64_t)t * tin + ti) * 2 + s) * 64 + l) * 8 + j] =
                                bf16_bits(w[(int64_t)kk * cout + 32 * t + (l & 31)]);
                        }
        o += (int64_t)(cout / 32) * tin * 2 * 64 * 8;
    };
    hidden(w2, c1, c2);
    hidden(w3, c2, c3);
    float *bo = reinterpret_cast<float *>(o);
    for (int i = 0; i < c1; ++i) *bo++ = b1[i];
    for (int i = 0; i < c2; ++i) *bo++ = b2[i];
    for (int i = 0; i < c3; ++i) *bo++ = b3[i];
    return LIDAR_OK;
}

LIDAR_EXPORT int lidar_sa_group_mlp_bf16(lidar_handle *h, const float *xyz, const float *feats,
                                         int64_t feat_stride, const float *centres, const int32_t *idx,
                                         int64_t batch, int64_t n, int64_t m, int32_t nsample, int32_t cfeat,
                                         int32_t c1, int32_t c2, int32_t c3, const void *packed, float *out,
                                         int64_t out_stride, int64_t out_offset, void *stream)
{
    REQUIRE(h && xyz && centres && idx && packed && out, "lidar_sa_group_mlp_bf16: null pointer");
    REQUIRE(cfeat == 0 || feats, "lidar_sa_group_mlp_bf16: feats is NULL");
    REQUIRE(batch >= 0 && n >= 1 && m >= 1, "lidar_sa_group_mlp_bf16: bad sizes");
    REQUIRE(cfeat == 0 || (feat_stride >= cfeat && feat_stride % 4 == 0),
            "lidar_sa_group_mlp_bf16: feat_stride must be >= cfeat and a multiple of 4");
    REQUIRE(out_offset >= 0 && out_offset + c3 <= out_stride,
            "lidar_sa_group_mlp_bf16: output columns exceed out_stride");
    if (batch == 0) return LIDAR_OK;
    HIP_TRY(hipSetDevice(h->device));
    for (const Variant16 &v : kVariants16)
        if (v.cf == cfeat && v.c1 == c1 && v.c2 == c2 && v.c3 == c3 && v.ns == nsample)
            return v.fn(xyz, feats, feat_stride, centres, idx, batch, n, m, packed, out, out_stride, out_offset,
                        static_cast<hipStream_t>(stream));
    return lidar::fail(LIDAR_EINVAL, "lidar_sa_group_mlp_bf16: unsupported (cfeat, widths, nsample) combination");
}
