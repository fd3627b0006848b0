// sa_mlp.hip — the SetAbstraction shared MLP on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// (1) sa_group_mlp_kernel: grouping gather + 3 layers (+bias, ReLU) + max-pool over the
//     nsample axis, fully fused: a wavefront owns 32 grouped rows (the 32 MFMA columns)
//     and chains the layers in registers.  Layer l's 32x32 accumulator tile holds
//     (channel row, point column); `acc reg r, lane half h` is channel rho(r)+4h, so it is
//     directly the K-operand of the next MFMA (the k order inside a 2-wide step is
//     absorbed into the packed weight image — no LDS, no transposes).  The last layer is
//     computed transposed (point rows, channel columns) so the max over points is a max
//     over the 16 registers plus one xor-32 swap.  Nothing but the pooled (M, C3) output
//     ever reaches HBM; the (M*nsample, C) intermediates of the reference formulation
//     are never materialised.
// (2) dense_relu_kernel: LDS-tiled 128x128x16 MFMA GEMM with bias+ReLU epilogue and an
//     optional fused row-group max-pool (group_all's SA3), for layers too wide to keep
//     in registers.
#include <cstdlib>
#include <vector>

#include "common.hpp"

// LDS-staged weight-stream kernels (sa_mlp_pre.hip); -1 = no variant for these widths
int lidar_sa_xyz_lds_dispatch(int c1, int c2, int c3, int ns, const float *xyz, const float *centres,
                              const int32_t *idx, int64_t batch, int64_t n, int64_t m, const float *packed,
                              float *out, int64_t os, int64_t oo, hipStream_t s);
int lidar_sa_pre_lds_dispatch(int cfeat, int c1, int c2, int c3, int ns, const float *p, int64_t stride,
                              const float *q, const int32_t *idx, int64_t batch, int64_t n, int64_t m,
                              const float *w23, float *out, int64_t os, int64_t oo, hipStream_t s);

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int rho(int r) { return (r & 3) + 8 * (r >> 2); }

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c)
{
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }

template <int CF, int C1, int C2, int C3>
struct MlpShape {
    static constexpr int S1 = CF / 2 + 2;              // layer-1 MFMA k-steps (K = CF + 4)
    static constexpr int S1P = (S1 + 3) / 4 * 4;       // padded to float4 weight loads
    static constexpr int T1 = C1 / 32, T2 = C2 / 32, T3 = C3 / 32;
    static constexpr int S2 = C1 / 2, S3 = C2 / 2;
    static constexpr int64_t W1 = (int64_t)T1 * S1P * 64;
    static constexpr int64_t W2 = (int64_t)T2 * S2 * 64;
    static constexpr int64_t W3 = (int64_t)T3 * S3 * 64;
    static constexpr int64_t size = W1 + W2 + W3 + C1 + C2 + C3;
};

// PRE: layer 1 was applied per POINT before grouping (P = [f, x] W1 + b1 over the level's
// N points, Q = c W1_xyz over its M centres, both plain GEMMs, dense_kernel below), so
// layer 1 of a grouped row is relu(P[k] - Q[c]) = relu(W1^T [x_k - c, f_k] + b1): 16x fewer
// layer-1 rows (N vs M*nsample) for the cost of one fp32 re-association.  `feats` is P and
// `centres` is Q (both with row stride feat_stride) and `packed` points at the layer-2 weights.
template <int CF, int C1, int C2, int C3, int NS, bool PRE = false>
__global__ __launch_bounds__(256) void sa_group_mlp_kernel(
    const float *__restrict__ xyz, const float *__restrict__ feats, int64_t feat_stride,
    const float *__restrict__ centres, const int32_t *__restrict__ idx, int n, int m,
    int64_t total, int64_t units, const float *__restrict__ packed, float *__restrict__ out,
    int64_t out_stride, int64_t out_offset)
{
    using S = MlpShape<CF, C1, C2, C3>;
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
        int64_t c;
        int s;
        if constexpr (NS >= 32) {
            c = unit;
            s = tile * 32 + col;
        } else {
            c = unit * 2 + (col >> 4);
            s = col & 15;
        }
        // the weights are loop-invariant: launder the pointer each tile so LLVM cannot hoist
        // (and keep in registers) every weight load of the whole chain
        const float *pk = packed;
        asm volatile("" : "+s"(pk));
        const float *W1 = pk;
        const float *W2 = PRE ? pk : W1 + S::W1;
        const float *W3 = W2 + S::W2;
        const float *B1 = W3 + S::W3;
        const float *B2 = B1 + C1;
        const float *B3 = B2 + C2;
        const int64_t cc = c < total ? c : total - 1;
        const int64_t b = cc / m;
        const int64_t k = idx[cc * NS + s];
        f32x16 y1[S::T1];
        if constexpr (PRE) {
            // y1[ti] reg 4j+i <- channel 32 ti + 8 j + 4 h + i of relu(P[k] - Q[c])
            const f32x4 *pp = reinterpret_cast<const f32x4 *>(feats + (b * n + k) * feat_stride + 4 * h);
            const f32x4 *qq = reinterpret_cast<const f32x4 *>(centres + cc * feat_stride + 4 * h);
#pragma unroll
            for (int ti = 0; ti < S::T1; ++ti)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x4 a = pp[8 * ti + 2 * j], q = qq[8 * ti + 2 * j];
#pragma unroll
                    for (int i = 0; i < 4; ++i) y1[ti][4 * j + i] = relu(a[i] - q[i]);
                }
        } else {
        const float *pr = xyz + (b * n + k) * 3;
        const float *ce = centres + cc * 3;
        const float dx = pr[0] - ce[0], dy = pr[1] - ce[1], dz = pr[2] - ce[2];

        // ---- layer-1 B operand: lane half h supplies features [h*CF/2, (h+1)*CF/2) and
        // (dx, dy) | (dz, 0)
        float x1[S::S1P];
        if constexpr (CF > 0) {
            const f32x4 *fr = reinterpret_cast<const f32x4 *>(feats + (b * n + k) * feat_stride + h * (CF / 2));
#pragma unroll
            for (int q = 0; q < CF / 8; ++q) {
                f32x4 v = fr[q];
                x1[4 * q] = v[0];
                x1[4 * q + 1] = v[1];
                x1[4 * q + 2] = v[2];
                x1[4 * q + 3] = v[3];
            }
        }
        x1[CF / 2] = h ? dz : dx;
        x1[CF / 2 + 1] = h ? 0.0f : dy;
#pragma unroll
        for (int q = CF / 2 + 2; q < S::S1P; ++q) x1[q] = 0.0f;

        // ---- layer 1 (channel rows x point columns)
#pragma unroll
        for (int t = 0; t < S::T1; ++t) {
            __builtin_amdgcn_sched_barrier(0);
            f32x16 acc = {};
            const f32x4 *w = reinterpret_cast<const f32x4 *>(W1) + (int64_t)t * (S::S1P / 4) * 64 + lane;
#pragma unroll
            for (int s4 = 0; s4 < S::S1P / 4; ++s4) {
                f32x4 wv = w[s4 * 64];
#pragma unroll
                for (int i = 0; i < 4; ++i) acc = mfma(wv[i], x1[4 * s4 + i], acc);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = relu(acc[r] + B1[32 * t + rho(r) + 4 * h]);
            y1[t] = acc;
        }
        }  // !PRE
        // ---- layer 2 (channel rows x point columns); y1 registers are the K operand
        f32x16 y2[S::T2];
#pragma unroll
        for (int t = 0; t < S::T2; ++t) {
            __builtin_amdgcn_sched_barrier(0);
            f32x16 acc = {};
            const f32x4 *w = reinterpret_cast<const f32x4 *>(W2) + (int64_t)t * (S::S2 / 4) * 64 + lane;
#pragma unroll
            for (int ti = 0; ti < S::T1; ++ti) {
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4) {
                    f32x4 wv = w[(ti * 4 + r4) * 64];
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc = mfma(wv[i], y1[ti][4 * r4 + i], acc);
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = relu(acc[r] + B2[32 * t + rho(r) + 4 * h]);
            y2[t] = acc;
        }
        // ---- layer 3, transposed (point rows x channel columns) + max over points
#pragma unroll
        for (int t = 0; t < S::T3; ++t) {
            __builtin_amdgcn_sched_barrier(0);
            f32x16 acc = {};
            const f32x4 *w = reinterpret_cast<const f32x4 *>(W3) + (int64_t)t * (S::S3 / 4) * 64 + lane;
#pragma unroll
            for (int ti = 0; ti < S::T2; ++ti) {
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4) {
                    f32x4 wv = w[(ti * 4 + r4) * 64];
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc = mfma(y2[ti][4 * r4 + i], wv[i], acc);
                }
            }
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

// ------------------------------------------------------------------ dense GEMM
constexpr int BM = 128, BN = 128, BK = 16;

__global__ __launch_bounds__(256) void dense_relu_kernel(const float *__restrict__ x, int K,
                                                         const float *__restrict__ w,
                                                         const float *__restrict__ bias,
                                                         int cout, int pool_rows,
                                                         float *__restrict__ y, int act)
{
    __shared__ float As[BK][BM];
    __shared__ float Bs[BK][BN];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int wm = wave >> 1, wn = wave & 1;
    const int64_t row0 = (int64_t)blockIdx.y * BM;
    const int col0 = blockIdx.x * BN;
    f32x16 acc[2][2] = {};

    const int ar = tid & 127, akq = tid >> 7;  // A: row, k-quad (0..1, and +2)
    const int bk = tid >> 5, bc = (tid & 31) * 4;  // B: k row (0..7, and +8), 4 columns
    for (int k0 = 0; k0 < K; k0 += BK) {
        const float *xa = x + (row0 + ar) * K + k0;
        f32x4 a0 = *reinterpret_cast<const f32x4 *>(xa + akq * 4);
        f32x4 a1 = *reinterpret_cast<const f32x4 *>(xa + (akq + 2) * 4);
        f32x4 b0 = *reinterpret_cast<const f32x4 *>(w + (int64_t)(k0 + bk) * cout + col0 + bc);
        f32x4 b1 = *reinterpret_cast<const f32x4 *>(w + (int64_t)(k0 + bk + 8) * cout + col0 + bc);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            As[akq * 4 + i][ar] = a0[i];
            As[(akq + 2) * 4 + i][ar] = a1[i];
        }
        *reinterpret_cast<f32x4 *>(&Bs[bk][bc]) = b0;
        *reinterpret_cast<f32x4 *>(&Bs[bk + 8][bc]) = b1;
        __syncthreads();
#pragma unroll
        for (int s = 0; s < BK / 2; ++s) {
            float a[2], bv[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = As[2 * s + h][wm * 64 + i * 32 + col];
#pragma unroll
            for (int j = 0; j < 2; ++j) bv[j] = Bs[2 * s + h][wn * 64 + j * 32 + col];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = mfma(a[i], bv[j], acc[i][j]);
        }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int c = col0 + wn * 64 + j * 32 + col;
        const float bb = bias[c];
        if (pool_rows == 0) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t row = row0 + wm * 64 + i * 32 + rho(r) + 4 * h;
                    const float v = acc[i][j][r] + bb;
                    y[row * cout + c] = act ? relu(v) : v;
                }
        } else {
            float v = 0.0f;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) v = fmaxf(v, relu(acc[i][j][r] + bb));
            v = fmaxf(v, __shfl_xor(v, 32, 64));
            if (h == 0) {
                // non-negative floats order as their bit patterns: an unsigned max is exact
                // and order-independent (deterministic)
                unsigned *dst = reinterpret_cast<unsigned *>(y + (row0 / pool_rows) * cout + c);
                atomicMax(dst, __float_as_uint(v));
            }
        }
    }
}

__global__ void concat_xyz_pad_kernel(const float *__restrict__ xyz, int64_t rows,
                                      float *__restrict__ y, int64_t ldy, int64_t col0)
{
    const int64_t width = ldy - col0;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * width) return;
    const int64_t r = i / width, cidx = i % width;
    y[r * ldy + col0 + cidx] = cidx < 3 ? xyz[r * 3 + cidx] : 0.0f;
}

// ------------------------------------------------------------------ dispatch
typedef int (*launch_fn)(const float *, const float *, int64_t, const float *, const int32_t *,
                         int64_t, int64_t, int64_t, const float *, float *, int64_t, int64_t,
                         hipStream_t);

template <int CF, int C1, int C2, int C3, int NS, bool PRE = false>
int launch_sa(const float *xyz, const float *feats, int64_t fs, const float *centres,
              const int32_t *idx, int64_t batch, int64_t n, int64_t m, const float *packed,
              float *out, int64_t os, int64_t oo, hipStream_t s)
{
    const int64_t total = batch * m;
    const int64_t units = NS >= 32 ? total : (total + 1) / 2;
    const int64_t blocks = (units + 3) / 4;
    REQUIRE(blocks <= 0x7fffffff, "sa_group_mlp: too many centres");
    hipLaunchKernelGGL((sa_group_mlp_kernel<CF, C1, C2, C3, NS, PRE>), dim3((unsigned)blocks), dim3(256), 0,
                       s, xyz, feats, fs, centres, idx, (int)n, (int)m, total, units, packed, out,
                       os, oo);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

struct Variant {
    int cf, c1, c2, c3, ns;
    launch_fn fn;
};

// the SetAbstraction branches of the BASELINE.json configs:
// SSG SA1/SA2, MSG SA1 (3 radii) and MSG SA2 (3 radii)
const Variant kVariants[] = {
    {0, 64, 64, 128, 32, launch_sa<0, 64, 64, 128, 32>},
    {128, 128, 128, 256, 64, launch_sa<128, 128, 128, 256, 64>},
    {0, 32, 32, 64, 16, launch_sa<0, 32, 32, 64, 16>},
    {0, 64, 96, 128, 128, launch_sa<0, 64, 96, 128, 128>},
    {320, 64, 64, 128, 32, launch_sa<320, 64, 64, 128, 32>},
    {320, 128, 128, 256, 64, launch_sa<320, 128, 128, 256, 64>},
    {320, 128, 128, 256, 128, launch_sa<320, 128, 128, 256, 128>},
};

// layer-1-per-point twins of the branches with point features (cf > 0)
const Variant kPreVariants[] = {
    {128, 128, 128, 256, 64, launch_sa<128, 128, 128, 256, 64, true>},
    {320, 64, 64, 128, 32, launch_sa<320, 64, 64, 128, 32, true>},
    {320, 128, 128, 256, 64, launch_sa<320, 128, 128, 256, 64, true>},
    {320, 128, 128, 256, 128, launch_sa<320, 128, 128, 256, 128, true>},
};

int64_t packed_size(int cf, int c1, int c2, int c3)
{
    const int64_t s1p = ((int64_t)cf / 2 + 2 + 3) / 4 * 4;
    return (c1 / 32) * s1p * 64 + (int64_t)(c2 / 32) * (c1 / 2) * 64 +
           (int64_t)(c3 / 32) * (c2 / 2) * 64 + c1 + c2 + c3;
}

}  // namespace

LIDAR_EXPORT int64_t lidar_mlp_packed_size(int32_t cfeat, int32_t c1, int32_t c2, int32_t c3)
{
    return packed_size(cfeat, c1, c2, c3);
}

LIDAR_EXPORT int lidar_mlp_pack_f32(int32_t cf, int32_t c1, int32_t c2, int32_t c3,
                                    const float *w1, const float *b1, const float *w2,
                                    const float *b2, const float *w3, const float *b3,
                                    float *packed)
{
    REQUIRE(w1 && b1 && w2 && b2 && w3 && b3 && packed, "lidar_mlp_pack_f32: null pointer");
    REQUIRE(cf >= 0 && cf % 8 == 0, "lidar_mlp_pack_f32: cfeat must be a multiple of 8");
    REQUIRE(c1 % 32 == 0 && c2 % 32 == 0 && c3 % 32 == 0 && c1 > 0 && c2 > 0 && c3 > 0,
            "lidar_mlp_pack_f32: widths must be positive multiples of 32");
    const int s1p = (cf / 2 + 2 + 3) / 4 * 4;
    float *o = packed;
    // layer 1: rows of W1 (3 + cf, c1) in canonical order [dx, dy, dz, feat...]
    auto row1 = [&](int s, int h) -> int {
        if (s < cf / 2) return 3 + s + h * (cf / 2);
        if (s == cf / 2) return h ? 2 : 0;
        if (s == cf / 2 + 1) return h ? -1 : 1;
        return -1;
    };
    for (int t = 0; t < c1 / 32; ++t)
        for (int s = 0; s < s1p; ++s)
            for (int l = 0; l < 64; ++l) {
                const int r = row1(s, l >> 5);
                o[(((int64_t)t * (s1p / 4) + s / 4) * 64 + l) * 4 + s % 4] =
                    r >= 0 ? w1[(int64_t)r * c1 + 32 * t + (l & 31)] : 0.0f;
            }
    o += (int64_t)(c1 / 32) * s1p * 64;
    auto hidden = [&](const float *w, int cin, int cout) {
        const int steps = cin / 2;
        for (int t = 0; t < cout / 32; ++t)
            for (int s = 0; s < steps; ++s)
                for (int l = 0; l < 64; ++l) {
                    const int kk = 32 * (s / 16) + rho(s % 16) + 4 * (l >> 5);
                    o[(((int64_t)t * (steps / 4) + s / 4) * 64 + l) * 4 + s % 4] =
                        w[(int64_t)kk * cout + 32 * t + (l & 31)];
                }
        o += (int64_t)(cout / 32) * steps * 64;
    };
    hidden(w2, c1, c2);
    hidden(w3, c2, c3);
    for (int i = 0; i < c1; ++i) *o++ = b1[i];
    for (int i = 0; i < c2; ++i) *o++ = b2[i];
    for (int i = 0; i < c3; ++i) *o++ = b3[i];
    return LIDAR_OK;
}

LIDAR_EXPORT int lidar_sa_group_mlp_f32(lidar_handle *h, const float *xyz, const float *feats,
                                        int64_t feat_stride, const float *centres,
                                        const int32_t *idx, int64_t batch, int64_t n, int64_t m,
                                        int32_t nsample, int32_t cfeat, int32_t c1, int32_t c2,
                                        int32_t c3, const float *packed, float *out,
                                        int64_t out_stride, int64_t out_offset, void *stream)
{
    REQUIRE(h && xyz && centres && idx && packed && out, "lidar_sa_group_mlp_f32: null pointer");
    REQUIRE(cfeat == 0 || feats, "lidar_sa_group_mlp_f32: feats is NULL");
    REQUIRE(batch >= 0 && n >= 1 && m >= 1, "lidar_sa_group_mlp_f32: bad sizes");
    REQUIRE(cfeat == 0 || (feat_stride >= cfeat && feat_stride % 4 == 0),
            "lidar_sa_group_mlp_f32: feat_stride must be >= cfeat and a multiple of 4");
    REQUIRE(out_offset >= 0 && out_offset + c3 <= out_stride,
            "lidar_sa_group_mlp_f32: output columns exceed out_stride");
    if (batch == 0) return LIDAR_OK;
    HIP_TRY(hipSetDevice(h->device));
    static const bool no_lds = getenv("LIDAR_PRE_NO_LDS") != nullptr;  // A/B tuning knob
    if (cfeat == 0 && !no_lds) {  // LDS-staged weight stream (sa_mlp_pre.hip)
        const int rc = lidar_sa_xyz_lds_dispatch(c1, c2, c3, nsample, xyz, centres, idx, batch, n, m, packed,
                                                 out, out_stride, out_offset, static_cast<hipStream_t>(stream));
        if (rc != -1) return rc;
    }
    for (const Variant &v : kVariants)
        if (v.cf == cfeat && v.c1 == c1 && v.c2 == c2 && v.c3 == c3 && v.ns == nsample)
            return v.fn(xyz, feats, feat_stride, centres, idx, batch, n, m, packed, out,
                        out_stride, out_offset, static_cast<hipStream_t>(stream));
    return lidar::fail(LIDAR_EINVAL, "lidar_sa_group_mlp_f32: unsupported (cfeat, widths, nsample) "
                                     "combination — add a kVariants entry");
}

LIDAR_EXPORT int lidar_dense_f32(lidar_handle *h, const float *x, int64_t rows, int32_t k,
                                 const float *w, const float *bias, int32_t cout, int32_t relu_on,
                                 int32_t pool_rows, float *y, void *stream)
{
    REQUIRE(h && x && w && bias && y, "lidar_dense_f32: null pointer");
    REQUIRE(rows % BM == 0 && k % BK == 0 && cout % BN == 0 && k > 0,
            "lidar_dense_f32: rows % 128, k % 16, cout % 128 must be 0");
    REQUIRE(pool_rows == 0 || (pool_rows % BM == 0 && rows % pool_rows == 0),
            "lidar_dense_f32: pool_rows must be a multiple of 128 dividing rows");
    REQUIRE(pool_rows == 0 || relu_on, "lidar_dense_f32: the fused max-pool needs relu (>= 0 outputs)");
    if (rows == 0) return LIDAR_OK;
    REQUIRE(rows / BM <= 65535, "lidar_dense_f32: too many rows");
    HIP_TRY(hipSetDevice(h->device));
    hipLaunchKernelGGL(dense_relu_kernel, dim3(cout / BN, (unsigned)(rows / BM)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), x, (int)k, w, bias, (int)cout,
                       (int)pool_rows, y, relu_on ? 1 : 0);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

LIDAR_EXPORT int lidar_dense_relu_f32(lidar_handle *h, const float *x, int64_t rows, int32_t k,
                                      const float *w, const float *bias, int32_t cout,
                                      int32_t pool_rows, float *y, void *stream)
{
    return lidar_dense_f32(h, x, rows, k, w, bias, cout, 1, pool_rows, y, stream);
}


LIDAR_EXPORT int lidar_sa_group_mlp_pre_f32(lidar_handle *h, const float *p, int64_t p_stride,
                                            const float *q, const int32_t *idx, int64_t batch,
                                            int64_t n, int64_t m, int32_t nsample, int32_t cfeat,
                                            int32_t c1, int32_t c2, int32_t c3, const float *packed,
                                            float *out, int64_t out_stride, int64_t out_offset,
                                            void *stream)
{
    REQUIRE(h && p && q && idx && packed && out, "lidar_sa_group_mlp_pre_f32: null pointer");
    REQUIRE(batch >= 0 && n >= 1 && m >= 1, "lidar_sa_group_mlp_pre_f32: bad sizes");
    REQUIRE(p_stride >= c1 && p_stride % 4 == 0, "lidar_sa_group_mlp_pre_f32: p_stride must be >= c1, % 4");
    REQUIRE(out_offset >= 0 && out_offset + c3 <= out_stride,
            "lidar_sa_group_mlp_pre_f32: output columns exceed out_stride");
    if (batch == 0) return LIDAR_OK;
    HIP_TRY(hipSetDevice(h->device));
    // the packed image is lidar_mlp_pack_f32's: skip its layer-1 block
    const int64_t s1p = ((int64_t)cfeat / 2 + 2 + 3) / 4 * 4;
    const float *w2 = packed + (int64_t)(c1 / 32) * s1p * 64;
    static const bool no_lds = getenv("LIDAR_PRE_NO_LDS") != nullptr;  // A/B tuning knob
    if (!no_lds) {
        const int rc = lidar_sa_pre_lds_dispatch(cfeat, c1, c2, c3, nsample, p, p_stride, q, idx, batch, n,
                                                 m, w2, out, out_stride, out_offset,
                                                 static_cast<hipStream_t>(stream));
        if (rc != -1) return rc;
    }
    for (const Variant &v : kPreVariants)
        if (v.cf == cfeat && v.c1 == c1 && v.c2 == c2 && v.c3 == c3 && v.ns == nsample)
            return v.fn(nullptr, p, p_stride, q, idx, batch, n, m, w2, out, out_stride, out_offset,
                        static_cast<hipStream_t>(stream));
    return lidar::fail(LIDAR_EINVAL, "lidar_sa_group_mlp_pre_f32: unsupported (cfeat, widths, nsample)");
}

LIDAR_EXPORT int lidar_concat_xyz_pad_f32(lidar_handle *h, const float *xyz, int64_t rows,
                                          float *y, int64_t ldy, int64_t col0, void *stream)
{
    REQUIRE(h && xyz && y, "lidar_concat_xyz_pad_f32: null pointer");
    REQUIRE(col0 >= 0 && col0 + 3 <= ldy, "lidar_concat_xyz_pad_f32: bad columns");
    if (rows == 0) return LIDAR_OK;
    HIP_TRY(hipSetDevice(h->device));
    const int64_t total = rows * (ldy - col0);
    hipLaunchKernelGGL(concat_xyz_pad_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), xyz, rows, y, ldy, col0);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
