// sa_mlp_pre.hip — SetAbstraction layers 2-3 + max-pool from per-point layer 1 (fp32 MFMA),
// with the weight stream staged through LDS.
//
// Layer 1 of a grouped row is relu(P[k] - Q[c]) (P, Q: per-point / per-centre GEMMs,
// sa_mlp.hip).  The MFMA chain is the one of sa_group_mlp_kernel (accumulator tiles are
// the next layer's K operand, the last layer transposed so the pool is a register max);
// what changes is where the weights come from.  A layer's weights are consumed in chunks
// of one 32-channel output tile (C_in/2 MFMA k-steps x 64 lanes x 4 B = 16 KiB for
// 128-wide layers).  The 4 waves of a workgroup run the same chunk sequence in lockstep:
// chunk c+1 is copied L2 -> LDS by global_load_lds (no VGPRs) while chunk c is read from
// the other LDS buffer by all 4 waves; one barrier per chunk.  L2 weight traffic drops 4x against per-wave streaming and no MFMA chain starts
// on an L2 round trip.
#include "common.hpp"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int rho(int r) { return (r & 3) + 8 * (r >> 2); }

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c)
{
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }

// XYZ = true: a level without point features (SA1): layer 1 runs here on the grouped
// offsets (dx, dy | dz, 0) as in sa_group_mlp_kernel (W1 and b1 resident in LDS; the two
// all-zero k-steps of its 4-step block are skipped, which changes no bit); P is xyz, Q is
// the centres and w23 is the whole lidar_mlp_pack_f32 image.
template <int C1, int C2, int C3, int NS, bool XYZ = false>
__global__ __launch_bounds__(256, 2) void sa_pre_lds_kernel(
    const float *__restrict__ P, int64_t stride, const float *__restrict__ Q,
    const int32_t *__restrict__ idx, int n, int m, int64_t total, const float *__restrict__ w23,
    float *__restrict__ out, int64_t out_stride, int64_t out_offset)
{
    static_assert(NS >= 32 && NS % 32 == 0, "one centre per wave, 32-row tiles");
    constexpr int T1 = C1 / 32, T2 = C2 / 32, T3 = C3 / 32;
    constexpr int S2 = C1 / 2, S3 = C2 / 2;            // MFMA k-steps per output tile
    constexpr int CH2 = S2 * 64 / 4, CH3 = S3 * 64 / 4;  // chunk sizes in float4
    constexpr int CHMAX = CH2 > CH3 ? CH2 : CH3;
    constexpr int NCH = T2 + T3;  // chunks per row tile
    constexpr int TILES = NS / 32;
    constexpr int PER = (CHMAX + 255) / 256;  // float4 per thread per chunk
    static_assert(CH2 % 256 == 0 && CH3 % 256 == 0, "chunks split evenly over 256 threads");

    __shared__ f32x4 buf[2][CHMAX];
    __shared__ float bias_s[C2 + C3];  // b2 | b3: no ordinary global load inside the chunk loop
    constexpr int W1N = XYZ ? T1 * 64 : 1;  // layer-1 weights (4 k-steps x 64 lanes per tile)
    __shared__ f32x4 w1_s[W1N];
    __shared__ float b1_s[XYZ ? C1 : 1];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int64_t unit = (int64_t)blockIdx.x * 4 + wave;
    const bool live = unit < total;        // every wave takes part in the barriers
    const int64_t cc = live ? unit : total - 1;
    const int64_t b = cc / m;

    const f32x4 *W2 = reinterpret_cast<const f32x4 *>(w23) + (XYZ ? T1 * 64 : 0);
    const f32x4 *W3 = W2 + (int64_t)T2 * CH2;
    const float *B2 = reinterpret_cast<const float *>(W3 + (int64_t)T3 * CH3) + C1;  // skip b1

    auto chunk_src = [&](int c) -> const f32x4 * { return c < T2 ? W2 + c * CH2 : W3 + (c - T2) * CH3; };
    auto chunk_len = [&](int c) -> int { return c < T2 ? CH2 : CH3; };

    // direct global -> LDS copy of a chunk (global_load_lds_dwordx4: each wave-instruction
    // writes 1 KiB at a wave-uniform LDS base + lane * 16; no VGPR staging)
    auto fetch = [&](int c, int dst) {
        const f32x4 *src = chunk_src(c);
        asm volatile("" : "+s"(src));  // keep each chunk's loads in their own iteration
        const int len = chunk_len(c);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int base = 256 * i + 64 * wave;
            if (base < len)
                __builtin_amdgcn_global_load_lds(
                    (__attribute__((address_space(1))) void *)(src + base + lane),
                    (__attribute__((address_space(3))) void *)(&buf[dst][base]), 16, 0, 0);
        }
    };
    fetch(0, 0);
    for (int i = tid; i < C2 + C3; i += 256) bias_s[i] = B2[i];  // B3 follows B2
    if constexpr (XYZ) {
        const f32x4 *W1 = reinterpret_cast<const f32x4 *>(w23);
        for (int i = tid; i < W1N; i += 256) w1_s[i] = W1[i];
        for (int i = tid; i < C1; i += 256) b1_s[i] = B2[i - C1];
    }
    __syncthreads();

    float mx[T3];
#pragma unroll
    for (int t = 0; t < T3; ++t) mx[t] = 0.0f;
    int par = 0;  // LDS buffer holding the current chunk

#pragma unroll 1
    for (int tile = 0; tile < TILES; ++tile) {
        // ---- layer 1 from the per-point rows: y1[ti] reg 4j+i <- channel 32ti+8j+4h+i
        const int64_t k = idx[cc * NS + tile * 32 + col];
        f32x16 y1[T1];
        if constexpr (XYZ) {
            const float *pr = P + ((int64_t)b * n + k) * 3;
            const float *ce = Q + cc * 3;
            const float dx = pr[0] - ce[0], dy = pr[1] - ce[1], dz = pr[2] - ce[2];
            const float xa = h ? dz : dx, xb = h ? 0.0f : dy;
#pragma unroll
            for (int t = 0; t < T1; ++t) {
                const f32x4 wv = w1_s[t * 64 + lane];
                f32x16 acc = {};
                acc = mfma(wv[0], xa, acc);
                acc = mfma(wv[1], xb, acc);
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = relu(acc[r] + b1_s[32 * t + rho(r) + 4 * h]);
                y1[t] = acc;
            }
        } else {
            const f32x4 *pp = reinterpret_cast<const f32x4 *>(P + ((int64_t)b * n + k) * stride + 4 * h);
            const f32x4 *qq = reinterpret_cast<const f32x4 *>(Q + cc * stride + 4 * h);
#pragma unroll
            for (int ti = 0; ti < T1; ++ti)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x4 a = pp[8 * ti + 2 * j], q = qq[8 * ti + 2 * j];
#pragma unroll
                    for (int i = 0; i < 4; ++i) y1[ti][4 * j + i] = relu(a[i] - q[i]);
                }
        }

        f32x16 y2[T2];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            // fetch the next chunk (the next tile's chunk 0 after the last one)
            const int cn = c + 1 < NCH ? c + 1 : 0;
            const bool more = c + 1 < NCH || tile + 1 < TILES;
            if (more) fetch(cn, par ^ 1);  // lands during this chunk's MFMAs
            const f32x4 *wb = buf[par] + lane;
            f32x16 acc = {};
            // operand reads written one 16-MFMA group ahead (LDS latency hidden behind 1024
            // MFMA cycles); the final order is left to the scheduler — pinning it with
            // sched_barriers measured 5 % slower (1.89 vs 1.79 ms, SA2 B=32)
            const int G = c < T2 ? T1 : T2;  // 16-MFMA groups in this chunk
            constexpr int GMAX = T1 > T2 ? T1 : T2;
            f32x4 wr[2][4];
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) wr[0][r4] = wb[r4 * 64];
#pragma unroll
            for (int ti = 0; ti < GMAX; ++ti) {
                if (ti >= G) break;
                if (ti + 1 < G) {
#pragma unroll
                    for (int r4 = 0; r4 < 4; ++r4) wr[(ti + 1) & 1][r4] = wb[((ti + 1) * 4 + r4) * 64];
                }
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if (c < T2)
                            acc = mfma(wr[ti & 1][r4][i], y1[ti < T1 ? ti : 0][4 * r4 + i], acc);
                        else
                            acc = mfma(y2[ti < T2 ? ti : 0][4 * r4 + i], wr[ti & 1][r4][i], acc);
                    }
            }
            if (c < T2) {  // layer 2, output tile c (channel rows x point columns)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = relu(acc[r] + bias_s[32 * c + rho(r) + 4 * h]);
                y2[c < T2 ? c : 0] = acc;
            } else {  // layer 3, output tile c - T2 (transposed) + max over the 32 rows
                const int t = c - T2;
                const float bias = bias_s[C2 + 32 * t + col];
                float v = 0.0f;
#pragma unroll
                for (int r = 0; r < 16; ++r) v = fmaxf(v, relu(acc[r] + bias));
                v = fmaxf(v, __shfl_xor(v, 32, 64));
                mx[t < T3 ? t : 0] = fmaxf(mx[t < T3 ? t : 0], v);
            }
            __syncthreads();  // (vmcnt(0)) chunk c+1 landed for everyone; buf[par] free for c+2
            par ^= 1;
        }
    }
    if (live && h == 0) {
        float *o = out + unit * out_stride + out_offset;
#pragma unroll
        for (int t = 0; t < T3; ++t) o[32 * t + col] = mx[t];
    }
}

template <int C1, int C2, int C3, int NS, bool XYZ = false>
int launch_pre(const float *p, int64_t stride, const float *q, const int32_t *idx, int64_t batch,
               int64_t n, int64_t m, const float *w23, float *out, int64_t os, int64_t oo, hipStream_t s)
{
    const int64_t total = batch * m;
    const int64_t blocks = (total + 3) / 4;
    REQUIRE(blocks <= 0x7fffffff, "sa_group_mlp_pre: too many centres");
    hipLaunchKernelGGL((sa_pre_lds_kernel<C1, C2, C3, NS, XYZ>), dim3((unsigned)blocks), dim3(256), 0, s, p,
                       stride, q, idx, (int)n, (int)m, total, w23, out, os, oo);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

}  // namespace

// dispatch used by lidar_sa_group_mlp_pre_f32 (sa_mlp.hip); -1 = no LDS-staged variant
int lidar_sa_pre_lds_dispatch(int cfeat, int c1, int c2, int c3, int ns, const float *p, int64_t stride,
                              const float *q, const int32_t *idx, int64_t batch, int64_t n, int64_t m,
                              const float *w23, float *out, int64_t os, int64_t oo, hipStream_t s)
{
    (void)cfeat;
    if (c1 == 128 && c2 == 128 && c3 == 256 && ns == 64)
        return launch_pre<128, 128, 256, 64>(p, stride, q, idx, batch, n, m, w23, out, os, oo, s);
    if (c1 == 128 && c2 == 128 && c3 == 256 && ns == 128)
        return launch_pre<128, 128, 256, 128>(p, stride, q, idx, batch, n, m, w23, out, os, oo, s);
    if (c1 == 64 && c2 == 64 && c3 == 128 && ns == 32)
        return launch_pre<64, 64, 128, 32>(p, stride, q, idx, batch, n, m, w23, out, os, oo, s);
    return -1;
}

// dispatch used by lidar_sa_group_mlp_f32 for levels without features (cfeat == 0):
// xyz / centres as usual, packed = the whole lidar_mlp_pack_f32 image; -1 = no variant
int lidar_sa_xyz_lds_dispatch(int c1, int c2, int c3, int ns, const float *xyz, const float *centres,
                              const int32_t *idx, int64_t batch, int64_t n, int64_t m, const float *packed,
                              float *out, int64_t os, int64_t oo, hipStream_t s)
{
    if (c1 == 64 && c2 == 64 && c3 == 128 && ns == 32)
        return launch_pre<64, 64, 128, 32, true>(xyz, 3, centres, idx, batch, n, m, packed, out, os, oo, s);
    if (c1 == 64 && c2 == 96 && c3 == 128 && ns == 128)
        return launch_pre<64, 96, 128, 128, true>(xyz, 3, centres, idx, batch, n, m, packed, out, os, oo, s);
    return -1;
}
