// dense_x3.hip — the dense layers (per-point layer 1 of SA2, group_all's three layers) in fp32
// arithmetic on the bf16 matrix cores, the GEMM counterpart of sa_mlp_x3.hip.
//
// y (rows, cout) = x (rows, K) W (K, cout) + b [-> ReLU] [-> max over runs of pool_rows rows],
// same contract and epilogue as lidar_dense_f32 (sa_mlp.hip).  Each fp32 operand is split
// exactly into bf16 hi + lo; a product is accumulated as ah*bh + ah*bl + al*bh on
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation (<= ~2^-15 per product).
//
// W is split once into a packed image of MFMA B fragments (lidar_dense_x3_pack_f32: per 32-column
// tile, 16-deep k-step and hi / lo half, 64 lanes x 8 bf16 — one contiguous KiB), so the kernel
// only splits the activations.  128x128 output tile per 4-wave workgroup (64x64 per wave = 2x2
// MFMA tiles), K in stages of 32 double-buffered in LDS by global_load_lds (no VGPR staging):
//   A stage: 128 rows x 32 fp32 = 16 KiB, row r's 16-byte chunk q at slot q ^ ((r >> 1) & 7) —
//            each lane of a load instruction picks the global chunk that lands in its slot, and
//            the fragment reads (ds_read_b128, rows 0..31 of a tile) are bank-conflict free;
//   B stage: 4 column tiles x 2 k-steps x hi / lo KiB fragments = 16 KiB, read lane-linear.
// One barrier per stage.  Workgroups are laid out so that the column tiles of a row tile share
// an XCD (blocks b and b + 8 do): A is fetched into one L2 once.
#include "common.hpp"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int XBM = 128, XBN = 128, XBK = 32;
constexpr int kStageA = XBM * XBK;        // floats per A stage
constexpr int kStageB = 4 * 2 * 2 * 512;  // bf16 per B stage (4 col tiles x 2 k-steps x hi/lo x 1 KiB)

__host__ __device__ constexpr int rho(int r) { return (r & 3) + 8 * (r >> 2); }
__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }

__device__ __forceinline__ f32x16 mfma_bf(bf16x8 a, bf16x8 b, f32x16 c)
{
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void split8(const f32x4 &a0, const f32x4 &a1, bf16x8 &hi, bf16x8 &lo)
{
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v = j < 4 ? a0[j] : a1[j - 4];
        const __bf16 h = (__bf16)v;
        hi[j] = h;
        lo[j] = (__bf16)(v - (float)h);
    }
}

// 16 bytes per lane from g (per-lane address) to LDS at l + 16 * lane (l: the wave-uniform base)
__device__ __forceinline__ void lds_dma16(const void *g, void *l)
{
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)l, 16, 0, 0);
}

// packed B: element (kk, n) of tile t = n / 32, k-step s = kk / 16 at
// ((((t * KS + s) * 2 + half) * 64 + lane) * 8 + j), lane = 32 * ((kk % 16) / 8) + n % 32, j = kk % 8
__global__ void dense_x3_pack_kernel(const float *__restrict__ w, int k, int cout, int ks,
                                     __bf16 *__restrict__ packed)
{
    const int64_t total = (int64_t)(cout / 32) * ks * 64;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int lane = (int)(i % 64), s = (int)((i / 64) % ks), t = (int)(i / 64 / ks);
    const int n = 32 * t + (lane & 31);
    bf16x8 hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int kk = 16 * s + 8 * (lane >> 5) + j;
        const float v = kk < k ? w[(int64_t)kk * cout + n] : 0.0f;
        const __bf16 h = (__bf16)v;
        hi[j] = h;
        lo[j] = (__bf16)(v - (float)h);
    }
    bf16x8 *o = reinterpret_cast<bf16x8 *>(packed) + (((int64_t)t * ks + s) * 2) * 64 + lane;
    o[0] = hi;
    o[64] = lo;
}

__global__ __launch_bounds__(256, 2) void dense_x3p_kernel(const float *__restrict__ x, int K,
                                                           const __bf16 *__restrict__ wp, int ks,
                                                           const float *__restrict__ bias, int cout,
                                                           int pool_rows, float *__restrict__ y, int act,
                                                           int ntn, int64_t total, int64_t per_xcd)
{
    __shared__ __attribute__((aligned(16))) float As[2][kStageA];
    __shared__ __attribute__((aligned(16))) __bf16 Bs[2][kStageB];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int wm = wave >> 1, wn = wave & 1;
    const int64_t L = blockIdx.x;
    const int64_t logical = (L & 7) * per_xcd + (L >> 3);
    if (logical >= total) return;  // whole workgroup
    const int64_t row0 = logical / ntn * XBM;
    const int tn = (int)(logical % ntn);
    const int col0 = tn * XBN;
    const int nst = (K + XBK - 1) / XBK;

    // A: wave w loads rows 32w .. 32w+31 (4 instructions of 8 rows); lane -> (row, slot)
    const int arow_l = lane >> 3, aslot = lane & 7;
    auto load_stage = [&](int st, int buf) {
        const int k0 = st * XBK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 32 * wave + 8 * i + arow_l;
            const int kq = aslot ^ ((r >> 1) & 7);
            if (k0 + 4 * kq < K)
                lds_dma16(x + (row0 + r) * K + k0 + 4 * kq, &As[buf][(32 * wave + 8 * i) * XBK]);
        }
        // B: wave w loads column tile 4 tn + w, k-steps 2 st, 2 st + 1, hi / lo: 4 KiB contiguous
        const __bf16 *src = wp + (((int64_t)(4 * tn + wave) * ks + 2 * st) * 2) * 512;
        const int nb = 2 * st + 1 < ks ? 4 : 2;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (i < nb) lds_dma16(src + i * 512 + lane * 8, &Bs[buf][(wave * 4 + i) * 512]);
    };

    f32x16 acc[2][2] = {};
    load_stage(0, 0);
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        __syncthreads();  // (vmcnt(0)) stage st landed everywhere; buf ^ 1 no longer read
        if (st + 1 < nst) load_stage(st + 1, buf ^ 1);
        const int nks = (st * XBK + 16 < K) ? 2 : 1;
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
            if (ss < nks) {
                bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int r = wm * 64 + i * 32 + col;
                    const int kq = 4 * ss + 2 * h;
                    const int sl = kq ^ ((r >> 1) & 7);  // kq even: the pair (sl, sl ^ 1)
                    const f32x4 a0 = *reinterpret_cast<const f32x4 *>(&As[buf][r * XBK + 4 * sl]);
                    const f32x4 a1 = *reinterpret_cast<const f32x4 *>(&As[buf][r * XBK + 4 * (sl ^ 1)]);
                    split8(a0, a1, ah[i], al[i]);
                }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int tt = 2 * wn + j;
                    bh[j] = *reinterpret_cast<const bf16x8 *>(&Bs[buf][((tt * 2 + ss) * 2 + 0) * 512 + lane * 8]);
                    bl[j] = *reinterpret_cast<const bf16x8 *>(&Bs[buf][((tt * 2 + ss) * 2 + 1) * 512 + lane * 8]);
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        acc[i][j] = mfma_bf(ah[i], bh[j], acc[i][j]);
                        acc[i][j] = mfma_bf(ah[i], bl[j], acc[i][j]);
                        acc[i][j] = mfma_bf(al[i], bh[j], acc[i][j]);
                    }
            }
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
            if (h == 0) {  // non-negative floats order as their bits: exact, order-free
                unsigned *dst = reinterpret_cast<unsigned *>(y + (row0 / pool_rows) * cout + c);
                atomicMax(dst, __float_as_uint(v));
            }
        }
    }
}

int64_t packed_bytes(int64_t k, int64_t cout) { return (cout / 32) * ((k + XBK - 1) / XBK * 2) * 2 * 1024; }

int launch_pack(const float *w, int32_t k, int32_t cout, void *packed, hipStream_t s)
{
    const int ks = (k + XBK - 1) / XBK * 2;
    const int64_t total = (int64_t)(cout / 32) * ks * 64;
    hipLaunchKernelGGL(dense_x3_pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, w, (int)k,
                       (int)cout, ks, static_cast<__bf16 *>(packed));
    LAUNCH_CHECK();
    return LIDAR_OK;
}

int launch_gemm(const float *x, int64_t rows, int32_t k, const void *packed, const float *bias, int32_t cout,
                int32_t relu_on, int32_t pool_rows, float *y, hipStream_t s)
{
    const int ks = (k + XBK - 1) / XBK * 2;
    const int ntn = cout / XBN;
    const int64_t total = (rows / XBM) * ntn, per_xcd = (total + 7) / 8;
    REQUIRE(per_xcd * 8 <= 0x7fffffff, "lidar_dense_x3: too many rows");
    hipLaunchKernelGGL(dense_x3p_kernel, dim3((unsigned)(per_xcd * 8)), dim3(256), 0, s, x, (int)k,
                       static_cast<const __bf16 *>(packed), ks, bias, (int)cout, (int)pool_rows, y,
                       relu_on ? 1 : 0, ntn, total, per_xcd);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

}  // namespace

#define DENSE_X3_CHECK(fn)                                                                             \
    REQUIRE(rows % XBM == 0 && k % 16 == 0 && cout % XBN == 0 && k > 0,                                \
            fn ": rows % 128, k % 16, cout % 128 must be 0");                                          \
    REQUIRE(pool_rows == 0 || (pool_rows % XBM == 0 && rows % pool_rows == 0),                         \
            fn ": pool_rows must be a multiple of 128 dividing rows");                                  \
    REQUIRE(pool_rows == 0 || relu_on, fn ": the fused max-pool needs relu (>= 0 outputs)")

// bytes of the packed weight image of a (k, cout) layer
LIDAR_EXPORT int64_t lidar_dense_x3_packed_size(int32_t k, int32_t cout)
{
    return k > 0 && cout > 0 && cout % XBN == 0 ? packed_bytes(k, cout) : 0;
}

// W (k, cout) fp32 on the device -> packed bf16 hi / lo B fragments (device, async on stream)
LIDAR_EXPORT int lidar_dense_x3_pack_f32(lidar_handle *h, const float *w, int32_t k, int32_t cout, void *packed,
                                         void *stream)
{
    REQUIRE(h && w && packed, "lidar_dense_x3_pack_f32: null pointer");
    REQUIRE(k > 0 && k % 16 == 0 && cout > 0 && cout % XBN == 0, "lidar_dense_x3_pack_f32: k % 16, cout % 128");
    HIP_TRY(hipSetDevice(h->device));
    return launch_pack(w, k, cout, packed, static_cast<hipStream_t>(stream));
}

// the GEMM on a packed weight image
LIDAR_EXPORT int lidar_dense_x3p_f32(lidar_handle *h, const float *x, int64_t rows, int32_t k, const void *packed,
                                     const float *bias, int32_t cout, int32_t relu_on, int32_t pool_rows, float *y,
                                     void *stream)
{
    REQUIRE(h && x && packed && bias && y, "lidar_dense_x3p_f32: null pointer");
    DENSE_X3_CHECK("lidar_dense_x3p_f32");
    if (rows == 0) return LIDAR_OK;
    HIP_TRY(hipSetDevice(h->device));
    return launch_gemm(x, rows, k, packed, bias, cout, relu_on, pool_rows, y, static_cast<hipStream_t>(stream));
}

// lidar_dense_f32's contract (rows % 128, k % 16, cout % 128; optional ReLU and fused max-pool
// with y zeroed by the caller) on the split-bf16 path; packs W into the handle's workspace
LIDAR_EXPORT int lidar_dense_x3_f32(lidar_handle *h, const float *x, int64_t rows, int32_t k, const float *w,
                                    const float *bias, int32_t cout, int32_t relu_on, int32_t pool_rows, float *y,
                                    void *stream)
{
    REQUIRE(h && x && w && bias && y, "lidar_dense_x3_f32: null pointer");
    DENSE_X3_CHECK("lidar_dense_x3_f32");
    if (rows == 0) return LIDAR_OK;
    HIP_TRY(hipSetDevice(h->device));
    void *ws = lidar::workspace(h, (uint64_t)packed_bytes(k, cout));
    if (!ws) return LIDAR_ENOMEM;
    hipStream_t s = static_cast<hipStream_t>(stream);
    int rc = launch_pack(w, k, cout, ws, s);
    if (rc) return rc;
    return launch_gemm(x, rows, k, ws, bias, cout, relu_on, pool_rows, y, s);
}
