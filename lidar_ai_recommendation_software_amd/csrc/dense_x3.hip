// dense_x3.hip — the dense layers (per-point layer 1 of SA2, group_all's three layers) in fp32
// arithmetic on the bf16 matrix cores, the GEMM counterpart of sa_mlp_x3.hip.
//
// y (rows, cout) = x (rows, K) W (K, cout) + b [-> ReLU] [-> max over runs of pool_rows rows],
// same contract and epilogue as lidar_dense_f32 (sa_mlp.hip).  Each fp32 operand is split
// exactly into bf16 hi + lo as it is staged into LDS; a product is accumulated as
// ah*bh + ah*bl + al*bh on v_mfma_f32_32x32x16_bf16 with fp32 accumulation (<= ~2^-15 per
// product).  128x128 output tile per 4-wave workgroup (64x64 per wave = 2x2
// MFMA tiles), K staged 16 at a time: A as [m][k] and B as [n][k] bf16 rows (k contiguous, so
// a lane's 8-element fragment A[row][8h..8h+7] / B[8h..8h+7][col] is one 16-byte read), each row
// padded by 8 elements against LDS bank conflicts.
#include "common.hpp"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int XBM = 128, XBN = 128, XBK = 16, XPAD = 8, XLD = XBK + XPAD;  // LDS row: 24 bf16

__host__ __device__ constexpr int rho(int r) { return (r & 3) + 8 * (r >> 2); }
__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }

__device__ __forceinline__ f32x16 mfma_bf(bf16x8 a, bf16x8 b, f32x16 c)
{
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(256) void dense_x3_kernel(const float *__restrict__ x, int K,
                                                       const float *__restrict__ w,
                                                       const float *__restrict__ bias, int cout, int pool_rows,
                                                       float *__restrict__ y, int act)
{
    // [hi/lo][row][k]
    __shared__ __attribute__((aligned(16))) __bf16 As[2][XBM][XLD];
    __shared__ __attribute__((aligned(16))) __bf16 Bs[2][XBN][XLD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int wm = wave >> 1, wn = wave & 1;
    const int64_t row0 = (int64_t)blockIdx.y * XBM;
    const int col0 = blockIdx.x * XBN;
    f32x16 acc[2][2] = {};

    // staging: A 128 x 16 (thread: row tid/2, 8 k at (tid&1)*8), B 16 x 128 (thread: k tid/16,
    // 8 columns at (tid%16)*8), both split into hi / lo bf16 on the way into LDS
    const int ar = tid >> 1, ak = (tid & 1) * 8;
    const int bk = tid >> 4, bc = (tid & 15) * 8;
    for (int k0 = 0; k0 < K; k0 += XBK) {
        const float *xa = x + (row0 + ar) * K + k0 + ak;
        const f32x4 a0 = *reinterpret_cast<const f32x4 *>(xa);
        const f32x4 a1 = *reinterpret_cast<const f32x4 *>(xa + 4);
        const float *wb = w + (int64_t)(k0 + bk) * cout + col0 + bc;
        const f32x4 b0 = *reinterpret_cast<const f32x4 *>(wb);
        const f32x4 b1 = *reinterpret_cast<const f32x4 *>(wb + 4);
        bf16x8 ah, al;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float v = j < 4 ? a0[j] : a1[j - 4];
            const __bf16 hv = (__bf16)v;
            ah[j] = hv;
            al[j] = (__bf16)(v - (float)hv);
        }
        __syncthreads();  // the previous k-block's reads are done
        *reinterpret_cast<bf16x8 *>(&As[0][ar][ak]) = ah;
        *reinterpret_cast<bf16x8 *>(&As[1][ar][ak]) = al;
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // B transposed into [n][k]
            const float v = j < 4 ? b0[j] : b1[j - 4];
            const __bf16 hv = (__bf16)v;
            Bs[0][bc + j][bk] = hv;
            Bs[1][bc + j][bk] = (__bf16)(v - (float)hv);
        }
        __syncthreads();
        bf16x8 fa[2][2], fb[2][2];  // [tile][hi/lo]
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                fa[i][p] = *reinterpret_cast<const bf16x8 *>(&As[p][wm * 64 + i * 32 + col][8 * h]);
                fb[i][p] = *reinterpret_cast<const bf16x8 *>(&Bs[p][wn * 64 + i * 32 + col][8 * h]);
            }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                acc[i][j] = mfma_bf(fa[i][0], fb[j][0], acc[i][j]);
                acc[i][j] = mfma_bf(fa[i][0], fb[j][1], acc[i][j]);
                acc[i][j] = mfma_bf(fa[i][1], fb[j][0], acc[i][j]);
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

}  // namespace

// lidar_dense_f32's contract (rows % 128, k % 16, cout % 128; optional ReLU and fused max-pool
// with y zeroed by the caller) on the split-bf16 path
LIDAR_EXPORT int lidar_dense_x3_f32(lidar_handle *h, const float *x, int64_t rows, int32_t k, const float *w,
                                    const float *bias, int32_t cout, int32_t relu_on, int32_t pool_rows, float *y,
                                    void *stream)
{
    REQUIRE(h && x && w && bias && y, "lidar_dense_x3_f32: null pointer");
    REQUIRE(rows % XBM == 0 && k % XBK == 0 && cout % XBN == 0 && k > 0,
            "lidar_dense_x3_f32: rows % 128, k % 16, cout % 128 must be 0");
    REQUIRE(pool_rows == 0 || (pool_rows % XBM == 0 && rows % pool_rows == 0),
            "lidar_dense_x3_f32: pool_rows must be a multiple of 128 dividing rows");
    REQUIRE(pool_rows == 0 || relu_on, "lidar_dense_x3_f32: the fused max-pool needs relu (>= 0 outputs)");
    if (rows == 0) return LIDAR_OK;
    REQUIRE(rows / XBM <= 65535, "lidar_dense_x3_f32: too many rows");
    HIP_TRY(hipSetDevice(h->device));
    hipLaunchKernelGGL(dense_x3_kernel, dim3(cout / XBN, (unsigned)(rows / XBM)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), x, (int)k, w, bias, (int)cout, (int)pool_rows, y,
                       relu_on ? 1 : 0);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
