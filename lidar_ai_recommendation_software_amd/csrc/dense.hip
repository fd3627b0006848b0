// dense.hip — the native fp32 dense layers on gfx950 MFMA (v_mfma_f32_32x32x2_f32, exact fp32).
//
// dense_relu_kernel: LDS-tiled 128x128x16 GEMM with a bias (+ReLU) epilogue and an optional fused
// row-group max-pool — the strict-fp32 path (PointNet2Backbone(x3=False)) of SA2's per-point
// layer 1 and group_all's three layers; the default x3 path runs them on dense_x3s.hip.
// concat_xyz_pad_kernel writes the [features, x, y, z, 0-pad] rows group_all and the per-point
// layer 1 read.
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

}  // namespace

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
    ON_DEVICE(h->device);
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


LIDAR_EXPORT int lidar_concat_xyz_pad_f32(lidar_handle *h, const float *xyz, int64_t rows,
                                          float *y, int64_t ldy, int64_t col0, void *stream)
{
    REQUIRE(h && xyz && y, "lidar_concat_xyz_pad_f32: null pointer");
    REQUIRE(col0 >= 0 && col0 + 3 <= ldy, "lidar_concat_xyz_pad_f32: bad columns");
    if (rows == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    const int64_t total = rows * (ldy - col0);
    hipLaunchKernelGGL(concat_xyz_pad_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), xyz, rows, y, ldy, col0);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
