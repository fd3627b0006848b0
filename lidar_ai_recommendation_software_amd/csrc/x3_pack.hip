// x3_pack.hip — the packed weight image of the x3 dense GEMM (dense_x3s.hip).
//
// x3 arithmetic: every fp32 operand is split exactly into bf16 hi + lo, and a product
// is accumulated as ah*bh + ah*bl + al*bh on bf16 MFMAs with fp32 accumulation.  The weights of a
// dense layer are split ONCE (at backbone construction) into MFMA B fragments of
// v_mfma_f32_32x32x16_bf16: per 32-column tile, 16-deep k-step and hi / lo half, 64 lanes x 8 bf16
// — one contiguous KiB that a wave's LDS-DMA moves whole.  K is padded to whole 32-deep stages
// with zero weights.
#include "common.hpp"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int XBN = 128, XBK = 32;

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

int64_t packed_bytes(int64_t k, int64_t cout) { return (cout / 32) * ((k + XBK - 1) / XBK * 2) * 2 * 1024; }

}  // namespace

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
    ON_DEVICE(h->device);
    const int ks = (k + XBK - 1) / XBK * 2;
    const int64_t total = (int64_t)(cout / 32) * ks * 64;
    hipLaunchKernelGGL(dense_x3_pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), w, (int)k, (int)cout, ks, static_cast<__bf16 *>(packed));
    LAUNCH_CHECK();
    return LIDAR_OK;
}
