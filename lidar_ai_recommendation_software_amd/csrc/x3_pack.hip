// x3_pack.hip — the packed weight images of the dense GEMM (dense_x3s.hip).
//
// h3 image (the fp32 contract, h3.hpp): a layer's weights W (k, cout) are scaled by one power of
// two 2^s (max |W| 2^s < 2^14) and split ONCE (at backbone construction) into fp16 hi / lo MFMA B
// fragments of v_mfma_f32_32x32x16_f16: per 32-column tile, 16-deep k-step and hi / lo half, 64
// lanes x 8 fp16 — one contiguous KiB that a wave's LDS-DMA moves whole.  K is padded to whole
// 32-deep stages with zero weights.  The image ends in a 256-byte tail whose first int32 is s and
// whose second is the image kind (h3.hpp kTagH3 / kTagX1, checked by the GEMM).
// bf16 image (X1, the bf16 spec): the same fragment order, hi = bf16(w) (lo = bf16(w - hi), not
// read by the X1 GEMM), no scaling.
#include "h3.hpp"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
using lidar_h3::f16x8;

constexpr int XBN = 128, XBK = 32;
constexpr int kTail = 256;  // bytes after the fragments: int32 layer exponent, padding

// max |W| over the layer (one workgroup) -> the layer exponent s in the image's tail
__global__ __launch_bounds__(1024) void dense_absmax_kernel(const float *__restrict__ w, int64_t n,
                                                            int32_t *__restrict__ tail)
{
    __shared__ uint32_t red[16];
    uint32_t m = 0;
    for (int64_t i = threadIdx.x; i < n; i += 1024) m = max(m, lidar_h3::abs_bits(w[i]));
    m = (uint32_t)lidar::wave_max_i32_dpp((int)m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 16; ++i) m = max(m, red[i]);
        tail[0] = 14 - lidar_h3::exp_of_bits(max(m, red[0]));
    }
}

// packed B: element (kk, n) of tile t = n / 32, k-step s = kk / 16 at
// ((((t * KS + s) * 2 + half) * 64 + lane) * 8 + j), lane = 32 * ((kk % 16) / 8) + n % 32, j = kk % 8
template <bool H3>
__global__ void dense_pack_kernel(const float *__restrict__ w, int k, int cout, int ks, uint16_t *__restrict__ packed,
                                  int32_t *__restrict__ tail)
{
    const int64_t total = (int64_t)(cout / 32) * ks * 64;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) tail[1] = H3 ? lidar_h3::kTagH3 : lidar_h3::kTagX1;
    if (i >= total) return;
    const int lane = (int)(i % 64), s = (int)((i / 64) % ks), t = (int)(i / 64 / ks);
    const int n = 32 * t + (lane & 31);
    uint16_t *o = packed + ((((int64_t)t * ks + s) * 2) * 64 + lane) * 8;
    if constexpr (H3) {
        const float sc = lidar_h3::scale_of(14 - tail[0]);
        f16x8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int kk = 16 * s + 8 * (lane >> 5) + j;
            const float v = (kk < k ? w[(int64_t)kk * cout + n] : 0.0f) * sc;
            const _Float16 hh = (_Float16)v;
            hi[j] = hh;
            lo[j] = (_Float16)(v - (float)hh);
        }
        *reinterpret_cast<f16x8 *>(o) = hi;
        *reinterpret_cast<f16x8 *>(o + 512) = lo;
    } else {
        bf16x8 hi, lo;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int kk = 16 * s + 8 * (lane >> 5) + j;
            const float v = kk < k ? w[(int64_t)kk * cout + n] : 0.0f;
            const __bf16 hh = (__bf16)v;
            hi[j] = hh;
            lo[j] = (__bf16)(v - (float)hh);
        }
        *reinterpret_cast<bf16x8 *>(o) = hi;
        *reinterpret_cast<bf16x8 *>(o + 512) = lo;
    }
}

int64_t fragment_bytes(int64_t k, int64_t cout) { return (cout / 32) * ((k + XBK - 1) / XBK * 2) * 2 * 1024; }

int pack(lidar_handle *h, const float *w, int32_t k, int32_t cout, void *packed, void *stream, bool h3,
         const char *who)
{
    REQUIRE(h && w && packed, std::string(who) + ": null pointer");
    REQUIRE(k > 0 && k % 16 == 0 && cout > 0 && cout % XBN == 0, std::string(who) + ": k % 16, cout % 128");
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int ks = (k + XBK - 1) / XBK * 2;
    const int64_t total = (int64_t)(cout / 32) * ks * 64;
    int32_t *tail = reinterpret_cast<int32_t *>(static_cast<char *>(packed) + fragment_bytes(k, cout));
    if (h3) {
        hipLaunchKernelGGL(dense_absmax_kernel, dim3(1), dim3(1024), 0, s, w, (int64_t)k * cout, tail);
        hipLaunchKernelGGL(dense_pack_kernel<true>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, w, (int)k,
                           (int)cout, ks, static_cast<uint16_t *>(packed), tail);
    } else {
        hipLaunchKernelGGL(dense_pack_kernel<false>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, w, (int)k,
                           (int)cout, ks, static_cast<uint16_t *>(packed), tail);
    }
    LAUNCH_CHECK();
    return LIDAR_OK;
}

}  // namespace

// the fragment bytes of a (k, cout) image (the tail starts there); internal to the library
int lidar_dense_x3_packed_image(int32_t k, int32_t cout, int64_t *bytes)
{
    REQUIRE(k > 0 && cout > 0 && cout % XBN == 0, "dense GEMM image: k > 0, cout % 128");
    *bytes = fragment_bytes(k, cout);
    return LIDAR_OK;
}

// bytes of the packed weight image of a (k, cout) layer (either image)
LIDAR_EXPORT int64_t lidar_dense_x3_packed_size(int32_t k, int32_t cout)
{
    return k > 0 && cout > 0 && cout % XBN == 0 ? fragment_bytes(k, cout) + kTail : 0;
}

// W (k, cout) fp32 on the device -> the h3 image: fp16 hi / lo B fragments of W 2^s and s (device,
// async on stream)
LIDAR_EXPORT int lidar_dense_x3_pack_f32(lidar_handle *h, const float *w, int32_t k, int32_t cout, void *packed,
                                         void *stream)
{
    return pack(h, w, k, cout, packed, stream, true, "lidar_dense_x3_pack_f32");
}

// W (k, cout) fp32 on the device -> the bf16 image of the X1 GEMM (the bf16 spec)
LIDAR_EXPORT int lidar_dense_x1_pack_f32(lidar_handle *h, const float *w, int32_t k, int32_t cout, void *packed,
                                         void *stream)
{
    return pack(h, w, k, cout, packed, stream, false, "lidar_dense_x1_pack_f32");
}
