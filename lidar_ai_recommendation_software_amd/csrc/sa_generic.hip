// sa_generic.hip — the two byte-moving halves of a set-abstraction branch of ANY shape (SURVEY §8a
// N3/N4, the pointnet2 PointnetSAModule(MSG) with arbitrary mlp widths and nsample), around the
// dense GEMMs (dense_x3s.hip h3 / bf16 spec, dense.hip fp32):
//
//   group rows  rows[(b M + m) ns + s] = [f[idx] (cfeat), xyz[idx] - centre (fp32), 0-pad to ldr]
//               — pointnet2's QueryAndGroup(use_xyz) (grouped_xyz - new_xyz, then the features) in
//               the layer-1 row order the packed weights use ([f, xyz], layer1_weights); rows past
//               B M ns up to `rows` are zero (the GEMM's 128-row tiles)
//   group max   out[g, off + c] = max over the ns rows of group g of in[., c] — the max-pool over
//               the nsample axis (F.max_pool2d over [1, nsample]: a NaN propagates)
//
// The fused kernels (sa_mlp16 / sa_mlp_x3 / sa_mlp_x1 / sa_mlp_bq) keep every grouped row in
// registers and LDS but exist only for the six instantiated shapes; this path materialises the
// grouped rows in HBM, so it serves every other shape at HBM cost (algorithmic bytes per grouped
// row: the gathered row ldr * 4 written + read by layer 1, per layer the fp32 activations written
// and read, the max reads c3 * 4).
#include "common.hpp"

namespace {

constexpr int GT = 256;

__global__ __launch_bounds__(GT) void group_rows_kernel(const float *__restrict__ feat, int64_t ldf, int cfeat,
                                                        const float *__restrict__ xyz,
                                                        const float *__restrict__ centres,
                                                        const int32_t *__restrict__ idx, int64_t n, int64_t m,
                                                        int ns, int64_t grouped, int64_t rows,
                                                        float *__restrict__ out, int64_t ldr)
{
    // one thread per (row, 4-column chunk): a row's chunks are adjacent threads (coalesced stores)
    const int64_t cpr = ldr / 4;
    const int64_t t = (int64_t)blockIdx.x * GT + threadIdx.x;
    if (t >= rows * cpr) return;
    const int64_t r = t / cpr;
    const int c0 = (int)(t % cpr) * 4;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (r < grouped) {
        const int64_t g = r / ns;           // b M + m
        const int64_t b = g / m;
        const int64_t p = b * n + idx[r];   // the neighbour's point row
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = c0 + j;
            if (c < cfeat) v[j] = feat[p * ldf + c];
            else if (c < cfeat + 3) v[j] = xyz[p * 3 + (c - cfeat)] - centres[g * 3 + (c - cfeat)];
        }
    }
    *reinterpret_cast<float4 *>(out + r * ldr + c0) = make_float4(v[0], v[1], v[2], v[3]);
}

__global__ __launch_bounds__(GT) void group_max_kernel(const float *__restrict__ in, int64_t ldi, int64_t groups,
                                                       int ns, int c, float *__restrict__ out, int64_t ldo,
                                                       int64_t off)
{
    const int64_t t = (int64_t)blockIdx.x * GT + threadIdx.x;
    if (t >= groups * c) return;
    const int64_t g = t / c;
    const int ch = (int)(t % c);
    const float *p = in + g * ns * ldi + ch;
    float mx = p[0];
    for (int s = 1; s < ns; ++s) {
        const float x = p[(int64_t)s * ldi];
        mx = (x > mx || x != x) ? x : mx;  // NaN propagates (first NaN wins)
        if (mx != mx) break;
    }
    out[g * ldo + off + ch] = mx;
}

}  // namespace

LIDAR_EXPORT int lidar_sa_group_rows_f32(lidar_handle *h, const float *feat, int64_t ldf, int32_t cfeat,
                                         const float *xyz, const float *centres, const int32_t *idx, int64_t batch,
                                         int64_t n, int64_t m, int32_t nsample, float *rows_out, int64_t rows,
                                         int64_t ldr, void *stream)
{
    REQUIRE(h && xyz && centres && idx && rows_out, "lidar_sa_group_rows_f32: null pointer");
    REQUIRE(cfeat >= 0 && (cfeat == 0 || (feat && ldf >= cfeat)), "lidar_sa_group_rows_f32: bad feature operand");
    REQUIRE(batch >= 0 && n > 0 && m >= 0 && nsample > 0, "lidar_sa_group_rows_f32: bad shape");
    REQUIRE(ldr % 4 == 0 && ldr >= cfeat + 3, "lidar_sa_group_rows_f32: ldr must be a multiple of 4 >= cfeat + 3");
    const int64_t grouped = batch * m * nsample;
    REQUIRE(rows >= grouped, "lidar_sa_group_rows_f32: rows < batch * m * nsample");
    if (rows == 0) return LIDAR_OK;
    const int64_t threads = rows * (ldr / 4);
    REQUIRE((threads + GT - 1) / GT <= 0x7fffffff, "lidar_sa_group_rows_f32: too many rows");
    ON_DEVICE(h->device);
    hipLaunchKernelGGL(group_rows_kernel, dim3((unsigned)((threads + GT - 1) / GT)), dim3(GT), 0,
                       static_cast<hipStream_t>(stream), feat, ldf, (int)cfeat, xyz, centres, idx, n, m,
                       (int)nsample, grouped, rows, rows_out, ldr);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

LIDAR_EXPORT int lidar_group_max_f32(lidar_handle *h, const float *in, int64_t ldi, int64_t groups, int32_t nsample,
                                     int32_t c, float *out, int64_t ldo, int64_t out_offset, void *stream)
{
    REQUIRE(h && in && out, "lidar_group_max_f32: null pointer");
    REQUIRE(groups >= 0 && nsample > 0 && c > 0 && ldi >= c && out_offset >= 0 && ldo >= out_offset + c,
            "lidar_group_max_f32: bad shape");
    if (groups == 0) return LIDAR_OK;
    const int64_t threads = groups * c;
    REQUIRE((threads + GT - 1) / GT <= 0x7fffffff, "lidar_group_max_f32: too many groups");
    ON_DEVICE(h->device);
    hipLaunchKernelGGL(group_max_kernel, dim3((unsigned)((threads + GT - 1) / GT)), dim3(GT), 0,
                       static_cast<hipStream_t>(stream), in, ldi, groups, (int)nsample, (int)c, out, ldo,
                       out_offset);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
