// ball_query.hip — first-nsample ball query on gfx950 (exact, index order).
//
// Spec (oracle orc_ball_query): for every centre, the first `nsample`
// point indices in ascending order with d < r*r (fp32, d = (dx*dx+dy*dy)+dz*dz, one
// rounding per op), unused slots repeat the first hit, no hit -> 0.
//
// One wavefront serves 8 centres of a frame: it scans the frame in index order, 128
// points per step (two coalesced 64-point chunks, the next pair prefetched), tests them
// against all 8 centres (the loads are shared 8 ways), __ballot collects each centre's hits, popcount ranks them,
// and the scan stops once every centre has nsample hits — for uniform frames at
// r = 0.2 that is ~12 % of the frame.
#include "common.hpp"

namespace {

constexpr int kC = 8;  // centres per wavefront: every loaded 64-point chunk is tested against all

__global__ __launch_bounds__(256) void ball_query_kernel(const float *__restrict__ xyz,
                                                         const float *__restrict__ centres,
                                                         int n, int m, int64_t groups_per_frame,
                                                         int64_t total_groups, float r2, int ns,
                                                         int32_t *__restrict__ out)
{
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gw >= total_groups) return;  // wave-uniform
    const int64_t b = gw / groups_per_frame;
    const int c0 = (int)(gw % groups_per_frame) * kC;
    const int nc = min(kC, m - c0);
    const float *p = xyz + b * (int64_t)n * 3;
    float cx[kC], cy[kC], cz[kC];
    int cnt[kC], first[kC];
#pragma unroll
    for (int j = 0; j < kC; ++j) {
        const int64_t c = b * m + c0 + (j < nc ? j : 0);
        cx[j] = centres[3 * c];
        cy[j] = centres[3 * c + 1];
        cz[j] = centres[3 * c + 2];
        cnt[j] = j < nc ? 0 : ns;  // padding centres start "done"
        first[j] = -1;
    }
    const uint64_t below = (1ull << lane) - 1;
    // the scan is load-latency bound (a wave waits on its chunk ~half the time): the next
    // chunk's 12-byte point is in flight while the current one is tested
    struct P3 {
        float x, y, z;
    };
    const P3 *pp = reinterpret_cast<const P3 *>(p);
    const P3 zero{0.f, 0.f, 0.f};
    // two 64-point chunks per iteration (each lane tests two points against the 8 centres:
    // independent work in flight), the next pair prefetched.  Hand-unrolled: a generic
    // k-chunk loop measured slower (0.96 / 0.93 ms for 2 / 4 chunks vs 0.86, B=32 SA1).
    P3 c0p = lane < n ? pp[lane] : zero, c1p = lane + 64 < n ? pp[lane + 64] : zero;
    for (int base = 0; base < n; base += 128) {
        bool open = false;
#pragma unroll
        for (int j = 0; j < kC; ++j) open |= cnt[j] < ns;
        if (!open) break;  // wave-uniform
        const int k0 = base + lane, k1 = k0 + 64;
        const P3 n0 = k0 + 128 < n ? pp[k0 + 128] : zero, n1 = k1 + 128 < n ? pp[k1 + 128] : zero;
        const P3 a0 = c0p, a1 = c1p;
        c0p = n0;
        c1p = n1;
#pragma unroll
        for (int j = 0; j < kC; ++j) {
            if (cnt[j] >= ns) continue;  // wave-uniform
            const bool h0 = k0 < n && lidar::dist2f(a0.x, a0.y, a0.z, cx[j], cy[j], cz[j]) < r2;
            const bool h1 = k1 < n && lidar::dist2f(a1.x, a1.y, a1.z, cx[j], cy[j], cz[j]) < r2;
            const uint64_t m0 = __ballot(h0), m1 = __ballot(h1);
            if (m0 | m1) {
                int32_t *o = out + (b * m + c0 + j) * (int64_t)ns;
                if (first[j] < 0)
                    first[j] = m0 ? base + __ffsll((unsigned long long)m0) - 1
                                  : base + 64 + __ffsll((unsigned long long)m1) - 1;
                const int r0 = cnt[j] + __popcll(m0 & below);
                const int r1 = cnt[j] + __popcll(m0) + __popcll(m1 & below);  // chunk 1 after chunk 0
                if (h0 && r0 < ns) o[r0] = k0;
                if (h1 && r1 < ns) o[r1] = k1;
                cnt[j] += __popcll(m0) + __popcll(m1);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kC; ++j) {
        if (j >= nc) break;
        int32_t *o = out + (b * m + c0 + j) * (int64_t)ns;
        const int fill = first[j] < 0 ? 0 : first[j];
        for (int s2 = min(cnt[j], ns) + lane; s2 < ns; s2 += 64) o[s2] = fill;
    }
}

}  // namespace

LIDAR_EXPORT int lidar_ball_query_f32(lidar_handle *h, const float *xyz, const float *centres,
                                      int64_t batch, int64_t n, int64_t m, float radius,
                                      int32_t nsample, int32_t *idx, void *stream)
{
    REQUIRE(h && xyz && centres && idx, "lidar_ball_query_f32: null pointer");
    REQUIRE(batch >= 0 && n >= 1 && m >= 0 && nsample >= 1, "lidar_ball_query_f32: bad sizes");
    REQUIRE(n < 0x7fffffff && m < 0x7fffffff, "lidar_ball_query_f32: sizes exceed int32");
    REQUIRE(radius >= 0.0f, "lidar_ball_query_f32: negative radius");
    const int64_t total = batch * m;
    if (total == 0) return LIDAR_OK;
    HIP_TRY(hipSetDevice(h->device));
    const float r2 = radius * radius;
    const int64_t gpf = (m + kC - 1) / kC, groups = batch * gpf;
    const int64_t blocks = (groups + 3) / 4;
    REQUIRE(blocks <= 0x7fffffff, "lidar_ball_query_f32: too many centres");
    hipLaunchKernelGGL(ball_query_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       static_cast<hipStream_t>(stream), xyz, centres, (int)n, (int)m, gpf, groups, r2,
                       (int)nsample, idx);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
