// fps.hip — farthest-point sampling on gfx950, exact, bucket-pruned.
//
// Spec (oracle/lidar_oracle.c orc_fps): idx[0] = 0, dist = +inf,
// then npoint-1 times: dist = min(dist, d(., last)), last = argmax dist (lowest index
// on ties), d = (dx*dx + dy*dy) + dz*dz in fp32 with one rounding per operation.
//
// One 1024-thread workgroup per frame.  Prologue: frame bbox, counting sort of the
// points by a 16^3 Morton cell into a sorted SoA copy in the workspace (x, y, z,
// dist, original index), cut into buckets of 64 consecutive sorted points (one
// wavefront-width each).  Every bucket keeps, in the registers of its owner lane,
// its bounding box and its (max dist, index) key and the coordinates of that point.
//
// Step: a bucket can only change if some member gets closer to the new sample than
// its current dist.  lb = dist-from-bbox(q) computed with the SAME rounded operations
// as d is a lower bound of every member's d (fl() is monotone), so `lb >= bucket max`
// proves no member changes and the bucket is skipped — an exact pruning, not an
// approximation.  Active buckets are streamed (64 lanes = 64 points, coalesced SoA
// loads, L2-resident), updated, and re-reduced; the frame argmax is a wave
// __shfl_xor max over 64-bit keys (dist bits << 32 | ~index) and a 16-way LDS merge.
#include "common.hpp"

namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr int kGrid = 16;  // Morton cells per axis for the bucket ordering
constexpr int kCells = kGrid * kGrid * kGrid;

__device__ __forceinline__ uint32_t spread3(uint32_t v)  // 4 bits -> every third bit
{
    v &= 0xf;
    v = (v | (v << 4)) & 0x0c3;
    v = (v | (v << 2)) & 0x249;
    return v;
}

struct FrameWs {
    float *x, *y, *z, *d;
    uint32_t *idx;
};

__device__ __forceinline__ float gap(float q, float lo, float hi)
{
    return q < lo ? __fsub_rn(lo, q) : (q > hi ? __fsub_rn(q, hi) : 0.0f);
}

template <int BPL>
__global__ __launch_bounds__(kThreads) void fps_bucket_kernel(const float *__restrict__ xyz,
                                                              int n, int npoint,
                                                              int32_t *__restrict__ out_idx,
                                                              float *__restrict__ out_xyz,
                                                              float *__restrict__ ws, int64_t ws_stride)
{
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const float *p = xyz + (int64_t)b * n * 3;
    float *wsb = ws + (int64_t)b * ws_stride;
    FrameWs W{wsb, wsb + n, wsb + 2 * (int64_t)n, wsb + 3 * (int64_t)n,
              reinterpret_cast<uint32_t *>(wsb + 4 * (int64_t)n)};

    __shared__ uint32_t hist[kCells];
    __shared__ float red[6][kWaves];
    __shared__ uint32_t wsum[kWaves];
    __shared__ uint64_t skey[2][kWaves];
    __shared__ float sxyz[2][kWaves][3];

    // ---- frame bounding box
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = tid; i < n; i += kThreads) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float v = p[3 * i + a];
            lo[a] = fminf(lo[a], v);
            hi[a] = fmaxf(hi[a], v);
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        lo[a] = lidar::wave_min_f(lo[a]);
        hi[a] = lidar::wave_max_f(hi[a]);
    }
    if (lane == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            red[a][wave] = lo[a];
            red[3 + a][wave] = hi[a];
        }
    }
    for (int c = tid; c < kCells; c += kThreads) hist[c] = 0;
    __syncthreads();
    float scale[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float l = red[a][0], h = red[3 + a][0];
        for (int w = 1; w < kWaves; ++w) {
            l = fminf(l, red[a][w]);
            h = fmaxf(h, red[3 + a][w]);
        }
        lo[a] = l;
        scale[a] = h > l ? (float)kGrid / (h - l) : 0.0f;
    }

    // ---- counting sort by Morton cell (order inside a cell is irrelevant: exactness
    // never depends on the bucket layout, only the pruning rate does)
    auto cell_of = [&](int i) -> uint32_t {
        uint32_t c[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            int v = (int)((p[3 * i + a] - lo[a]) * scale[a]);
            c[a] = (uint32_t)min(max(v, 0), kGrid - 1);
        }
        return spread3(c[0]) | (spread3(c[1]) << 1) | (spread3(c[2]) << 2);
    };
    for (int i = tid; i < n; i += kThreads) atomicAdd(&hist[cell_of(i)], 1u);
    __syncthreads();
    {  // exclusive scan of 4096 counts, 4 per thread
        uint32_t v0 = hist[4 * tid], v1 = hist[4 * tid + 1], v2 = hist[4 * tid + 2], v3 = hist[4 * tid + 3];
        uint32_t s = v0 + v1 + v2 + v3, incl = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t t = __shfl_up(incl, o, 64);
            if (lane >= o) incl += t;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t base = 0;
        for (int w = 0; w < wave; ++w) base += wsum[w];
        uint32_t e = base + incl - s;
        hist[4 * tid] = e;
        hist[4 * tid + 1] = e + v0;
        hist[4 * tid + 2] = e + v0 + v1;
        hist[4 * tid + 3] = e + v0 + v1 + v2;
    }
    __syncthreads();
    for (int i = tid; i < n; i += kThreads) {
        uint32_t pos = atomicAdd(&hist[cell_of(i)], 1u);
        W.x[pos] = p[3 * i];
        W.y[pos] = p[3 * i + 1];
        W.z[pos] = p[3 * i + 2];
        W.d[pos] = INFINITY;
        W.idx[pos] = (uint32_t)i;
    }
    __threadfence_block();
    __syncthreads();

    // ---- per-bucket state in the owner lane: bucket = wave + 16 * (q * 64 + lane)
    const int nb = (n + 63) / 64;
    float bmin[BPL][3], bmax[BPL][3], bx[BPL][3];
    uint64_t bkey[BPL];
#pragma unroll
    for (int q = 0; q < BPL; ++q) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            bmin[q][a] = INFINITY;
            bmax[q][a] = -INFINITY;
            bx[q][a] = 0.0f;
        }
        bkey[q] = 0;  // dist 0: never active, never the argmax
        for (int bb = 0; bb < 64; ++bb) {
            int bucket = wave + kWaves * (q * 64 + bb);
            if (bucket >= nb) break;  // wave-uniform
            int pos = bucket * 64 + lane;
            float v[3] = {INFINITY, INFINITY, INFINITY}, u[3] = {-INFINITY, -INFINITY, -INFINITY};
            if (pos < n) {
                v[0] = u[0] = W.x[pos];
                v[1] = u[1] = W.y[pos];
                v[2] = u[2] = W.z[pos];
            }
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                v[a] = lidar::wave_min_f(v[a]);
                u[a] = lidar::wave_max_f(u[a]);
            }
            if (lane == bb) {
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    bmin[q][a] = v[a];
                    bmax[q][a] = u[a];
                }
                bkey[q] = lidar::make_key(INFINITY, 0u);
            }
        }
    }

    // ---- sample 0 is index 0
    float qx = p[0], qy = p[1], qz = p[2];
    if (tid == 0) {
        out_idx[(int64_t)b * npoint] = 0;
        if (out_xyz) {
            float *o = out_xyz + (int64_t)b * npoint * 3;
            o[0] = qx;
            o[1] = qy;
            o[2] = qz;
        }
    }

    for (int it = 1; it < npoint; ++it) {
#pragma unroll
        for (int q = 0; q < BPL; ++q) {
            float gx = gap(qx, bmin[q][0], bmax[q][0]);
            float gy = gap(qy, bmin[q][1], bmax[q][1]);
            float gz = gap(qz, bmin[q][2], bmax[q][2]);
            float lb = __fadd_rn(__fadd_rn(__fmul_rn(gx, gx), __fmul_rn(gy, gy)), __fmul_rn(gz, gz));
            bool active = lb < lidar::key_dist(bkey[q]);
            uint64_t mask = __ballot(active);
            while (mask) {
                int bb = __ffsll((unsigned long long)mask) - 1;
                mask &= mask - 1;
                int bucket = wave + kWaves * (q * 64 + bb);
                int pos = bucket * 64 + lane;
                uint64_t key = 0;
                float px = 0.f, py = 0.f, pz = 0.f;
                if (pos < n) {
                    px = W.x[pos];
                    py = W.y[pos];
                    pz = W.z[pos];
                    float od = W.d[pos];
                    float d = lidar::dist2f(px, py, pz, qx, qy, qz);
                    if (d < od) {
                        W.d[pos] = d;
                        od = d;
                    }
                    key = lidar::make_key(od, W.idx[pos]);
                }
                uint64_t km = lidar::wave_max_u64(key);
                int wl = __ffsll((unsigned long long)__ballot(key == km)) - 1;
                float wx = __shfl(px, wl, 64), wy = __shfl(py, wl, 64), wz = __shfl(pz, wl, 64);
                if (lane == bb) {
                    bkey[q] = km;
                    bx[q][0] = wx;
                    bx[q][1] = wy;
                    bx[q][2] = wz;
                }
            }
        }
        // frame argmax over bucket keys
        uint64_t best = bkey[0];
        float cx = bx[0][0], cy = bx[0][1], cz = bx[0][2];
#pragma unroll
        for (int q = 1; q < BPL; ++q) {
            if (bkey[q] > best) {
                best = bkey[q];
                cx = bx[q][0];
                cy = bx[q][1];
                cz = bx[q][2];
            }
        }
        uint64_t wm = lidar::wave_max_u64(best);
        const int par = it & 1;
        const int first = __ffsll((unsigned long long)__ballot(best == wm)) - 1;
        if (lane == first) {
            skey[par][wave] = wm;
            sxyz[par][wave][0] = cx;
            sxyz[par][wave][1] = cy;
            sxyz[par][wave][2] = cz;
        }
        __syncthreads();
        uint64_t g = skey[par][0];
        int gw = 0;
#pragma unroll
        for (int w = 1; w < kWaves; ++w) {
            uint64_t k = skey[par][w];
            if (k > g) {
                g = k;
                gw = w;
            }
        }
        qx = sxyz[par][gw][0];
        qy = sxyz[par][gw][1];
        qz = sxyz[par][gw][2];
        if (tid == 0) {
            out_idx[(int64_t)b * npoint + it] = (int32_t)lidar::key_index(g);
            if (out_xyz) {
                float *o = out_xyz + ((int64_t)b * npoint + it) * 3;
                o[0] = qx;
                o[1] = qy;
                o[2] = qz;
            }
        }
    }
}

}  // namespace

LIDAR_EXPORT int lidar_fps_f32(lidar_handle *h, const float *xyz, int64_t batch, int64_t n,
                               int64_t npoint, int32_t *idx, float *new_xyz, void *stream)
{
    REQUIRE(h && xyz && idx, "lidar_fps_f32: null pointer");
    REQUIRE(batch >= 0 && n >= 1 && npoint >= 1, "lidar_fps_f32: need n >= 1 and npoint >= 1");
    REQUIRE(n <= 4 * 65536, "lidar_fps_f32: n > 262144 points per frame");
    REQUIRE(batch <= 0x7fffffff, "lidar_fps_f32: batch too large");
    if (batch == 0) return LIDAR_OK;
    HIP_TRY(hipSetDevice(h->device));
    int64_t stride = lidar::align_up(5 * n, 64);
    float *ws = static_cast<float *>(lidar::workspace(h, (uint64_t)(batch * stride) * 4));
    if (!ws) return LIDAR_ENOMEM;
    hipStream_t s = static_cast<hipStream_t>(stream);
    dim3 grid((unsigned)batch), block(kThreads);
    int nb = (int)((n + 63) / 64);
    if (nb <= 1024)
        hipLaunchKernelGGL(fps_bucket_kernel<1>, grid, block, 0, s, xyz, (int)n, (int)npoint, idx,
                           new_xyz, ws, stride);
    else if (nb <= 2048)
        hipLaunchKernelGGL(fps_bucket_kernel<2>, grid, block, 0, s, xyz, (int)n, (int)npoint, idx,
                           new_xyz, ws, stride);
    else
        hipLaunchKernelGGL(fps_bucket_kernel<4>, grid, block, 0, s, xyz, (int)n, (int)npoint, idx,
                           new_xyz, ws, stride);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
