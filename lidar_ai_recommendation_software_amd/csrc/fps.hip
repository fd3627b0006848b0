// fps.hip — farthest-point sampling on gfx950, exact, bucket-pruned.
//
// Spec (oracle/lidar_oracle.c orc_fps): idx[0] = 0, dist = +inf,
// then npoint-1 times: dist = min(dist, d(., last)), last = argmax dist (lowest index
// on ties), d = (dx*dx + dy*dy) + dz*dz in fp32 with one rounding per operation.
//
// One 1024-thread workgroup per frame.  Prologue: frame bbox, counting sort of the
// points by a 16^3 Morton cell into a sorted copy in the workspace ((x, y, z,
// original index) float4s + a separate dist array), cut into buckets of 64 consecutive sorted points (one
// wavefront-width each).  Every bucket keeps, in the registers of its owner lane,
// its bounding box and its (max dist, index) key and the coordinates of that point.
//
// Step: a bucket can only change if some member gets closer to the new sample than
// its current dist.  lb = dist-from-bbox(q) computed with the SAME rounded operations
// as d is a lower bound of every member's d (fl() is monotone), so `lb >= bucket max`
// proves no member changes and the bucket is skipped — an exact pruning, not an
// approximation.  Active buckets are streamed (64 lanes = 64 points, one coalesced float4
// (x, y, z, dist) load each, up to 4 buckets' loads in flight together; the workspace is
// padded to whole buckets with dist -1 sentinels so the batch is branch-free), updated,
// and re-reduced with DPP argmax reductions (max dist, lowest index on ties).  A wave
// whose buckets changed recomputes its DPP argmax; every wave then submits
// (dist bits << 32 | (2^27 - index) << 4 | wave) to ONE LDS 64-bit atomic max and its
// coordinates to a per-wave slot, so the frame argmax costs a single barrier per step.
//
// Nested FPS (SA2 samples SA1's centroids): FPS over the first m points of an FPS ordering
// is the identity 0..m-1 while the parent's winning distance stayed > 0 — the parent
// run records the first step whose winning distance was 0 (`first_zero`), the child run
// takes it as `prefix_ok` and copies the prefix when m <= prefix_ok.
#include <algorithm>
#include <atomic>

#include "common.hpp"

namespace {

#ifndef FPS_THREADS
#define FPS_THREADS 1024
#endif
// default workgroup size: 16 waves (active-bucket updates and their reductions run in parallel
// across waves; the merge is an LDS atomic max).  lidar_fps_ex_f32 also offers 512 (8 waves,
// 2 buckets per lane: ~25 % longer steps, half the CU footprint beside other kernels)
constexpr int kThreads = FPS_THREADS;
// FPS_MAXK: the most active buckets of one owner slot updated per memory round trip (A/B builds: fewer
// means fewer registers)
#ifndef FPS_MAXK
#define FPS_MAXK 4
#endif
// one point per lane: 8 bucket slots per lane of a 512-thread workgroup (the register budget) hold
// 262 144 points; larger frames take buckets of 64 x PPL points (PPL 2 .. 16: up to 4 Mi points)
constexpr int64_t kMaxBucketPoints = 8 * 512 * 64;
constexpr int64_t kMaxFpsPoints = 16 * kMaxBucketPoints;
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
    float4 *p;  // sorted (x, y, z, original index bits): read-only after the prologue
    float *d;   // running min distance of each sorted point: the only per-step store, so an
                // update dirties 2 cache lines per bucket, not 8 (the L2 holds ~4 frames per XCD)
};

// distance from q to [lo, hi] along one axis: lo - q below, q - hi above, else 0 — as
// max3(lo - q, q - hi, 0) (one of the two differences is <= 0 whenever the other is > 0)
__device__ __forceinline__ float gap(float q, float lo, float hi)
{
    return fmaxf(fmaxf(__fsub_rn(lo, q), __fsub_rn(q, hi)), 0.0f);
}

// Update K active buckets of one owner slot (their loads issued together, their DPP
// reductions interleaved): new distances against q, bucket max + its lowest-index argmax
// point into the owner lane's registers.  A bucket is 64 lanes x PPL points (lane l holds the
// bucket's points j * 64 + l: coalesced per j); bp encodes the argmax member as j * 64 + lane.
template <int K, int NW, int PPL = 1>
__device__ __forceinline__ void update_batch(uint64_t &mask, const FrameWs &W, int wave, int q, int lane,
                                             float qx, float qy, float qz, float &bd, uint32_t &bi, float *bx,
                                             int &bp, int target, bool &hit)
{
    // branch-free: the workspace is padded to whole buckets with sentinel points
    // (dist -1: never the max, never updated since every real d >= 0)
    int bbs[K];
    uint32_t pos[K];  // unsigned: the loads take the SGPR base + 32-bit offset form
    float4 P[K][PPL];
    float D[K][PPL];
#pragma unroll
    for (int u = 0; u < K; ++u) {
        bbs[u] = __ffsll((unsigned long long)mask) - 1;
        mask &= mask - 1;
        pos[u] = (uint32_t)((wave + NW * (q * 64 + bbs[u])) * 64 * PPL + lane);
    }
#pragma unroll
    for (int u = 0; u < K; ++u)
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
            P[u][j] = W.p[pos[u] + 64 * j];
            D[u][j] = W.d[pos[u] + 64 * j];
        }
    // distances in bit space (>= +0 or the -1 sentinel: signed int order = float order); per lane
    // the best of its PPL points (max dist, lowest index)
    int od[K], dm[K], lj[K];
    uint32_t I[K];
    // a bucket's key (max dist, lowest index) can only change if its argmax member got
    // closer: distances only decrease, so with that member untouched the max and its
    // lowest-index holder stand — the reduction is skipped (bp = the member, -1 unknown)
    bool redo[K];
#pragma unroll
    for (int u = 0; u < K; ++u) {
        od[u] = -1;
        I[u] = 0xffffffffu;
        lj[u] = 0;
        uint64_t chm = 0;
        const int bpu = __builtin_amdgcn_readlane(bp, bbs[u]);
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
            // d >= +0 or NaN; the sign bit cleared, a NaN d (inf - inf) orders above every dist and never
            // replaces one, as in the oracle (a bare bit compare let a negative NaN in)
            const int db = __float_as_int(lidar::dist2f(P[u][j].x, P[u][j].y, P[u][j].z, qx, qy, qz)) & 0x7fffffff;
            const int o = min(db, __float_as_int(D[u][j]));
            const bool lower = o != __float_as_int(D[u][j]);
            if (lower) W.d[pos[u] + 64 * j] = __int_as_float(o);  // only changed members dirty a line
            const uint64_t ch = __ballot(lower);
            if (PPL == 1 || (bpu >> 6) == j) chm = ch;
            const uint32_t ij = __float_as_uint(P[u][j].w);
            if (PPL == 1 || o > od[u] || (o == od[u] && ij < I[u])) {
                od[u] = o;
                I[u] = ij;
                lj[u] = j;
            }
        }
        redo[u] = bpu < 0 || ((chm >> (bpu & 63)) & 1ull);
    }
#pragma unroll
    for (int u = 0; u < K; ++u) {
        dm[u] = 0;
        if (redo[u]) dm[u] = lidar::wave_max_i32_dpp(od[u]);  // wave-uniform
    }
#pragma unroll
    for (int u = 0; u < K; ++u) {
        if (!redo[u]) continue;  // wave-uniform
        hit = hit || bbs[u] == target;
        const uint64_t c = __ballot(od[u] == dm[u]);
        int wl;
        if (__popcll(c) == 1) {
            wl = __ffsll((unsigned long long)c) - 1;
        } else {
            const uint32_t mi = lidar::wave_min_u32_dpp(od[u] == dm[u] ? I[u] : 0xffffffffu);
            wl = __ffsll((unsigned long long)__ballot(od[u] == dm[u] && I[u] == mi)) - 1;
        }
        float4 pb = P[u][0];
#pragma unroll
        for (int j = 1; j < PPL; ++j)
            if (lj[u] == j) pb = P[u][j];
        const uint32_t wi = (uint32_t)__builtin_amdgcn_readlane((int)I[u], wl);
        const float wx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pb.x), wl));
        const float wy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pb.y), wl));
        const float wz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pb.z), wl));
        const int wj = PPL == 1 ? 0 : __builtin_amdgcn_readlane(lj[u], wl);
        const bool me = lane == bbs[u];
        bp = me ? wj * 64 + wl : bp;
        bd = me ? __int_as_float(dm[u]) : bd;
        bi = me ? wi : bi;
        bx[0] = me ? wx : bx[0];
        bx[1] = me ? wy : bx[1];
        bx[2] = me ? wz : bx[2];
    }
}

__device__ __forceinline__ uint64_t stamp()
{
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// Prologue of one frame, run by the whole workgroup: frame bbox, counting sort of the points
// by 16^3 Morton cell into W (padded to whole buckets with dist -1 sentinels).  Ends with a
// barrier (hist is free afterwards).
template <int T>
__device__ __forceinline__ void fps_prologue(const float *__restrict__ p, int n, int npad, const FrameWs &W,
                                             uint32_t *hist, float (*red)[T / 64], uint32_t *wsum)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // ---- frame bounding box
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = tid; i < n; i += T) {
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
    for (int c = tid; c < kCells; c += T) hist[c] = 0;
    __syncthreads();
    float scale[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float l = red[a][0], h = red[3 + a][0];
        for (int w = 1; w < (T / 64); ++w) {
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
    for (int i = tid; i < n; i += T) atomicAdd(&hist[cell_of(i)], 1u);
    __syncthreads();
    {  // exclusive scan of the cell counts, kCells / T consecutive cells per thread
        constexpr int per = kCells / T;
        uint32_t v[per], s = 0;
#pragma unroll
        for (int j = 0; j < per; ++j) {
            v[j] = hist[per * tid + j];
            s += v[j];
        }
        uint32_t incl = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t t = __shfl_up(incl, o, 64);
            if (lane >= o) incl += t;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t e = incl - s;
        for (int w = 0; w < wave; ++w) e += wsum[w];
#pragma unroll
        for (int j = 0; j < per; ++j) {
            hist[per * tid + j] = e;
            e += v[j];
        }
    }
    __syncthreads();
    for (int i = tid; i < n; i += T) {
        uint32_t pos = atomicAdd(&hist[cell_of(i)], 1u);
        W.p[pos] = make_float4(p[3 * i], p[3 * i + 1], p[3 * i + 2], __uint_as_float((uint32_t)i));
        W.d[pos] = INFINITY;
    }
    for (int i = n + tid; i < npad; i += T) {
        W.p[i] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(0xffffffffu));
        W.d[i] = -1.0f;
    }
    __threadfence_block();
    __syncthreads();

}
// DIAG builds (lidar_diag_fps_phases only) accumulate per-phase shader cycles per wave:
// [0] bucket tests + active-bucket updates, [1] wave argmax + LDS publish, [2] barrier
// wait, [3] 16-way merge, [4] active-bucket batches processed, [5] steps
template <int T, int BPL, bool DIAG = false, int PPL = 1>
__global__ __launch_bounds__(T) void fps_bucket_kernel(const float *__restrict__ xyz,
                                                              int n, int npoint,
                                                              int32_t *__restrict__ out_idx,
                                                              float *__restrict__ out_xyz,
                                                              int32_t *__restrict__ first_zero,
                                                              const int32_t *__restrict__ prefix_ok,
                                                              float *__restrict__ ws, int64_t ws_stride,
                                                              uint64_t *__restrict__ diag = nullptr)
{
    uint64_t dacc[6] = {0, 0, 0, 0, 0, 0};
    uint64_t t0 = 0, t1 = 0;
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const float *p = xyz + (int64_t)b * n * 3;

    // nested FPS shortcut: FPS over the first m points of an FPS ordering returns 0..m-1
    // as long as the parent's winning distance stayed > 0 — exact.
    if (prefix_ok != nullptr && prefix_ok[b] >= npoint) {
        for (int i = tid; i < npoint; i += T) {
            out_idx[(int64_t)b * npoint + i] = i;
            if (out_xyz) {
                float *o = out_xyz + ((int64_t)b * npoint + i) * 3;
                o[0] = p[3 * i];
                o[1] = p[3 * i + 1];
                o[2] = p[3 * i + 2];
            }
        }
        if (first_zero && tid == 0) first_zero[b] = prefix_ok[b];
        return;
    }

    float *wsb = ws + (int64_t)b * ws_stride;
    const int npad = (n + 64 * PPL - 1) / (64 * PPL) * (64 * PPL);  // whole buckets; the tail holds sentinels
    FrameWs W{reinterpret_cast<float4 *>(wsb), wsb + 4 * (int64_t)npad};

    __shared__ uint32_t hist[kCells];
    __shared__ float red[6][(T / 64)];
    __shared__ uint32_t wsum[(T / 64)];
    // per-step merge: every wave submits its argmax as one 64-bit key to an LDS atomic max
    // (triple-buffered so a slot is cleared two barriers after its last read) and its
    // coordinates to a per-wave slot (double-buffered); one barrier per step
    __shared__ unsigned long long mkey[3];
    __shared__ __attribute__((aligned(16))) float mcrd[2][(T / 64)][4];

    fps_prologue<T>(p, n, npad, W, hist, red, wsum);
    const int nb = npad / (64 * PPL);
        // ---- per-bucket state in the owner lane: bucket = wave + 4 * (q * 64 + lane)
    float bmin[BPL][3], bmax[BPL][3], bx[BPL][3], bd[BPL];
    uint32_t bi[BPL];
    int bp[BPL];  // lane (within the bucket) of the bucket's argmax member; -1 until reduced
#pragma unroll
    for (int q = 0; q < BPL; ++q)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            bmin[q][a] = INFINITY;
            bmax[q][a] = -INFINITY;
        }
    // bucket bounding boxes: every wave reduces 64-point buckets into a table in the (now free)
    // hist array, 512 buckets per pass (12 KiB), and the owner lanes pick theirs up — no LDS is
    // held for it through the step loop (the kernel's LDS stays ~17 KiB beside other kernels)
    float *tab = reinterpret_cast<float *>(hist);
    static_assert(kCells >= 512 * 6, "bbox pass table");
    for (int p0 = 0; p0 < nb; p0 += 512) {
        for (int bucket = p0 + wave; bucket < nb && bucket < p0 + 512; bucket += (T / 64)) {
            float v[3] = {INFINITY, INFINITY, INFINITY}, u[3] = {-INFINITY, -INFINITY, -INFINITY};
#pragma unroll
            for (int j = 0; j < PPL; ++j) {
                const int pos = (bucket * PPL + j) * 64 + lane;
                if (pos < n) {
                    const float4 P = W.p[pos];
                    v[0] = fminf(v[0], P.x);
                    v[1] = fminf(v[1], P.y);
                    v[2] = fminf(v[2], P.z);
                    u[0] = fmaxf(u[0], P.x);
                    u[1] = fmaxf(u[1], P.y);
                    u[2] = fmaxf(u[2], P.z);
                }
            }
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                v[a] = lidar::wave_min_f(v[a]);
                u[a] = lidar::wave_max_f(u[a]);
            }
            if (lane == 0) {
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    tab[(bucket - p0) * 6 + a] = v[a];
                    tab[(bucket - p0) * 6 + 3 + a] = u[a];
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < BPL; ++q) {
            const int bucket = wave + (T / 64) * (q * 64 + lane);
            if (bucket >= p0 && bucket < p0 + 512 && bucket < nb)
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    bmin[q][a] = tab[(bucket - p0) * 6 + a];
                    bmax[q][a] = tab[(bucket - p0) * 6 + 3 + a];
                }
        }
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < BPL; ++q) {
        const int bucket = wave + (T / 64) * (q * 64 + lane);
        const bool have = bucket < nb;
#pragma unroll
        for (int a = 0; a < 3; ++a) bx[q][a] = 0.0f;
        bp[q] = -1;
        bd[q] = have ? INFINITY : 0.0f;  // empty slot: never active, never the argmax
        bi[q] = have ? 0u : 0xffffffffu;
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
    int zero_at = npoint;  // first step whose winning distance is 0

    float w_d = 0.0f, w_x = 0.0f, w_y = 0.0f, w_z = 0.0f;  // this wave's current argmax
    uint32_t w_i = 0xffffffffu;
    if (tid < 3) mkey[tid] = 0ull;
    __syncthreads();
    int cur3 = 1, nxt3 = 2;
    // the wave's argmax bucket (slot w_q of lane w_lane): updates only lower bucket keys (max
    // dist, then lowest index), so while that bucket is untouched the wave argmax stands
    int w_q = 0, w_lane = 0;
    for (int it = 1; it < npoint; ++it) {
        bool wave_dirty = it == 1;
        if constexpr (DIAG) {
            __builtin_amdgcn_sched_barrier(0);
            t0 = stamp();
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int q = 0; q < BPL; ++q) {
            const float gx = gap(qx, bmin[q][0], bmax[q][0]);
            const float gy = gap(qy, bmin[q][1], bmax[q][1]);
            const float gz = gap(qz, bmin[q][2], bmax[q][2]);
            const float lb = __fadd_rn(__fadd_rn(__fmul_rn(gx, gx), __fmul_rn(gy, gy)), __fmul_rn(gz, gz));
            uint64_t mask = __ballot(lb < bd[q]);
            // the wave argmax is recomputed only when its bucket's key changed
            const int target = q == w_q ? w_lane : -1;
            while (mask) {  // wave-uniform
                if constexpr (DIAG) dacc[4]++;
                const int cnt = __popcll(mask);
                // up to 4 loads per lane in flight: K buckets of PPL points
                if (PPL == 1 && FPS_MAXK >= 4 && cnt >= 4)
                    update_batch<4, T / 64, PPL>(mask, W, wave, q, lane, qx, qy, qz, bd[q], bi[q], bx[q], bp[q],
                                                 target, wave_dirty);
                else if (PPL == 1 && FPS_MAXK >= 3 && cnt == 3)  // one round trip instead of 2 + 1
                    update_batch<3, T / 64, PPL>(mask, W, wave, q, lane, qx, qy, qz, bd[q], bi[q], bx[q], bp[q],
                                                 target, wave_dirty);
                else if (PPL <= 2 && cnt >= 2)
                    update_batch<2, T / 64, PPL>(mask, W, wave, q, lane, qx, qy, qz, bd[q], bi[q], bx[q], bp[q],
                                                 target, wave_dirty);
                else
                    update_batch<1, T / 64, PPL>(mask, W, wave, q, lane, qx, qy, qz, bd[q], bi[q], bx[q], bp[q],
                                                 target, wave_dirty);
            }
        }
        if constexpr (DIAG) {
            __builtin_amdgcn_sched_barrier(0);
            t1 = stamp();
            dacc[0] += t1 - t0;
            t0 = t1;
            __builtin_amdgcn_sched_barrier(0);
        }
        // frame argmax: lane best over its buckets -> wave argmax (DPP, only when the wave's
        // argmax bucket was touched) -> LDS atomic max of the packed key -> barrier -> broadcast
        if (wave_dirty) {
            float best = bd[0];
            uint32_t besti = bi[0];
            float cx = bx[0][0], cy = bx[0][1], cz = bx[0][2];
            int bq = 0;
#pragma unroll
            for (int q = 1; q < BPL; ++q) {
                if (bd[q] > best || (bd[q] == best && bi[q] < besti)) {
                    best = bd[q];
                    besti = bi[q];
                    cx = bx[q][0];
                    cy = bx[q][1];
                    cz = bx[q][2];
                    bq = q;
                }
            }
            int wdb;
            const int wl = lidar::wave_argmax_lane_i32(__float_as_int(best), besti, &wdb);
            w_d = __int_as_float(wdb);
            w_i = (uint32_t)__builtin_amdgcn_readlane((int)besti, wl);
            w_x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cx), wl));
            w_y = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cy), wl));
            w_z = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cz), wl));
            w_lane = wl;
            w_q = BPL > 1 ? __builtin_amdgcn_readlane(bq, wl) : 0;
        }
        if constexpr (DIAG) {
            __builtin_amdgcn_sched_barrier(0);
            t1 = stamp();
            dacc[1] += t1 - t0;
            t0 = t1;
            __builtin_amdgcn_sched_barrier(0);
        }
        // key: dist bits (d >= 0 orders as unsigned) | (2^27 - idx) << 4 | wave; a larger key
        // is a larger distance, then a smaller index (n <= 2^27); empty slots carry field 0
        const int slot = cur3, cslot = it & 1;
        if (lane == 0) {
            const uint32_t fld = w_i < (1u << 27) ? (1u << 27) - w_i : 0u;
            const unsigned long long key =
                ((unsigned long long)__float_as_uint(w_d) << 32) | (fld << 4) | (uint32_t)wave;
            mcrd[cslot][wave][0] = w_x;
            mcrd[cslot][wave][1] = w_y;
            mcrd[cslot][wave][2] = w_z;
            atomicMax(&mkey[slot], key);
        }
        if (tid == 0) mkey[nxt3] = 0ull;  // step it+1's slot, last read before the previous barrier
        __syncthreads();
        if constexpr (DIAG) {
            __builtin_amdgcn_sched_barrier(0);
            t1 = stamp();
            dacc[2] += t1 - t0;
            t0 = t1;
            __builtin_amdgcn_sched_barrier(0);
        }
        {
            // the winner's key and every wave's candidate coordinates are read side by side
            // (lane l < 16 reads wave l's slot); the winner's come back by readlane — one
            // LDS round trip after the barrier instead of two dependent ones
            const unsigned long long key = mkey[slot];
            float4 cand = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (lane < (T / 64))  // 16 lanes read: 256 B per wave instead of 1 KiB of LDS traffic
                cand = *reinterpret_cast<const float4 *>(mcrd[cslot][lane]);
            const int ww = __builtin_amdgcn_readfirstlane((int)(key & 15u));
            const float gdist = __uint_as_float((uint32_t)(key >> 32));
            const uint32_t gidx = (1u << 27) - (((uint32_t)key) >> 4);
            qx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cand.x), ww));
            qy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cand.y), ww));
            qz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cand.z), ww));
            if (tid == 0) {
                out_idx[(int64_t)b * npoint + it] = (int32_t)gidx;
                if (out_xyz) {
                    float *o = out_xyz + ((int64_t)b * npoint + it) * 3;
                    o[0] = qx;
                    o[1] = qy;
                    o[2] = qz;
                }
            }
            if (zero_at == npoint && gdist == 0.0f) zero_at = it;
        }
        cur3 = nxt3;
        nxt3 = nxt3 == 2 ? 0 : nxt3 + 1;
        if constexpr (DIAG) {
            __builtin_amdgcn_sched_barrier(0);
            t1 = stamp();
            dacc[3] += t1 - t0;
            dacc[5]++;
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (first_zero && tid == 0) first_zero[b] = zero_at;
    if constexpr (DIAG) {
        if (lane == 0)
            for (int k = 0; k < 6; ++k) diag[((int64_t)b * (T / 64) + wave) * 6 + k] = dacc[k];
    }
}


}  // namespace

#ifdef LIDAR_DIAG
// diagnostic build only: phase stamps of the SA1 FPS launches a pipeline issues (lidar_diag_fps_record).
// Every 512-thread, one-point-per-lane launch without prefix_ok (SA1, not SA2's nested FPS) of n <= 65 536
// points takes the DIAG instantiation and appends its per-(frame, wave) phase totals (6 words, as
// lidar_diag_fps_eager512_phases) to the registered buffer while it has room.
static uint64_t *g_fps_rec = nullptr;
static int64_t g_fps_rec_cap = 0;
static std::atomic<int64_t> g_fps_rec_used{0};
#endif

template <int T>
static int launch_fps(const float *xyz, int64_t batch, int64_t n, int64_t npoint, int32_t *idx, float *new_xyz,
                      int32_t *first_zero, const int32_t *prefix_ok, float *ws, int64_t stride, hipStream_t s)
{
    dim3 grid((unsigned)batch), block(T);
    const int nb = (int)((n + 63) / 64);
    const int lanes = T;  // one bucket per lane and slot
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, block, 0, s, xyz, (int)n, (int)npoint, idx, new_xyz, first_zero, prefix_ok, ws,
                           stride, nullptr);
    };
    if (n > kMaxBucketPoints) {
        // large frames: 8 bucket slots per lane at 512 threads, each bucket 64 x PPL points
        // (lidar_fps_ex_f32 sends every n > kMaxBucketPoints here with T = 512)
        if constexpr (T == 512) {
            const int64_t ppl = (n + kMaxBucketPoints - 1) / kMaxBucketPoints;
            if (ppl <= 2) go(fps_bucket_kernel<T, 8, false, 2>);
            else if (ppl <= 4) go(fps_bucket_kernel<T, 8, false, 4>);
            else if (ppl <= 8) go(fps_bucket_kernel<T, 8, false, 8>);
            else go(fps_bucket_kernel<T, 8, false, 16>);
        }
    } else {
#ifdef LIDAR_DIAG
        if constexpr (T == 512) {
            if (g_fps_rec && prefix_ok == nullptr && nb <= 2 * lanes) {
                const int64_t need = batch * (T / 64) * 6;
                const int64_t off = g_fps_rec_used.fetch_add(need);
                if (off + need <= g_fps_rec_cap) {
                    auto god = [&](auto kern) {
                        hipLaunchKernelGGL(kern, grid, block, 0, s, xyz, (int)n, (int)npoint, idx, new_xyz, first_zero,
                                           prefix_ok, ws, stride, g_fps_rec + off);
                    };
                    if (nb <= lanes) god(fps_bucket_kernel<T, 1, true>);
                    else god(fps_bucket_kernel<T, 2, true>);
                    LAUNCH_CHECK();
                    return LIDAR_OK;
                }
            }
        }
#endif
        if (nb <= lanes) go(fps_bucket_kernel<T, 1>);
        else if (nb <= 2 * lanes) go(fps_bucket_kernel<T, 2>);
        else if (nb <= 4 * lanes) go(fps_bucket_kernel<T, 4>);
        else go(fps_bucket_kernel<T, 8>);
    }
    LAUNCH_CHECK();
    return LIDAR_OK;
}

// workspace bytes lidar_fps_f32 / lidar_fps_ex_f32 take from the handle for (batch, n)
static int64_t fps_stride(int64_t n)  // floats per frame: (x, y, z, index) + dist over whole buckets
{
    const int64_t unit = n > kMaxBucketPoints ? 64 * 16 : 64;
    return lidar::align_up(5 * lidar::align_up(n, unit), 64);
}

LIDAR_EXPORT uint64_t lidar_fps_workspace_bytes(int64_t batch, int64_t n)
{
    return (uint64_t)(batch * fps_stride(n)) * 4;
}

// threads: workgroup size per frame, 0 (the build default, 1024), 1024 or 512 — same results
LIDAR_EXPORT int lidar_fps_ex_f32(lidar_handle *h, const float *xyz, int64_t batch, int64_t n, int64_t npoint,
                                  int32_t *idx, float *new_xyz, int32_t *first_zero, const int32_t *prefix_ok,
                                  int32_t threads, void *stream)
{
    REQUIRE(h && xyz && idx, "lidar_fps_f32: null pointer");
    REQUIRE(batch >= 0 && n >= 1 && npoint >= 1, "lidar_fps_f32: need n >= 1 and npoint >= 1");
    REQUIRE(n <= kMaxFpsPoints, "lidar_fps_f32: n > 4194304 points per frame");
    if (threads == 0) threads = kThreads;
    REQUIRE(threads == 1024 || threads == 512, "lidar_fps_ex_f32: threads must be 0, 512 or 1024");
    if (n > kMaxBucketPoints) threads = 512;  // the large-frame kernel: 512 threads
    REQUIRE(n > kMaxBucketPoints || (n + 63) / 64 <= 8 * (int64_t)threads,
            "lidar_fps_f32: too many buckets for this workgroup size");
    REQUIRE(batch <= 0x7fffffff, "lidar_fps_f32: batch too large");
    if (batch == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    REQUIRE(prefix_ok == nullptr || npoint <= n, "lidar_fps_f32: prefix_ok needs npoint <= n");
    const int64_t stride = fps_stride(n);
    float *ws = static_cast<float *>(lidar::workspace(h, (uint64_t)(batch * stride) * 4));
    if (!ws) return LIDAR_ENOMEM;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (threads == 512)
        return launch_fps<512>(xyz, batch, n, npoint, idx, new_xyz, first_zero, prefix_ok, ws, stride, s);
    return launch_fps<1024>(xyz, batch, n, npoint, idx, new_xyz, first_zero, prefix_ok, ws, stride, s);
}

LIDAR_EXPORT int lidar_fps_f32(lidar_handle *h, const float *xyz, int64_t batch, int64_t n, int64_t npoint,
                               int32_t *idx, float *new_xyz, int32_t *first_zero, const int32_t *prefix_ok,
                               void *stream)
{
    return lidar_fps_ex_f32(h, xyz, batch, n, npoint, idx, new_xyz, first_zero, prefix_ok, 0, stream);
}

#ifdef LIDAR_DIAG
// diagnostic build only (`make diag`, not part of the product library or ABI): per-wave phase cycle
// totals of one FPS run
// register (buf, cap_words) for the SA1 FPS launches' phase records (buf NULL: stop); returns 0
LIDAR_EXPORT int lidar_diag_fps_record(uint64_t *buf, int64_t cap_words)
{
    g_fps_rec = buf;
    g_fps_rec_cap = buf ? cap_words : 0;
    g_fps_rec_used = 0;
    return LIDAR_OK;
}
// words the registered buffer has received so far (launches past its capacity ran unstamped)
LIDAR_EXPORT int64_t lidar_diag_fps_recorded(void) { return std::min<int64_t>(g_fps_rec_used, g_fps_rec_cap); }

// the eager kernel's phases at 512 threads (BPL from n), diag[(frame * 8 + wave) * 6 + k]
LIDAR_EXPORT int lidar_diag_fps_eager512_phases(lidar_handle *h, const float *xyz, int64_t batch, int64_t n,
                                                int64_t npoint, int32_t *idx, uint64_t *diag, void *stream)
{
    REQUIRE(h && xyz && idx && diag && n <= 65536 && n >= 1 && npoint >= 1, "lidar_diag_fps_eager512_phases: bad args");
    ON_DEVICE(h->device);
    int64_t stride = lidar::align_up(5 * lidar::align_up(n, 64), 64);
    float *ws = static_cast<float *>(lidar::workspace(h, (uint64_t)(batch * stride) * 4));
    if (!ws) return LIDAR_ENOMEM;
    const int nb = (int)((n + 63) / 64);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3((unsigned)batch), dim3(512), 0, static_cast<hipStream_t>(stream), xyz, (int)n,
                           (int)npoint, idx, nullptr, nullptr, nullptr, ws, stride, diag);
    };
    if (nb <= 512) go(fps_bucket_kernel<512, 1, true>);
    else go(fps_bucket_kernel<512, 2, true>);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

LIDAR_EXPORT int lidar_diag_fps_phases(lidar_handle *h, const float *xyz, int64_t batch, int64_t n,
                                       int64_t npoint, int32_t *idx, uint64_t *diag, void *stream)
{
    REQUIRE(h && xyz && idx && diag && n <= 65536 && n >= 1 && npoint >= 1, "lidar_diag_fps_phases: bad args");
    ON_DEVICE(h->device);
    int64_t stride = lidar::align_up(5 * lidar::align_up(n, 64), 64);
    float *ws = static_cast<float *>(lidar::workspace(h, (uint64_t)(batch * stride) * 4));
    if (!ws) return LIDAR_ENOMEM;
    REQUIRE((n + 63) / 64 <= kThreads, "lidar_diag_fps_phases: n too large for BPL=1");
    hipLaunchKernelGGL((fps_bucket_kernel<kThreads, 1, true>), dim3((unsigned)batch), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), xyz, (int)n, (int)npoint, idx, nullptr, nullptr,
                       nullptr, ws, stride, diag);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
#endif
