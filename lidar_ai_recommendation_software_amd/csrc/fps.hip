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
// (dist bits << 32 | (2^18 - index) << 4 | wave) to ONE LDS 64-bit atomic max and its
// coordinates to a per-wave slot, so the frame argmax costs a single barrier per step.
//
// Nested FPS (SA2 samples SA1's centroids): FPS over the first m points of an FPS ordering
// is the identity 0..m-1 while the parent's winning distance stayed > 0 — the parent
// run records the first step whose winning distance was 0 (`first_zero`), the child run
// takes it as `prefix_ok` and copies the prefix when m <= prefix_ok.
#include <algorithm>

#include "common.hpp"

namespace {

#ifndef FPS_THREADS
#define FPS_THREADS 1024
#endif
// default workgroup size: 16 waves (active-bucket updates and their reductions run in parallel
// across waves; the merge is an LDS atomic max).  lidar_fps_ex_f32 also offers 512 (8 waves,
// 2 buckets per lane: ~25 % longer steps, half the CU footprint beside other kernels)
constexpr int kThreads = FPS_THREADS;
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
// point into the owner lane's registers.
template <int K, int NW>
__device__ __forceinline__ void update_batch(uint64_t &mask, const FrameWs &W, int wave, int q, int lane,
                                             float qx, float qy, float qz, float &bd, uint32_t &bi, float *bx,
                                             int &bp, int target, bool &hit)
{
    // branch-free: the workspace is padded to whole buckets with sentinel points
    // (dist -1: never the max, never updated since every real d >= 0)
    int bbs[K];
    uint32_t pos[K];  // unsigned: the loads take the SGPR base + 32-bit offset form
    float4 P[K];
    float D[K];
    uint32_t I[K];
#pragma unroll
    for (int u = 0; u < K; ++u) {
        bbs[u] = __ffsll((unsigned long long)mask) - 1;
        mask &= mask - 1;
        pos[u] = (uint32_t)((wave + NW * (q * 64 + bbs[u])) * 64 + lane);
    }
#pragma unroll
    for (int u = 0; u < K; ++u) {
        P[u] = W.p[pos[u]];
        D[u] = W.d[pos[u]];
    }
#pragma unroll
    for (int u = 0; u < K; ++u) I[u] = __float_as_uint(P[u].w);
    // distances in bit space (>= +0 or the -1 sentinel: signed int order = float order)
    int od[K], dm[K];
    // a bucket's key (max dist, lowest index) can only change if its argmax member got
    // closer: distances only decrease, so with that member untouched the max and its
    // lowest-index holder stand — the reduction is skipped (bp = the member's lane, -1 unknown)
    bool redo[K];
#pragma unroll
    for (int u = 0; u < K; ++u) {
        const float d = lidar::dist2f(P[u].x, P[u].y, P[u].z, qx, qy, qz);
        const bool lower = d < D[u];  // float order: a NaN d (inf - inf) never replaces a dist, as in the oracle
        od[u] = lower ? __float_as_int(d) : __float_as_int(D[u]);
        if (lower) W.d[pos[u]] = __int_as_float(od[u]);  // only changed members dirty a line
        const uint64_t ch = __ballot(lower);
        const int bpu = __builtin_amdgcn_readlane(bp, bbs[u]);
        redo[u] = bpu < 0 || ((ch >> bpu) & 1ull);
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
        const uint32_t wi = (uint32_t)__builtin_amdgcn_readlane((int)I[u], wl);
        const float wx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(P[u].x), wl));
        const float wy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(P[u].y), wl));
        const float wz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(P[u].z), wl));
        const bool me = lane == bbs[u];
        bp = me ? wl : bp;
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
__device__ __forceinline__ void fps_prologue(const float *__restrict__ p, int n, const FrameWs &W,
                                             uint32_t *hist, float (*red)[T / 64], uint32_t *wsum)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int npad = (n + 63) / 64 * 64;
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
template <int T, int BPL, bool DIAG = false>
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
    const int npad = (n + 63) / 64 * 64;  // whole buckets; the tail holds sentinel points
    FrameWs W{reinterpret_cast<float4 *>(wsb), wsb + 4 * (int64_t)npad};

    __shared__ uint32_t hist[kCells];
    __shared__ float red[6][(T / 64)];
    __shared__ uint32_t wsum[(T / 64)];
    // per-step merge: every wave submits its argmax as one 64-bit key to an LDS atomic max
    // (triple-buffered so a slot is cleared two barriers after its last read) and its
    // coordinates to a per-wave slot (double-buffered); one barrier per step
    __shared__ unsigned long long mkey[3];
    __shared__ __attribute__((aligned(16))) float mcrd[2][(T / 64)][4];

    fps_prologue<T>(p, n, W, hist, red, wsum);
    const int nb = (n + 63) / 64;
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
            const int pos = bucket * 64 + lane;
            float v[3] = {INFINITY, INFINITY, INFINITY}, u[3] = {-INFINITY, -INFINITY, -INFINITY};
            if (pos < n) {
                const float4 P = W.p[pos];
                v[0] = u[0] = P.x;
                v[1] = u[1] = P.y;
                v[2] = u[2] = P.z;
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
                if (cnt >= 4)
                    update_batch<4, T / 64>(mask, W, wave, q, lane, qx, qy, qz, bd[q], bi[q], bx[q], bp[q], target,
                                             wave_dirty);
                else if (cnt == 3)  // one round trip instead of 2 + 1
                    update_batch<3, T / 64>(mask, W, wave, q, lane, qx, qy, qz, bd[q], bi[q], bx[q], bp[q], target,
                                             wave_dirty);
                else if (cnt >= 2)
                    update_batch<2, T / 64>(mask, W, wave, q, lane, qx, qy, qz, bd[q], bi[q], bx[q], bp[q], target,
                                             wave_dirty);
                else
                    update_batch<1, T / 64>(mask, W, wave, q, lane, qx, qy, qz, bd[q], bi[q], bx[q], bp[q], target,
                                             wave_dirty);
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
        // key: dist bits (d >= 0 orders as unsigned) | (2^18 - idx) << 4 | wave; a larger key
        // is a larger distance, then a smaller index (n <= 2^18); empty slots carry field 0
        const int slot = cur3, cslot = it & 1;
        if (lane == 0) {
            const uint32_t fld = w_i < (1u << 18) ? (1u << 18) - w_i : 0u;
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
            const uint32_t gidx = (1u << 18) - (((uint32_t)key) >> 4);
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

// ----------------------------------------------------------------- one-wave FPS (round 3)
// The kernel above spends 8-16 waves per frame on ~20 active buckets per step, and those waves'
// registers cost the MFMA levels that share the CUs a wave slot per SIMD.  Here a
// frame is ONE wavefront: no barriers, one wave of CU footprint per frame in flight, and under
// 11 KiB of LDS for a 65 536-point frame (measured: a 64-thread workgroup with ~116 VGPRs and
// 11 KiB of LDS per frame costs the MFMA levels nothing measurable; 22 KiB costs them a workgroup
// slot per CU, tools/micro/contend.py).
//
// Buckets are 128 consecutive Morton-sorted points (two per lane), grouped into slots of 64
// buckets (8 192 points: 1/8 of a 65 536-point frame's Morton curve).  Bucket b = 64 q + lane.
//   registers: lane l holds the boxes of buckets (q, l) for every slot q, quantised to 8 bits per
//              bound relative to slot q's box (2 VGPRs per bucket); lane q < S holds slot q's box,
//              its quantisation step, and the slot's key (max dist, lowest index, coordinates, and
//              which bucket holds it);
//   LDS:       every bucket's key: kd = max-dist bits, kc = (x, y, z, index | argmax member << 24).
// A step tests the S slot boxes (one instruction), then the buckets of the active slots, appends
// the active buckets to an LDS list, streams them in batches (all loads of a batch in flight
// together, the reductions of a batch interleaved), re-keys the slots whose argmax bucket changed
// and takes the frame argmax over the slot keys — all inside one wave.
// Exactness: a quantised box CONTAINS the bucket's fp32 box (each bound is rounded outward and
// checked in the same fp32 fma the test uses), so its bound lb is still <= every member's d
// (the argument in the header); frames with a non-finite coordinate test nothing (lb = 0).
constexpr int kWaveMaxSlots = 16;  // 16 x 64 buckets x 128 points = 131 072 points per frame
constexpr int kWB = 128;           // points per bucket

struct WaveLayout {  // the one-wave FPS's per-frame workspace, offsets in floats
    int npad, nbs, S;
    int64_t p, d, qbox, init, slot, total;
};
__host__ __device__ inline WaveLayout wave_layout(int n)
{
    WaveLayout L;
    const int nb = (n + kWB - 1) / kWB;
    L.npad = nb * kWB;
    int S = 1;
    while (S * 64 < nb) S *= 2;
    L.S = S;
    L.nbs = S * 64;
    L.p = 0;                        // (npad + kWB) float4 (x, y, z, index): points, sentinels, a dummy bucket
    L.d = 4 * (int64_t)(L.npad + kWB);
    L.qbox = L.d + L.npad + kWB;    // 2 u32 per bucket record
    L.init = L.qbox + 2 * L.nbs;    // float4 per bucket: its key at dist +inf (lowest index member)
    L.slot = L.init + 4 * L.nbs;    // 16 floats per slot: lo[3], hi[3], step[3], no-filter flag
    L.total = L.slot + 16 * kWaveMaxSlots;
    return L;
}

__device__ __forceinline__ float wave_min_dpp(float v)
{
    v = fminf(v, __int_as_float(lidar::dpp_i<0xB1>(__float_as_int(v))));
    v = fminf(v, __int_as_float(lidar::dpp_i<0x4E>(__float_as_int(v))));
    v = fminf(v, __int_as_float(lidar::dpp_i<0x141>(__float_as_int(v))));
    v = fminf(v, __int_as_float(lidar::dpp_i<0x140>(__float_as_int(v))));
    const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return fminf(fminf(a, b), fminf(c, d));
}

// max over the wave in EVERY lane, in VALU only (4 DPP row steps, then the xor-32 / xor-16
// partners by v_permlane32_swap / v_permlane16_swap): independent reductions interleave freely
__device__ __forceinline__ int wave_max_all(int v)
{
    v = max(v, lidar::dpp_i<0xB1>(v));
    v = max(v, lidar::dpp_i<0x4E>(v));
    v = max(v, lidar::dpp_i<0x141>(v));
    v = max(v, lidar::dpp_i<0x140>(v));
    const auto a = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
    v = max(v, max((int)a[0], (int)a[1]));
    const auto c = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
    return max(v, max((int)c[0], (int)c[1]));
}
__device__ __forceinline__ uint32_t wave_min_all_u32(uint32_t v)
{
    v = min(v, (uint32_t)lidar::dpp_i<0xB1>((int)v));
    v = min(v, (uint32_t)lidar::dpp_i<0x4E>((int)v));
    v = min(v, (uint32_t)lidar::dpp_i<0x141>((int)v));
    v = min(v, (uint32_t)lidar::dpp_i<0x140>((int)v));
    const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = min(v, min((uint32_t)a[0], (uint32_t)a[1]));
    const auto c = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return min(v, min((uint32_t)c[0], (uint32_t)c[1]));
}

__device__ __forceinline__ float rdl(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }

// lower bound of d(., q) over a box, with the rounded operations of lidar::dist2f
__device__ __forceinline__ float box_lb(float qx, float qy, float qz, float lx, float ly, float lz, float hx, float hy,
                                        float hz)
{
    const float gx = gap(qx, lx, hx), gy = gap(qy, ly, hy), gz = gap(qz, lz, hz);
    return __fadd_rn(__fadd_rn(__fmul_rn(gx, gx), __fmul_rn(gy, gy)), __fmul_rn(gz, gz));
}

// Prologue of the one-wave FPS, one 1 024-thread workgroup per frame: the Morton counting sort
// (fps_prologue), padding to whole 128-point buckets plus the dummy bucket, every bucket's box and
// key at dist +inf, every slot's box and step, and the quantised bucket boxes.
__global__ __launch_bounds__(1024) void fps_wave_prep_kernel(const float *__restrict__ xyz, int n, int npoint,
                                                             const int32_t *__restrict__ prefix_ok,
                                                             float *__restrict__ ws, int64_t ws_stride)
{
    constexpr int T = 1024;
    const int b = blockIdx.x;
    if (prefix_ok != nullptr && prefix_ok[b] >= npoint) return;  // the step kernel copies the prefix
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float *p = xyz + (int64_t)b * n * 3;
    const WaveLayout L = wave_layout(n);
    float *wsb = ws + (int64_t)b * ws_stride;
    const FrameWs W{reinterpret_cast<float4 *>(wsb + L.p), wsb + L.d};
    __shared__ uint32_t hist[kCells];
    __shared__ float red[6][T / 64];
    __shared__ uint32_t wsum[T / 64];
    __shared__ float box[kWaveMaxSlots * 64][6];
    __shared__ int nonfinite;
    if (tid == 0) nonfinite = 0;  // fps_prologue's barriers order this before every use
    fps_prologue<T>(p, n, W, hist, red, wsum);
    const int nb = L.npad / kWB, S = L.S;
    // fps_prologue pads to whole 64-point groups; the rest of the last bucket and the dummy bucket
    // that pads a step's last batch (never closer, never reduced): dist -1 sentinels
    for (int i = (n + 63) / 64 * 64 + tid; i < L.npad + kWB; i += T) {
        W.p[i] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(0xffffffffu));
        W.d[i] = -1.0f;
    }
    float4 *init = reinterpret_cast<float4 *>(wsb + L.init);
    uint32_t *qbox = reinterpret_cast<uint32_t *>(wsb + L.qbox);
    float *slotp = wsb + L.slot;
    for (int bucket = wave; bucket < L.nbs; bucket += T / 64) {
        const int pos = bucket * kWB + lane;
        const bool r0 = pos < n, r1 = pos + 64 < n;
        const float4 P0 = r0 ? W.p[pos] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const float4 P1 = r1 ? W.p[pos + 64] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const bool bad = (r0 && !(isfinite(P0.x) && isfinite(P0.y) && isfinite(P0.z))) ||
                         (r1 && !(isfinite(P1.x) && isfinite(P1.y) && isfinite(P1.z)));
        const float lx = wave_min_dpp(fminf(r0 ? P0.x : INFINITY, r1 ? P1.x : INFINITY));
        const float ly = wave_min_dpp(fminf(r0 ? P0.y : INFINITY, r1 ? P1.y : INFINITY));
        const float lz = wave_min_dpp(fminf(r0 ? P0.z : INFINITY, r1 ? P1.z : INFINITY));
        const float hx = lidar::wave_max_dpp(fmaxf(r0 ? P0.x : -INFINITY, r1 ? P1.x : -INFINITY));
        const float hy = lidar::wave_max_dpp(fmaxf(r0 ? P0.y : -INFINITY, r1 ? P1.y : -INFINITY));
        const float hz = lidar::wave_max_dpp(fmaxf(r0 ? P0.z : -INFINITY, r1 ? P1.z : -INFINITY));
        const uint32_t i0 = r0 ? __float_as_uint(P0.w) : 0xffffffffu, i1 = r1 ? __float_as_uint(P1.w) : 0xffffffffu;
        const uint32_t mi = lidar::wave_min_u32_dpp(min(i0, i1));
        const uint64_t c0 = __ballot(i0 == mi);
        const int sub = c0 ? 0 : 1;  // index 0xffffffff (no member) only in buckets past nb
        const int wl = __ffsll((unsigned long long)(c0 ? c0 : __ballot(i1 == mi))) - 1;
        const float wx = rdl(sub ? P1.x : P0.x, wl), wy = rdl(sub ? P1.y : P0.y, wl), wz = rdl(sub ? P1.z : P0.z, wl);
        const bool any_bad = __ballot(bad) != 0;
        if (lane == 0) {
            box[bucket][0] = lx;
            box[bucket][1] = ly;
            box[bucket][2] = lz;
            box[bucket][3] = hx;
            box[bucket][4] = hy;
            box[bucket][5] = hz;
            // key at dist +inf: the lowest-index member (the argmax member); empty records carry
            // index 2^24 - 1 and member 0 (never changes: the padding dist is -1)
            init[bucket] = bucket < nb ? make_float4(wx, wy, wz, __uint_as_float(mi | ((uint32_t)(wl + 64 * sub) << 24)))
                                       : make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(0xffffffu));
            if (any_bad) nonfinite = 1;
        }
    }
    __syncthreads();
    if (wave < S) {  // slot `wave`: lane = bucket within the slot
        const int bucket = wave * 64 + lane;
        const bool real = bucket < nb;
        float lo[3], hi[3], slo[3], shi[3], st[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = real ? box[bucket][a] : INFINITY;
            hi[a] = real ? box[bucket][3 + a] : -INFINITY;
            slo[a] = wave_min_dpp(lo[a]);
            shi[a] = lidar::wave_max_dpp(hi[a]);
        }
        bool nof = nonfinite != 0;  // wave-uniform throughout
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float s = __fdiv_rn(__fsub_rn(shi[a], slo[a]), 255.0f);
            if (!(isfinite(slo[a]) && isfinite(shi[a]) && isfinite(s))) {
                nof = true;
                s = 0.0f;
            }
            // the top code must reach the slot's upper bound in the step kernel's own fma
            for (int k = 0; k < 8 && !nof && __fmaf_rn(255.0f, s, slo[a]) < shi[a]; ++k) s = nextafterf(s, INFINITY);
            if (!nof && !(__fmaf_rn(255.0f, s, slo[a]) >= shi[a])) nof = true;
            st[a] = s;
        }
        uint32_t ql[3] = {0, 0, 0}, qh[3] = {0, 0, 0};
        if (!nof && real) {
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                if (st[a] > 0.0f) {
                    int v = (int)fminf(fmaxf(floorf(__fdiv_rn(__fsub_rn(lo[a], slo[a]), st[a])), 0.0f), 255.0f);
                    while (v > 0 && __fmaf_rn((float)v, st[a], slo[a]) > lo[a]) --v;  // outward: <= lo
                    int w = (int)fminf(fmaxf(ceilf(__fdiv_rn(__fsub_rn(hi[a], slo[a]), st[a])), 0.0f), 255.0f);
                    while (w < 255 && __fmaf_rn((float)w, st[a], slo[a]) < hi[a]) ++w;  // outward: >= hi
                    ql[a] = (uint32_t)v;
                    qh[a] = (uint32_t)w;
                }  // step 0: the slot is one point on this axis, code 0 decodes to it exactly
            }
        }
        qbox[2 * bucket] = ql[0] | (ql[1] << 8) | (ql[2] << 16) | (qh[0] << 24);
        qbox[2 * bucket + 1] = qh[1] | (qh[2] << 8);
        if (lane < 10) {
            const float v = lane < 3 ? slo[lane % 3] : lane < 6 ? shi[lane % 3] : lane < 9 ? st[lane % 3] : (nof ? 1.0f : 0.0f);
            slotp[wave * 16 + lane] = v;
        }
    }
}

// One round of up to 8 active buckets: lane group g = lane / 8 takes the list entry k + g (the
// dummy bucket past the list's end), lane j = lane % 8 of it the bucket's points 8 i + j, i < 16
// (each load instruction reads one 128-B line per group).  All 32 loads of a lane are in flight
// together; per point the new distance, per lane the max and its lowest index, then a 3-step DPP
// reduction inside the group gives the bucket's key (max dist bits, lowest index, position).  A
// bucket whose key changed and is its slot's argmax bucket marks the slot for a re-key.
__device__ __forceinline__ void group_round(int e, const float4 *__restrict__ P4, float *__restrict__ Dd, int *kd,
                                            uint32_t *kc, const uint8_t *sbbl, int lane, float qx, float qy, float qz,
                                            uint32_t &touched)
{
    const int j = lane & 7;
    const int bb = __builtin_amdgcn_ds_bpermute((lane >> 3) << 2, e);  // entry g of the round
    const uint32_t base = (uint32_t)(bb * kWB + j);
    float4 P[16];
    float D[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        P[i] = P4[base + 8 * i];
        D[i] = Dd[base + 8 * i];
    }
    const int old_d = kd[bb];
    const uint32_t old_c = kc[bb];
    const int slot_arg = sbbl[bb >> 6];
    int o[16], best = INT_MIN;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const float d = lidar::dist2f(P[i].x, P[i].y, P[i].z, qx, qy, qz);
        // float order: a NaN d (inf - inf) never replaces a dist, as in the oracle
        const bool lower = d < D[i];
        o[i] = lower ? __float_as_int(d) : __float_as_int(D[i]);
        Dd[base + 8 * i] = __int_as_float(o[i]);  // unchanged members rewrite their own dist
        best = max(best, o[i]);
    }
    // the group's max, then the lowest index holding it
    best = max(best, lidar::dpp_i<0xB1>(best));
    best = max(best, lidar::dpp_i<0x4E>(best));
    best = max(best, lidar::dpp_i<0x141>(best));
    uint32_t mi = 0xffffffffu;
    int mpos = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t I = __float_as_uint(P[i].w);
        const bool c = o[i] == best && I < mi;
        mi = c ? I : mi;
        mpos = c ? 8 * i + j : mpos;
    }
    uint32_t gmi = min(mi, (uint32_t)lidar::dpp_i<0xB1>((int)mi));
    gmi = min(gmi, (uint32_t)lidar::dpp_i<0x4E>((int)gmi));
    gmi = min(gmi, (uint32_t)lidar::dpp_i<0x141>((int)gmi));
    // the holder's position: lanes with mi == gmi hold it (one lane: indices are distinct)
    int gpos = mi == gmi ? mpos : 0;
    gpos = max(gpos, lidar::dpp_i<0xB1>(gpos));
    gpos = max(gpos, lidar::dpp_i<0x4E>(gpos));
    gpos = max(gpos, lidar::dpp_i<0x141>(gpos));
    const uint32_t rec = (gmi & 0xffffffu) | ((uint32_t)gpos << 24);
    if (j == 0) {
        kd[bb] = best;
        kc[bb] = rec;
    }
    // keys only decrease: a slot's key can change only when its argmax bucket's key did
    const bool mark = j == 0 && (best != old_d || rec != old_c) && (bb & 63) == slot_arg;
    uint32_t m = mark ? 1u << (bb >> 6) : 0u;
    m |= (uint32_t)lidar::dpp_i<0xB1>((int)m);
    m |= (uint32_t)lidar::dpp_i<0x4E>((int)m);
    m |= (uint32_t)lidar::dpp_i<0x141>((int)m);
    m |= (uint32_t)lidar::dpp_i<0x140>((int)m);
    const auto a = __builtin_amdgcn_permlane32_swap(m, m, false, false);
    m |= a[0] | a[1];
    const auto c = __builtin_amdgcn_permlane16_swap(m, m, false, false);
    m |= c[0] | c[1];
    touched |= (uint32_t)__builtin_amdgcn_readfirstlane((int)m);
}

// DIAG builds (lidar_diag_fps_wave only) accumulate, per frame: shader cycles of [0] slot tests and
// the list, [1] batches, [2] slot re-keys, [3] frame argmax; counts of [4] active slots, [5] active
// buckets, [6] batches, [7] re-keyed slots, [8] steps
template <int S, bool DIAG = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_vgpr(128))) void fps_wave_kernel(
    const float *__restrict__ xyz, int n, int npoint, int32_t *__restrict__ out_idx, float *__restrict__ out_xyz,
    int32_t *__restrict__ first_zero, const int32_t *__restrict__ prefix_ok, float *__restrict__ ws, int64_t ws_stride,
    uint64_t *__restrict__ diag)
{
    uint64_t dacc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t t0 = 0, t1 = 0;
    auto tick = [&](int k) {
        if constexpr (DIAG) {
            __builtin_amdgcn_sched_barrier(0);
            t1 = stamp();
            dacc[k] += t1 - t0;
            t0 = t1;
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    constexpr int NBS = S * 64;
    const int b = blockIdx.x, lane = threadIdx.x;
    const float *p = xyz + (int64_t)b * n * 3;
    if (prefix_ok != nullptr && prefix_ok[b] >= npoint) {  // nested FPS shortcut (see the header)
        for (int i = lane; i < npoint; i += 64) {
            out_idx[(int64_t)b * npoint + i] = i;
            if (out_xyz) {
                float *o = out_xyz + ((int64_t)b * npoint + i) * 3;
                o[0] = p[3 * i];
                o[1] = p[3 * i + 1];
                o[2] = p[3 * i + 2];
            }
        }
        if (first_zero && lane == 0) first_zero[b] = prefix_ok[b];
        return;
    }
    const WaveLayout L = wave_layout(n);
    float *wsb = ws + (int64_t)b * ws_stride;
    const float4 *P4 = reinterpret_cast<const float4 *>(wsb + L.p);
    float *Dd = wsb + L.d;
    const int nb = L.npad / kWB;  // also the dummy bucket's number
    __shared__ int kd[NBS + 1];
    __shared__ uint32_t kc[NBS + 1];  // index | position of the argmax member in the bucket << 24
    __shared__ uint16_t list[NBS];
    __shared__ uint8_t sbbl[S];       // each slot's argmax bucket (lane), as sbb below
    constexpr int kInf = 0x7f800000, kNeg1 = (int)0xbf800000u;

    uint32_t qb0[S], qb1[S];
    {
        const uint32_t *qbox = reinterpret_cast<const uint32_t *>(wsb + L.qbox);
        const float4 *init = reinterpret_cast<const float4 *>(wsb + L.init);
#pragma unroll
        for (int q = 0; q < S; ++q) {
            const int bucket = q * 64 + lane;
            qb0[q] = qbox[2 * bucket];
            qb1[q] = qbox[2 * bucket + 1];
            kd[bucket] = bucket < nb ? kInf : kNeg1;
            kc[bucket] = __float_as_uint(init[bucket].w);
        }
        if (lane == 0) {  // the dummy's record when every bucket of the last slot is real
            kd[NBS] = kNeg1;
            kc[NBS] = 0xffffffu;
        }
    }
    // slot q's box lo[3], hi[3], step[3], no-filter flag (LDS: read per step, not held in VGPRs)
    __shared__ __attribute__((aligned(16))) float slp[S][12];
    for (int i = lane; i < 10 * S; i += 64) slp[i / 10][i % 10] = wsb[L.slot + (i / 10) * 16 + i % 10];
    // lane q < S: slot q's key (max dist bits, lowest index), the lane (bucket within the slot) that
    // holds it and the member's position in that bucket; INT_MIN elsewhere
    int sbd = INT_MIN, sbb = 0, sbp = 0;
    uint32_t sbi = 0xffffffffu;
    auto slot_key = [&](int q) {
        const int v = kd[q * 64 + lane];
        const uint32_t r = kc[q * 64 + lane];
        const uint32_t id = r & 0xffffffu;
        const int m = wave_max_all(v);
        const uint64_t c = __ballot(v == m);
        int wl;
        if (__popcll(c) == 1) {
            wl = __ffsll((unsigned long long)c) - 1;
        } else {
            const uint32_t mi = wave_min_all_u32(v == m ? id : 0xffffffffu);
            wl = __ffsll((unsigned long long)__ballot(v == m && id == mi)) - 1;
        }
        const uint32_t wr = (uint32_t)__builtin_amdgcn_readlane((int)r, wl);
        const bool me = lane == q;
        sbd = me ? m : sbd;
        sbb = me ? wl : sbb;
        sbi = me ? (wr & 0xffffffu) : sbi;
        sbp = me ? (int)(wr >> 24) : sbp;
        if (lane == 0) sbbl[q] = (uint8_t)wl;
    };
#pragma unroll
    for (int q = 0; q < S; ++q) slot_key(q);

    float qx = p[0], qy = p[1], qz = p[2];
    if (lane == 0) {
        out_idx[(int64_t)b * npoint] = 0;
        if (out_xyz) {
            float *o = out_xyz + (int64_t)b * npoint * 3;
            o[0] = qx;
            o[1] = qy;
            o[2] = qz;
        }
    }
    int zero_at = npoint;
    for (int it = 1; it < npoint; ++it) {
        int lane = threadIdx.x;  // opaque per step: keeps per-slot lane offsets from being hoisted
        asm volatile("" : "+v"(lane));
        if constexpr (DIAG) {
            __builtin_amdgcn_sched_barrier(0);
            t0 = stamp();
            __builtin_amdgcn_sched_barrier(0);
        }
        // slots whose box may hold a point closer to q than the slot's max
        const int ls = lane < S ? lane : 0;
        const float lbs = slp[ls][9] != 0.0f ? 0.0f
                                             : box_lb(qx, qy, qz, slp[ls][0], slp[ls][1], slp[ls][2], slp[ls][3],
                                                      slp[ls][4], slp[ls][5]);
        const uint32_t act = (uint32_t)__ballot(lane < S && __float_as_int(lbs) < sbd);
        // their buckets' keys (all reads in flight together), then the bucket tests; the active
        // buckets are appended to the list
        int kdv[S];
#pragma unroll
        for (int q = 0; q < S; ++q)
            if ((act >> q) & 1u) kdv[q] = kd[q * 64 + lane];
        int cnt = 0;
#pragma unroll
        for (int q = 0; q < S; ++q) {
            if (!((act >> q) & 1u)) continue;  // wave-uniform
            const float b0 = slp[q][0], b1 = slp[q][1], b2 = slp[q][2];
            const float s0 = slp[q][6], s1 = slp[q][7], s2 = slp[q][8];
            uint32_t w0 = qb0[q], w1 = qb1[q];
            // opaque per step: otherwise the decoded boxes (6 VGPRs per slot) are hoisted out of
            // the step loop and the kernel needs ~3x the registers
            asm volatile("" : "+v"(w0), "+v"(w1));
            const float lx = __fmaf_rn((float)(w0 & 0xff), s0, b0);
            const float ly = __fmaf_rn((float)((w0 >> 8) & 0xff), s1, b1);
            const float lz = __fmaf_rn((float)((w0 >> 16) & 0xff), s2, b2);
            const float hx = __fmaf_rn((float)(w0 >> 24), s0, b0);
            const float hy = __fmaf_rn((float)(w1 & 0xff), s1, b1);
            const float hz = __fmaf_rn((float)((w1 >> 8) & 0xff), s2, b2);
            float lb = box_lb(qx, qy, qz, lx, ly, lz, hx, hy, hz);
            if (slp[q][9] != 0.0f) lb = 0.0f;  // no-filter slot: every bucket is tested
            const uint64_t mk = __ballot(__float_as_int(lb) < kdv[q]);
            if ((mk >> lane) & 1ull) {
                const int at = cnt + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
                list[at] = (uint16_t)(q * 64 + lane);
            }
            cnt += __popcll(mk);
        }
        if constexpr (DIAG) {
            dacc[4] += __popc(act);
            dacc[5] += cnt;
            dacc[6] += (cnt + 7) / 8;
        }
        tick(0);
        uint32_t touched = 0;
        for (int k = 0; k < cnt; k += 8) {  // wave-uniform
            const int e = lane < 8 && k + lane < cnt ? (int)list[k + lane] : nb;
            group_round(e, P4, Dd, kd, kc, sbbl, lane, qx, qy, qz, touched);
        }
        tick(1);
        if constexpr (DIAG) dacc[7] += __popc(touched);
#pragma unroll
        for (int q = 0; q < S; ++q)
            if ((touched >> q) & 1u) slot_key(q);
        tick(2);
        // the frame argmax over the slot keys (lanes < S; the rest hold INT_MIN)
        const int gm = wave_max_all(sbd);
        const uint64_t gc = __ballot(sbd == gm);
        int g;
        if (__popcll(gc) == 1) {
            g = __ffsll((unsigned long long)gc) - 1;
        } else {
            const uint32_t mi = wave_min_all_u32(sbd == gm ? sbi : 0xffffffffu);
            g = __ffsll((unsigned long long)__ballot(sbd == gm && sbi == mi)) - 1;
        }
        {  // the winner's coordinates (one uniform load: the sorted copy is read-only here)
            const int wb = g * 64 + __builtin_amdgcn_readlane(sbb, g);
            const float4 W = P4[wb * kWB + __builtin_amdgcn_readlane(sbp, g)];
            qx = W.x;
            qy = W.y;
            qz = W.z;
        }
        if (lane == 0) {
            out_idx[(int64_t)b * npoint + it] = __builtin_amdgcn_readlane((int)sbi, g);
            if (out_xyz) {
                float *o = out_xyz + ((int64_t)b * npoint + it) * 3;
                o[0] = qx;
                o[1] = qy;
                o[2] = qz;
            }
        }
        if (zero_at == npoint && gm == 0) zero_at = it;
        tick(3);
        if constexpr (DIAG) dacc[8]++;
    }
    if (first_zero && lane == 0) first_zero[b] = zero_at;
    if constexpr (DIAG) {
        if (lane == 0)
            for (int k = 0; k < 9; ++k) diag[(int64_t)b * 9 + k] = dacc[k];
    }
}

}  // namespace

static int launch_fps_wave(const float *xyz, int64_t batch, int64_t n, int64_t npoint, int32_t *idx, float *new_xyz,
                           int32_t *first_zero, const int32_t *prefix_ok, float *ws, int64_t stride, hipStream_t s)
{
    const WaveLayout L = wave_layout((int)n);
    hipLaunchKernelGGL(fps_wave_prep_kernel, dim3((unsigned)batch), dim3(1024), 0, s, xyz, (int)n, (int)npoint,
                       prefix_ok, ws, stride);
    LAUNCH_CHECK();
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3((unsigned)batch), dim3(64), 0, s, xyz, (int)n, (int)npoint, idx, new_xyz,
                           first_zero, prefix_ok, ws, stride, nullptr);
    };
    // batches of 8 buckets (80 VGPRs of loads in flight) up to 8 slots; 4 beside 16 slots' boxes
    switch (L.S) {
        case 1: go(fps_wave_kernel<1>); break;
        case 2: go(fps_wave_kernel<2>); break;
        case 4: go(fps_wave_kernel<4>); break;
        case 8: go(fps_wave_kernel<8>); break;
        default: go(fps_wave_kernel<16>); break;
    }
    LAUNCH_CHECK();
    return LIDAR_OK;
}

static int64_t fps_stride(int64_t n)
{
    const int64_t old = 5 * (int64_t)lidar::align_up(n, 64);
    const int64_t wave = (n + kWB - 1) / kWB <= kWaveMaxSlots * 64 ? wave_layout((int)n).total : 0;
    return (int64_t)lidar::align_up((uint64_t)std::max(old, wave), 64);
}

template <int T>
static int launch_fps(const float *xyz, int64_t batch, int64_t n, int64_t npoint, int32_t *idx, float *new_xyz,
                      int32_t *first_zero, const int32_t *prefix_ok, float *ws, int64_t stride, hipStream_t s)
{
    dim3 grid((unsigned)batch), block(T);
    const int nb = (int)((n + 63) / 64);
    const int lanes = T;  // one bucket per lane and slot
    auto go = [&](auto kern) -> int {
        hipLaunchKernelGGL(kern, grid, block, 0, s, xyz, (int)n, (int)npoint, idx, new_xyz, first_zero,
                           prefix_ok, ws, stride, nullptr);
        return LIDAR_OK;
    };
    int rc;
    if (nb <= lanes) rc = go(fps_bucket_kernel<T, 1>);
    else if (nb <= 2 * lanes) rc = go(fps_bucket_kernel<T, 2>);
    else if (nb <= 4 * lanes) rc = go(fps_bucket_kernel<T, 4>);
    else rc = go(fps_bucket_kernel<T, 8>);
    if (rc) return rc;
    LAUNCH_CHECK();
    return LIDAR_OK;
}

// workspace bytes lidar_fps_f32 / lidar_fps_ex_f32 take from the handle for (batch, n)
LIDAR_EXPORT uint64_t lidar_fps_workspace_bytes(int64_t batch, int64_t n)
{
    return (uint64_t)(batch * fps_stride(n)) * 4;
}

// threads: workgroup size per frame — 0 (auto: the one-wave kernel up to 65 536 points, 1024
// threads above), 64 (one wavefront per frame), 1024 or 512 — same results
LIDAR_EXPORT int lidar_fps_ex_f32(lidar_handle *h, const float *xyz, int64_t batch, int64_t n, int64_t npoint,
                                  int32_t *idx, float *new_xyz, int32_t *first_zero, const int32_t *prefix_ok,
                                  int32_t threads, void *stream)
{
    REQUIRE(h && xyz && idx, "lidar_fps_f32: null pointer");
    REQUIRE(batch >= 0 && n >= 1 && npoint >= 1, "lidar_fps_f32: need n >= 1 and npoint >= 1");
    REQUIRE(n <= 4 * 65536, "lidar_fps_f32: n > 262144 points per frame");
    const int64_t nb = (n + 63) / 64, nbw = (n + kWB - 1) / kWB;
    if (threads == 0) threads = nbw <= kWaveMaxSlots * 64 ? 64 : kThreads;
    REQUIRE(threads == 1024 || threads == 512 || threads == 64, "lidar_fps_ex_f32: threads must be 0, 64, 512 or 1024");
    REQUIRE(threads == 64 ? nbw <= kWaveMaxSlots * 64 : nb <= 8 * (int64_t)threads,
            "lidar_fps_f32: too many buckets for this workgroup size");
    REQUIRE(batch <= 0x7fffffff, "lidar_fps_f32: batch too large");
    if (batch == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    REQUIRE(prefix_ok == nullptr || npoint <= n, "lidar_fps_f32: prefix_ok needs npoint <= n");
    const int64_t stride = fps_stride(n);
    float *ws = static_cast<float *>(lidar::workspace(h, (uint64_t)(batch * stride) * 4));
    if (!ws) return LIDAR_ENOMEM;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (threads == 64)
        return launch_fps_wave(xyz, batch, n, npoint, idx, new_xyz, first_zero, prefix_ok, ws, stride, s);
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

// diagnostic build (not part of the product ABI): per-frame phase cycles and counts of the one-wave
// FPS (65 536-point frames: 8 slots), diag (batch, 9) u64
LIDAR_EXPORT int lidar_diag_fps_wave(lidar_handle *h, const float *xyz, int64_t batch, int64_t n, int64_t npoint,
                                     int32_t *idx, uint64_t *diag, void *stream)
{
    REQUIRE(h && xyz && idx && diag && n <= 65536 && n > 32768 && npoint >= 1, "lidar_diag_fps_wave: bad args");
    ON_DEVICE(h->device);
    const int64_t stride = fps_stride(n);
    float *ws = static_cast<float *>(lidar::workspace(h, (uint64_t)(batch * stride) * 4));
    if (!ws) return LIDAR_ENOMEM;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(fps_wave_prep_kernel, dim3((unsigned)batch), dim3(1024), 0, s, xyz, (int)n, (int)npoint,
                       nullptr, ws, stride);
    hipLaunchKernelGGL((fps_wave_kernel<8, true>), dim3((unsigned)batch), dim3(64), 0, s, xyz, (int)n, (int)npoint,
                       idx, nullptr, nullptr, nullptr, ws, stride, diag);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

// diagnostic build (not part of the product ABI): per-wave phase cycle totals of one FPS run
LIDAR_EXPORT int lidar_diag_fps_phases(lidar_handle *h, const float *xyz, int64_t batch, int64_t n,
                                       int64_t npoint, int32_t *idx, uint64_t *diag, void *stream)
{
    REQUIRE(h && xyz && idx && diag && n <= 65536 && n >= 1 && npoint >= 1, "lidar_diag_fps_phases: bad args");
    ON_DEVICE(h->device);
    const int64_t stride = fps_stride(n);
    float *ws = static_cast<float *>(lidar::workspace(h, (uint64_t)(batch * stride) * 4));
    if (!ws) return LIDAR_ENOMEM;
    REQUIRE((n + 63) / 64 <= kThreads, "lidar_diag_fps_phases: n too large for BPL=1");
    hipLaunchKernelGGL((fps_bucket_kernel<kThreads, 1, true>), dim3((unsigned)batch), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), xyz, (int)n, (int)npoint, idx, nullptr, nullptr,
                       nullptr, ws, stride, diag);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
