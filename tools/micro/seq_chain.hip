// The preprocess kernel's sequential-chain structure in isolation (density.hip block_seq_chain):
// a 1024-thread workgroup, waves 1..15 stage 1024-row (n, 3) fp64 chunks into LDS (double
// buffered), lanes 0..2 of wave 0 run the dependent adds.  Variants of the consumer loop:
//   0: batches of 16 reads, then 16 dependent adds (the kernel's form)
//   1: software pipelined: the next batch's 16 reads issued before this batch's adds
//   2: reads of 8 rows ahead, one row at a time (rolling window)
// Times one frame of 65 536 rows per variant.  usage: ./seq_chain
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kT = 1024, kRows = 1024;

template <int MODE>
__global__ __launch_bounds__(kT) void chain(const double *x, int n, double *out)
{
    __shared__ double st[2][kRows * 3];
    const int tid = threadIdx.x;
    const int nch = (n + kRows - 1) / kRows;
    auto stage = [&](int k) {
        if (tid < 64 || k >= nch) return;
        const int cnt = (n - k * kRows < kRows ? n - k * kRows : kRows) * 3;
        for (int e = tid - 64; e < cnt; e += kT - 64) st[k & 1][e] = x[3 * k * kRows + e];
    };
    double a = 0.0;
    stage(0);
    __syncthreads();
    for (int k = 0; k < nch; ++k) {
        stage(k + 1);
        if (tid < 3) {
            const int rows = n - k * kRows < kRows ? n - k * kRows : kRows;
            const double *b = st[k & 1] + tid;
            int i = 0;
            if (MODE == 0) {
                for (; i + 16 <= rows; i += 16) {
                    double v[16];
#pragma unroll
                    for (int u = 0; u < 16; ++u) v[u] = b[3 * (i + u)];
#pragma unroll
                    for (int u = 0; u < 16; ++u) a = __dadd_rn(a, v[u]);
                }
            } else if (MODE == 1) {
                // two register batches in alternation: batch B's reads are in flight while batch A's
                // dependent adds run, and vice versa (8 ds_read2_b64 per batch: lgkmcnt(8) separates them)
                double v[16], w[16];
                if (rows >= 16) {
#pragma unroll
                    for (int u = 0; u < 16; ++u) v[u] = b[3 * u];
                }
                for (; i + 48 <= rows; i += 32) {
#pragma unroll
                    for (int u = 0; u < 16; ++u) w[u] = b[3 * (i + 16 + u)];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int u = 0; u < 16; ++u) a = __dadd_rn(a, v[u]);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int u = 0; u < 16; ++u) v[u] = b[3 * (i + 32 + u)];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int u = 0; u < 16; ++u) a = __dadd_rn(a, w[u]);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (i + 16 <= rows) {
#pragma unroll
                    for (int u = 0; u < 16; ++u) a = __dadd_rn(a, v[u]);
                    i += 16;
                }
            } else if (MODE == 3) {
                // the dependent adds alone: 16 register operands loaded once per chunk, re-added
                // for every 16 rows (same add count, no LDS reads on the path)
                double v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) v[u] = b[3 * u];
                for (; i + 16 <= rows; i += 16) {
#pragma unroll
                    for (int u = 0; u < 16; ++u) a = __dadd_rn(a, v[u]);
                    asm volatile("" : "+v"(a));
                }
            } else if (MODE == 5) {
                // the next batch's reads interleaved one per dependent add (each read issues in the
                // shadow of the previous add), two register batches in alternation
                double v[16], w[16];
                if (rows >= 16) {
#pragma unroll
                    for (int u = 0; u < 16; ++u) v[u] = b[3 * u];
                }
                for (; i + 48 <= rows; i += 32) {
#pragma unroll
                    for (int u = 0; u < 16; ++u) {
                        w[u] = b[3 * (i + 16 + u)];
                        a = __dadd_rn(a, v[u]);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one DS read
                        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);  // then one VALU
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int u = 0; u < 16; ++u) {
                        v[u] = b[3 * (i + 32 + u)];
                        a = __dadd_rn(a, w[u]);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
                        __builtin_amdgcn_sched_group_barrier(0x002, 1, 1);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (i + 16 <= rows) {
#pragma unroll
                    for (int u = 0; u < 16; ++u) a = __dadd_rn(a, v[u]);
                    i += 16;
                }
            } else if (MODE == 4) {
                // batches of 8 reads, then 8 dependent adds
                for (; i + 8 <= rows; i += 8) {
                    double v[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) v[u] = b[3 * (i + u)];
#pragma unroll
                    for (int u = 0; u < 8; ++u) a = __dadd_rn(a, v[u]);
                }
            } else {
                double win[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) win[u] = u < rows ? b[3 * u] : 0.0;
                for (; i + 8 <= rows; i += 8) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const double cur = win[u];
                        win[u] = i + 8 + u < rows ? b[3 * (i + 8 + u)] : 0.0;
                        a = __dadd_rn(a, cur);
                    }
                }
            }
            for (; i < rows; ++i) a = __dadd_rn(a, b[3 * i]);
        }
        __syncthreads();
    }
    if (tid < 3) out[tid] = a;
}

int main()
{
    const int n = 65536;
    double *x, *o;
    hipMalloc(&x, (size_t)n * 3 * 8);
    hipMalloc(&o, 3 * 8);
    double *h = new double[(size_t)n * 3];
    for (int i = 0; i < 3 * n; ++i) h[i] = ((i * 2654435761u) % 1000003) * 1e-5 - 5.0;
    hipMemcpy(x, h, (size_t)n * 3 * 8, hipMemcpyHostToDevice);
    double ref[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i)
        for (int c = 0; c < 3; ++c) ref[c] += h[3 * i + c];
    const char *names[6] = {"batch16 (kernel form)", "alternating 16 / 16", "rolling window 8",
                            "adds only (no LDS)", "batch8", "interleaved read/add"};
    for (int m = 0; m < 6; ++m) {
        float best = 1e9;
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            if (m == 0) chain<0><<<1, kT>>>(x, n, o);
            if (m == 1) chain<1><<<1, kT>>>(x, n, o);
            if (m == 2) chain<2><<<1, kT>>>(x, n, o);
            if (m == 3) chain<3><<<1, kT>>>(x, n, o);
            if (m == 4) chain<4><<<1, kT>>>(x, n, o);
            if (m == 5) chain<5><<<1, kT>>>(x, n, o);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        double got[3];
        hipMemcpy(got, o, 24, hipMemcpyDeviceToHost);
        const bool ok = got[0] == ref[0] && got[1] == ref[1] && got[2] == ref[2];
        printf("%-24s %.3f ms  %.2f ns/row  %s\n", names[m], best, best * 1e6 / n,
               m == 3 ? "(sum not the reference's)" : ok ? "exact" : "MISMATCH");
    }
    return 0;
}
