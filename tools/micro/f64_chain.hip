// Dependent fp64 add latency on gfx950: one wave runs a chain of N dependent adds (lanes 0..2
// active, as the preprocess chains), timed with s_memtime; variants: v_add_f64, v_fma_f64 with
// a multiplier of 1.0, and two interleaved chains.  usage: ./f64_chain
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 1 << 16;

template <int MODE>
__global__ void chain(const double *v, double *out, long long *cyc)
{
    const int lane = threadIdx.x;
    double a = 0.0, b = 0.0;
    long long t0 = clock64();
    if (lane < 3) {
#pragma unroll 16
        for (int i = 0; i < N; ++i) {
            const double x = MODE >= 3 ? v[i & 255] : v[0] + (double)(i & 1) * 1e-9;
            if (MODE == 0 || MODE == 3) a = __dadd_rn(a, x);
            else if (MODE == 1) a = __fma_rn(x, 1.0, a);
            else { a = __dadd_rn(a, x); b = __dadd_rn(b, x); }
        }
    }
    long long t1 = clock64();
    if (lane == 0) { out[0] = a + b; cyc[0] = t1 - t0; }
}

int main()
{
    double *v, *o; long long *c;
    hipMalloc(&v, 256 * 8); hipMalloc(&o, 8); hipMalloc(&c, 8);
    double h[256]; for (int i = 0; i < 256; ++i) h[i] = 1.0 + i * 1e-3;
    hipMemcpy(v, h, sizeof h, hipMemcpyHostToDevice);
    const char *names[4] = {"v_add_f64 (reg x)", "v_fma_f64 (reg x)", "2 interleaved (reg x)", "v_add_f64 (loaded x)"};
    for (int m = 0; m < 4; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            if (m == 0) chain<0><<<1, 64>>>(v, o, c);
            if (m == 1) chain<1><<<1, 64>>>(v, o, c);
            if (m == 2) chain<2><<<1, 64>>>(v, o, c);
            if (m == 3) chain<3><<<1, 64>>>(v, o, c);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            long long cy; hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
            if (rep) printf("%-22s %.2f ns/add  %.1f clock64 ticks/add  (kernel %.3f ms)\n", names[m], ms * 1e6 / N, (double)cy / N, ms);
        }
    }
    return 0;
}
