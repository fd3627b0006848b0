// diag.hip — diagnostic kernels for contention experiments (tools/contend.py); not part of
// the drop-in ABI (not declared in include/lidar_amd.h).
//
// lidar_diag_occupy: workgroups shaped like fps_bucket_kernel's (1024 threads, 56 VGPRs,
// ~42 KiB LDS) that only sleep, so a concurrent kernel's slowdown can be split into "the CU
// resources FPS holds" (this kernel reproduces it) and "what FPS does with them" (it does not).
#include "common.hpp"

namespace {

__global__ __launch_bounds__(1024) void occupy_kernel(int64_t iters, int *sink)
{
    __shared__ float pad[10752];  // 42 KiB
    // hold 56 VGPRs like the FPS kernel
    asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13",
                 "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27",
                 "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41",
                 "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55");
    for (int64_t i = 0; i < iters; ++i) __builtin_amdgcn_s_sleep(127);
    pad[threadIdx.x] = 0.0f;
    __syncthreads();
    if (threadIdx.x == 0 && pad[1] != 0.0f) *sink = 1;
}

}  // namespace

LIDAR_EXPORT int lidar_diag_occupy(lidar_handle *h, int64_t blocks, int64_t iters, int *sink, void *stream)
{
    REQUIRE(h && sink && blocks >= 1 && blocks <= 4096 && iters >= 0 && iters <= (1ll << 24),
            "lidar_diag_occupy: bad args");
    HIP_TRY(hipSetDevice(h->device));
    hipLaunchKernelGGL(occupy_kernel, dim3((unsigned)blocks), dim3(1024), 0, static_cast<hipStream_t>(stream), iters,
                       sink);
    LAUNCH_CHECK();
    return LIDAR_OK;
}
