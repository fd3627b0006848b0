// voxel.hip — single-frame voxel downsampling: the batched path of voxel_batch.hip
// with one frame, its voxel count copied back to the host (one stream synchronisation).
#include "common.hpp"

extern "C" uint64_t lidar_voxel_batch_workspace_bytes(int64_t batch, int64_t n);
extern "C" int lidar_voxel_downsample_batch_f32(lidar_handle *h, const float *xyz, int64_t batch, int64_t n,
                                                double voxel, int32_t *voxel_id, float *centroids, int32_t *counts,
                                                int32_t *nvox, void *stream);

LIDAR_EXPORT int lidar_voxel_downsample_f32(lidar_handle *h, const float *xyz, int64_t n, double voxel,
                                            int32_t *voxel_id, float *centroids, int32_t *counts,
                                            int64_t *nvox_host, void *stream)
{
    REQUIRE(h && xyz && voxel_id && centroids && counts && nvox_host, "lidar_voxel_downsample_f32: null pointer");
    REQUIRE(n >= 0 && n < 0x7fffffff, "lidar_voxel_downsample_f32: n out of range");
    REQUIRE(voxel > 0.0 && voxel < INFINITY, "lidar_voxel_downsample_f32: voxel size must be finite and > 0");
    *nvox_host = 0;
    if (n == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    // the voxel count lands in a word past the batched path's workspace (same block: workspace() only
    // grows), then in the handle's pinned host word
    const uint64_t need = lidar_voxel_batch_workspace_bytes(1, n) + 256;
    char *ws = static_cast<char *>(lidar::workspace(h, need));
    if (!ws) return LIDAR_ENOMEM;
    int32_t *dn = reinterpret_cast<int32_t *>(ws + need - 256);
    int rc = lidar_voxel_downsample_batch_f32(h, xyz, 1, n, voxel, voxel_id, centroids, counts, dn, stream);
    int32_t *hm = static_cast<int32_t *>(h->host_pinned);
    if (rc == LIDAR_OK) {
        const hipError_t e = hipMemcpyAsync(hm, dn, sizeof(int32_t), hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) rc = lidar::fail(LIDAR_EHIP, std::string("voxel count copy: ") + hipGetErrorString(e));
    }
    if (rc != LIDAR_OK) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    REQUIRE(hm[0] != -2, "lidar_voxel_downsample_f32: an in-launch hand-off timed out (a bug; please report)");
    REQUIRE(hm[0] != -3, "lidar_voxel_downsample_f32: an inconsistent voxel bucket table (a bug; please report)");
    REQUIRE(hm[0] >= 0, "lidar_voxel_downsample_f32: the extent is not finite or the voxel grid has 2^32 keys or more");
    *nvox_host = hm[0];
    return LIDAR_OK;
}
