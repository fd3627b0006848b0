// handle.hip — handle lifetime, thread-local errors, workspace growth, per-launch profiling.
#include <algorithm>
#include <cstring>
#include <string>

#include "common.hpp"

namespace lidar {

static thread_local std::string g_err;

void set_error(const std::string &msg) { g_err = msg; }

int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

void *workspace(lidar_handle *h, uint64_t bytes)
{
    if (bytes <= h->ws_bytes) return h->ws;
    // 25 % headroom, and at least double the current block: the retired blocks (freed by lidar_trim
    // where the caller knows the handle idle, or by lidar_destroy) then stay below the live block
    // however demand grows
    const uint64_t want = align_up(std::max(bytes + bytes / 4, 2 * h->ws_bytes), 1 << 20);
    void *fresh = nullptr;
    const hipError_t e = hipMalloc(&fresh, want);
    if (e != hipSuccess) {
        set_error(std::string("workspace hipMalloc(") + std::to_string(want) + "): " + hipGetErrorString(e));
        return nullptr;  // the current workspace stays as it was
    }
    if (h->ws) {
        // queued kernels (on whichever streams the caller used) may still read the old block:
        // retire it instead of synchronising the device (lidar_trim / lidar_destroy free it)
        h->retired.push_back(h->ws);
        h->retired_bytes += h->ws_bytes;
    }
    h->ws = fresh;
    h->ws_bytes = want;
    return h->ws;
}

static void drop_records(Prof *p)
{
    for (auto &r : p->recs) {
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    p->recs.clear();
}

}  // namespace lidar

LIDAR_EXPORT int lidar_version(void) { return 5; }

LIDAR_EXPORT const char *lidar_last_error(void) { return lidar::g_err.c_str(); }

LIDAR_EXPORT int lidar_create(int device, lidar_handle **out)
{
    REQUIRE(out != nullptr, "lidar_create: out is NULL");
    *out = nullptr;
    ON_DEVICE(device);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return lidar::fail(LIDAR_EDEVICE, std::string("device is ") + prop.gcnArchName +
                                              ", this library is built for gfx950 only");
    lidar_handle *h = new lidar_handle();
    h->device = device;
    const hipError_t e = hipHostMalloc(&h->host_pinned, 4096, hipHostMallocDefault);
    if (e != hipSuccess) {
        delete h;
        return lidar::fail(LIDAR_ENOMEM, std::string("pinned host buffer: ") + hipGetErrorString(e));
    }
    *out = h;
    return LIDAR_OK;
}

// Releases everything the handle owns.  Every step runs even if an earlier one fails (the
// handle is gone either way); the first failure is reported.
LIDAR_EXPORT int lidar_destroy(lidar_handle *h)
{
    if (!h) return LIDAR_OK;
    int rc = LIDAR_OK;
    auto note = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == LIDAR_OK) rc = lidar::fail(LIDAR_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    };
    {
        lidar::DeviceScope scope(h->device);
        note(scope.rc, "lidar_destroy: hipSetDevice");
        note(hipDeviceSynchronize(), "lidar_destroy: hipDeviceSynchronize");
        if (h->prof) {
            lidar::drop_records(h->prof);
            delete h->prof;
        }
        if (h->ws) note(hipFree(h->ws), "lidar_destroy: hipFree");
        if (h->vx_tags) note(hipFree(h->vx_tags), "lidar_destroy: hipFree (voxel tags)");
        for (void *r : h->retired) note(hipFree(r), "lidar_destroy: hipFree (retired workspace)");
        if (h->host_pinned) note(hipHostFree(h->host_pinned), "lidar_destroy: hipHostFree");
    }
    delete h;
    return rc;
}

LIDAR_EXPORT int lidar_reserve(lidar_handle *h, uint64_t bytes)
{
    REQUIRE(h != nullptr, "lidar_reserve: null handle");
    ON_DEVICE(h->device);
    if (!lidar::workspace(h, bytes)) return LIDAR_ENOMEM;
    return LIDAR_OK;
}

#ifdef LIDAR_DIAG
// testing aids: the diagnostic library only (`make diag`, liblidar_amd_diag.so), not the product ABI
namespace {
__global__ void fill_workspace_kernel(unsigned long long *w, uint64_t words, unsigned long long seed)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x)
        w[i] = ((unsigned long long)(i % 64 + 1) << 32) | (unsigned long long)(uint32_t)(seed * (i + 1));
}
}  // namespace

// Testing aid: grows the workspace to `bytes` and fills it with words whose high halves cycle through
// 1..64 (the tags the next in-launch hand-offs of a fresh handle use), on `stream`: no operation may
// trust what an earlier one left there (tests/test_gpu_tier_r.py::test_voxel_ignores_workspace_leftovers).
LIDAR_EXPORT int lidar_debug_fill_workspace(lidar_handle *h, uint64_t bytes, uint64_t seed, void *stream)
{
    REQUIRE(h != nullptr, "lidar_debug_fill_workspace: null handle");
    ON_DEVICE(h->device);
    void *w = lidar::workspace(h, bytes);
    if (!w) return LIDAR_ENOMEM;
    const uint64_t words = h->ws_bytes / 8;
    if (words == 0) return LIDAR_OK;
    hipLaunchKernelGGL(fill_workspace_kernel, dim3(1024), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<unsigned long long *>(h->ws), words, (unsigned long long)seed);
    LAUNCH_CHECK();
    return LIDAR_OK;
}

// Testing aid: sets the handle's call epoch (the next voxel call takes epoch + 1; 0xffffffff: it wraps).
LIDAR_EXPORT int lidar_debug_set_epoch(lidar_handle *h, uint32_t epoch)
{
    REQUIRE(h != nullptr, "lidar_debug_set_epoch: null handle");
    h->epoch = epoch;
    return LIDAR_OK;
}
#endif  // LIDAR_DIAG

// Frees the workspaces retired by growth.  The caller guarantees that no work it queued with this
// handle before the growth is still pending (e.g. after synchronising the streams it used).
LIDAR_EXPORT int lidar_trim(lidar_handle *h, uint64_t *freed)
{
    REQUIRE(h != nullptr, "lidar_trim: null handle");
    ON_DEVICE(h->device);
    const uint64_t bytes = h->retired_bytes;
    int rc = LIDAR_OK;
    for (void *r : h->retired) {
        const hipError_t e = hipFree(r);
        if (e != hipSuccess && rc == LIDAR_OK)
            rc = lidar::fail(LIDAR_EHIP, std::string("lidar_trim: hipFree: ") + hipGetErrorString(e));
    }
    h->retired.clear();
    h->retired_bytes = 0;
    if (freed) *freed = bytes;
    return rc;
}

// enable != 0: record HIP events around the handle's kernel phases from now on (previous records
// dropped); enable == 0: stop and drop the records.
LIDAR_EXPORT int lidar_profile(lidar_handle *h, int32_t enable)
{
    REQUIRE(h != nullptr, "lidar_profile: null handle");
    ON_DEVICE(h->device);
    if (h->prof) {
        lidar::drop_records(h->prof);
        if (!enable) {
            delete h->prof;
            h->prof = nullptr;
        }
    } else if (enable) {
        h->prof = new lidar::Prof();
    }
    return LIDAR_OK;
}

// The recorded spans in launch order: names '\n'-separated into `names` (names_cap bytes, NUL
// terminated), durations in ms into ms[0 .. *count); waits for the events and drops them.
LIDAR_EXPORT int lidar_profile_read(lidar_handle *h, char *names, int64_t names_cap, float *ms, int64_t cap,
                                    int64_t *count)
{
    REQUIRE(h && names && ms && count && names_cap > 0, "lidar_profile_read: null pointer");
    *count = 0;
    names[0] = '\0';
    if (!h->prof) return LIDAR_OK;
    ON_DEVICE(h->device);
    std::string joined;
    int64_t k = 0;
    int rc = LIDAR_OK;
    for (auto &r : h->prof->recs) {
        if (k >= cap) break;
        float t = 0.0f;
        hipError_t e = hipEventSynchronize(r.b);
        if (e == hipSuccess) e = hipEventElapsedTime(&t, r.a, r.b);
        if (e != hipSuccess && rc == LIDAR_OK)
            rc = lidar::fail(LIDAR_EHIP, std::string("lidar_profile_read: ") + hipGetErrorString(e));
        ms[k++] = t;
        joined += r.name;
        joined += '\n';
    }
    lidar::drop_records(h->prof);
    REQUIRE((int64_t)joined.size() < names_cap, "lidar_profile_read: names buffer too small");
    std::memcpy(names, joined.c_str(), joined.size() + 1);
    *count = k;
    return rc;
}

// ---- downsample_point_cloud's gather (utils/data_processing.py:247-249): rows copied as raw
// bytes, 16 / 8 / 4 / 1 bytes per lane by the row size's alignment; indices out of range are
// skipped (the host draws them with np.random.choice, always in range)
namespace {
template <class T>
__global__ void gather_rows_kernel(const T *__restrict__ src, int64_t n_rows, int64_t row_words,
                                   const int64_t *__restrict__ idx, int64_t k, T *__restrict__ dst)
{
    const int64_t total = k * row_words;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / row_words, w = e - r * row_words;
        const int64_t j = idx[r];
        if (j >= 0 && j < n_rows) dst[e] = src[j * row_words + w];
    }
}
}  // namespace

LIDAR_EXPORT int lidar_gather_rows(lidar_handle *h, const void *src, int64_t n_rows, int64_t row_bytes,
                                   const int64_t *idx, int64_t k, void *dst, void *stream)
{
    REQUIRE(h && (k == 0 || (src && idx && dst)), "lidar_gather_rows: null pointer");
    REQUIRE(n_rows >= 0 && row_bytes >= 0 && k >= 0, "lidar_gather_rows: negative size");
    if (k == 0 || row_bytes == 0) return LIDAR_OK;
    ON_DEVICE(h->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | (uintptr_t)row_bytes;
    auto go = [&](auto tag) {
        using T = decltype(tag);
        const int64_t words = row_bytes / (int64_t)sizeof(T), total = k * words;
        const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
        hipLaunchKernelGGL(gather_rows_kernel<T>, dim3(blocks), dim3(256), 0, s, static_cast<const T *>(src), n_rows,
                           words, idx, k, static_cast<T *>(dst));
    };
    if (al % 16 == 0) go(uint4{});
    else if (al % 8 == 0) go(uint2{});
    else if (al % 4 == 0) go(uint32_t{});
    else go(uint8_t{});
    LAUNCH_CHECK();
    return LIDAR_OK;
}
