// handle.hip — handle lifetime, thread-local errors, workspace growth.
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
    uint64_t want = align_up(bytes + bytes / 4, 1 << 20);
    if (h->ws) {
        // the previous workspace may still be read by queued kernels
        hipDeviceSynchronize();
        hipFree(h->ws);
        h->ws = nullptr;
        h->ws_bytes = 0;
    }
    if (hipMalloc(&h->ws, want) != hipSuccess) {
        h->ws = nullptr;
        set_error("workspace hipMalloc failed");
        return nullptr;
    }
    h->ws_bytes = want;
    return h->ws;
}

}  // namespace lidar

LIDAR_EXPORT int lidar_version(void) { return 1; }

LIDAR_EXPORT const char *lidar_last_error(void) { return lidar::g_err.c_str(); }

LIDAR_EXPORT int lidar_create(int device, lidar_handle **out)
{
    REQUIRE(out != nullptr, "lidar_create: out is NULL");
    *out = nullptr;
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return lidar::fail(LIDAR_EDEVICE, std::string("device is ") + prop.gcnArchName +
                                              ", this library is built for gfx950 only");
    lidar_handle *h = new lidar_handle();
    h->device = device;
    if (hipHostMalloc(&h->host_pinned, 4096, hipHostMallocDefault) != hipSuccess) {
        delete h;
        return lidar::fail(LIDAR_ENOMEM, "pinned host buffer allocation failed");
    }
    *out = h;
    return LIDAR_OK;
}

LIDAR_EXPORT int lidar_destroy(lidar_handle *h)
{
    if (!h) return LIDAR_OK;
    hipSetDevice(h->device);
    hipDeviceSynchronize();
    if (h->ws) hipFree(h->ws);
    if (h->host_pinned) hipHostFree(h->host_pinned);
    delete h;
    return LIDAR_OK;
}

LIDAR_EXPORT int lidar_reserve(lidar_handle *h, uint64_t bytes)
{
    REQUIRE(h != nullptr, "lidar_reserve: null handle");
    HIP_TRY(hipSetDevice(h->device));
    if (!lidar::workspace(h, bytes)) return LIDAR_ENOMEM;
    return LIDAR_OK;
}

// A stream restricted to a subset of the device's compute units (bit i of mask[i / 32]
// enables CU i).  Used by StreamingSSG to keep the latency-bound SA1 FPS chains and the
// MFMA levels on disjoint CUs.  Returns the hipStream_t through *out.
LIDAR_EXPORT int lidar_stream_create_cu_mask(int device, const uint32_t *mask, int32_t nwords, void **out)
{
    REQUIRE(mask && out && nwords > 0, "lidar_stream_create_cu_mask: bad arguments");
    HIP_TRY(hipSetDevice(device));
    hipStream_t s = nullptr;
    HIP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask));
    *out = s;
    return LIDAR_OK;
}

LIDAR_EXPORT int lidar_stream_destroy(void *stream)
{
    if (stream) HIP_TRY(hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return LIDAR_OK;
}

LIDAR_EXPORT int lidar_device_cu_count(int device, int32_t *out)
{
    REQUIRE(out, "lidar_device_cu_count: null pointer");
    int v = 0;
    HIP_TRY(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device));
    *out = v;
    return LIDAR_OK;
}
