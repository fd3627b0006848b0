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
