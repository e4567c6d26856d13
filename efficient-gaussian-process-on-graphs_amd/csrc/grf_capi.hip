// grf_capi.hip -- error reporting, version and device selection of the C ABI.
#include <stdarg.h>
#include <stdio.h>

#include "grf_common.h"

namespace grf {
static thread_local char g_err[1024] = "";
void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace grf

extern "C" {
#pragma GCC visibility push(default)

const char *grf_last_error(void) { return grf::g_err; }

int32_t grf_version(void) { return GRF_ABI_VERSION; }

int32_t grf_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int32_t grf_set_device(int32_t device) {
    GRF_CHECK_HIP(hipSetDevice(device));
    return GRF_OK;
}

// np.array_split(arange(n), n_chunks): the first n % n_chunks chunks hold one extra node
int64_t grf_chunk_bounds(int64_t n, int64_t n_chunks, int64_t c) {
    if (n_chunks <= 0) return 0;
    int64_t base = n / n_chunks, extra = n % n_chunks;
    return c * base + (c < extra ? c : extra);
}

}  // extern "C"
