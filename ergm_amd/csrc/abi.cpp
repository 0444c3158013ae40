#include <cstdlib>
// Library-level C-ABI: version and thread-local error reporting (ergm_hip.h).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "common.h"

namespace ergm {

static thread_local char g_err[512] = {0};
thread_local LaunchBind g_bind;  // fork point bound to the next launches (common.h ERGM_LAUNCH)

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ERGM_EHIP, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
    return ERGM_OK;
}

}  // namespace ergm

extern "C" int ergm_version(void) { return ERGM_ABI_VERSION; }

extern "C" int ergm_last_error(char* buf, size_t n) {
    if (!buf || n == 0) return ERGM_EINVAL;
    strncpy(buf, ergm::g_err, n - 1);
    buf[n - 1] = 0;
    return ERGM_OK;
}
