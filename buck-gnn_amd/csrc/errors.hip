// Error reporting for the C-ABI: a per-thread message buffer (the wrappers are
// called from the Python thread for forward and from PyTorch's autograd thread
// for backward, so the message must not be shared between them).
#include "common.h"

namespace bgnn {

static thread_local char g_err[1024] = "no error";

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

}  // namespace bgnn

extern "C" int bgnn_abi_version(void) { return BGNN_ABI_VERSION; }

extern "C" const char* bgnn_last_error_string(void) { return bgnn::g_err; }
