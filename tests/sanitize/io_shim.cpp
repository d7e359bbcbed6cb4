// io_shim.cpp — the two symbols gs_io.cpp takes from gs_capi.cpp (the thread-local last-error
// text), so the host-only scene-format code links into the sanitizer driver without HIP.
#include <string>

namespace gs {
static thread_local std::string g_io_error;
int io_fail(int code, const std::string& msg) {
    g_io_error = msg;
    return code;
}
}  // namespace gs

extern "C" const char* gs_last_error(void) { return gs::g_io_error.c_str(); }
