// rt_host.h — internal helpers shared by the host-side translation units of librtamd.so.
#pragma once
#include <string>

namespace rtamd {
extern thread_local std::string g_error;
// Records `msg` as the thread's rt_last_error() and returns `code`.
int fail(int code, const std::string &msg);
}  // namespace rtamd
