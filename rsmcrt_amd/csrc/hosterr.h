// hosterr.h — the per-thread message behind smcrt_last_error(), shared by the host-side
// translation units of libsmcrt.so.
#pragma once
#include <string>

namespace smcrt {
extern thread_local std::string g_last_error;
inline int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
}  // namespace smcrt
