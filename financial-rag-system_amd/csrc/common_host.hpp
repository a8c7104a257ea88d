// common_host.hpp — error plumbing for the C ABI (int status + thread-local message).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ragmi.h"

namespace ragmi {

inline std::string& last_error() {
  static thread_local std::string msg;
  return msg;
}

inline void clear_error() { last_error().clear(); }

inline int fail(int code, const std::string& msg) {
  last_error() = msg;
  return code;
}

}  // namespace ragmi

#define RAG_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return ragmi::fail(_e == hipErrorOutOfMemory ? RAG_ENOMEM : RAG_EHIP,             \
                         std::string(#expr) + ": " + hipGetErrorString(_e));            \
  } while (0)
