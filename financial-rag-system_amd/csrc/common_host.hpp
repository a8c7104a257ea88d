// common_host.hpp — error plumbing for the C ABI (int status + thread-local message).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

// ---- diagnostic A/B knobs -------------------------------------------
// The RAGMI_* environment variables that switch kernels for A/B measurements (scan grid,
// seed sample, rescan grid, GEMM variants, attention variant, ...) are honoured only once a
// handle of this process was created with RAG_CREATE_DIAGNOSTIC (rag_index_create_ex's
// storage argument, rag_encoder_create_ex's flags). Otherwise every knob reads as its
// production default, and a knob that is set but ignored is reported once on stderr, so a
// stray variable in a serving process cannot change results or speed unnoticed.
inline std::atomic<bool>& diagnostics_on() {
  static std::atomic<bool> on{false};
  return on;
}

class Knob {
 public:
  explicit Knob(const char* name) : name_(name) {
    const char* v = std::getenv(name);
    set_ = v != nullptr;
    if (set_) text_ = v;
  }
  // integer value when honoured, else `dflt`
  int get(int dflt) {
    if (!honoured()) return dflt;
    return std::atoi(text_.c_str());
  }
  // string value when honoured, else nullptr
  const char* str() { return honoured() ? text_.c_str() : nullptr; }

 private:
  bool honoured() {
    if (!set_) return false;
    if (diagnostics_on().load(std::memory_order_relaxed)) return true;
    if (!warned_.exchange(true))
      std::fprintf(stderr,
                   "ragmi: %s=%s ignored: A/B knobs need a handle created with "
                   "RAG_CREATE_DIAGNOSTIC\n",
                   name_, text_.c_str());
    return false;
  }
  const char* name_;
  bool set_ = false;
  std::string text_;
  std::atomic<bool> warned_{false};
};

}  // namespace ragmi

#define RAG_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return ragmi::fail(_e == hipErrorOutOfMemory ? RAG_ENOMEM : RAG_EHIP,             \
                         std::string(#expr) + ": " + hipGetErrorString(_e));            \
  } while (0)
