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
// seed sample, rescan grid, GEMM variant, LayerNorm modes, ...) are honoured only while a
// handle of this process created with RAG_CREATE_DIAGNOSTIC (rag_index_create_ex's storage
// argument, rag_encoder_create_ex's flags) is alive: a successful create counts it, its
// destroy releases it, and the first one says so on stderr. Otherwise every knob reads as its
// production default, and a knob that is set but ignored is reported once on stderr, so a
// stray variable in a serving process cannot change results or speed unnoticed.
inline std::atomic<int>& diagnostic_handles() {
  static std::atomic<int> n{0};
  return n;
}
inline void diagnostic_acquire() {
  static std::atomic<bool> said{false};
  diagnostic_handles().fetch_add(1);
  if (!said.exchange(true))
    std::fprintf(stderr, "ragmi: diagnostic handle created: RAGMI_* A/B knobs are honoured "
                         "while diagnostic handles live\n");
}
inline void diagnostic_release() { diagnostic_handles().fetch_sub(1); }

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
    if (diagnostic_handles().load(std::memory_order_relaxed) > 0) return true;
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
