// Shared host/device helpers for libleastereo_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "leastereo_hip.h"

namespace lea {

// Last error text of the calling host thread (lea_last_error()).
void set_error(const char* fmt, ...);
void clear_error();

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Map a launch result to the ABI return code, recording the HIP error string.
inline int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return static_cast<int>(e);
  }
  return LEA_OK;
}

#define LEA_CHECK_ARG(cond, ...)   \
  do {                             \
    if (!(cond)) {                 \
      ::lea::set_error(__VA_ARGS__); \
      return LEA_E_INVALID;        \
    }                              \
  } while (0)

constexpr int kWave = 64;

}  // namespace lea
