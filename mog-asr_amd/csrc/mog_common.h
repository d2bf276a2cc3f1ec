// Common device helpers for the MI355X (gfx950) AIR hot-path kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mog_math.h"

#define MOG_WAVE 64

typedef float floatx4 __attribute__((ext_vector_type(4)));

// error codes returned by the C ABI besides hipError_t values
#define MOG_ERR_INVALID 1001

#define MOG_CHECK_ARG(cond) \
  do {                      \
    if (!(cond)) return MOG_ERR_INVALID; \
  } while (0)

#define MOG_LAUNCH_RET() return (int)hipGetLastError()

// propagate a nonzero status of a launch helper
#define MOG_TRY(expr)            \
  do {                           \
    const int mog_rc_ = (expr);  \
    if (mog_rc_ != 0) return mog_rc_; \
  } while (0)

static inline hipStream_t mog_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Profiling / A-B overrides (forced tile forms, phase masks, per-phase
// timing): read from the environment only in the profiling build
// (-DMOG_PROFILING: `make PROFILE=1`, mog_air/_lib/prof/libmog_air.so, loaded
// by the measurement scripts through MOG_AIR_LIB).  In the product library
// this is a constant nullptr: its launch paths never read the environment, so
// a test process and a bench process run the same code.
#ifdef MOG_PROFILING
#include <stdlib.h>
static inline const char* mog_prof_env(const char* name) { return getenv(name); }
#else
static inline constexpr const char* mog_prof_env(const char*) { return nullptr; }
#endif

static inline unsigned mog_cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

// wave64 sum via DPP-free shuffles
__device__ __forceinline__ float mog_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block sum for blockDim.x == 256; result valid in all threads. `red` >= 4 floats.
__device__ __forceinline__ float mog_block_sum256(float v, float* red) {
  v = mog_wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  const float r = (red[0] + red[1]) + (red[2] + red[3]);
  return r;
}

// TF LinSpace(-1, 1, n)[i] in fp32 (transformer.py:119-136)
__device__ __forceinline__ float mog_linspace(int i, int n) {
#pragma clang fp contract(off)
  if (n == 1) return -1.0f;
  if (i == n - 1) return 1.0f;
  const float step = 2.0f / (float)(n - 1);
  return -1.0f + step * (float)i;
}
