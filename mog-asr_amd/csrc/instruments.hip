// Measurement and test instruments (no reference counterpart).
//
// mog_copy_f4: the device's copy bandwidth, the yardstick the bench quotes
// next to the 8 TB/s spec for the HBM-bound fused step.
//
// mog_spin: one wave that occupies `stream` for a wall-clock interval.  tests/test_gpu_streams.py launches it at the head of
// one stream of a forked train step, so that a cross-stream dependency the
// host code forgot (a fork without its wait, a join without its event, a
// buffer the other stream still reads) turns from a rare timing accident into
// a failure on every run.
#include <cstdlib>

#include "mog_common.h"

namespace {

__global__ __launch_bounds__(64) void spin_kernel(long long ticks) {
  // wall_clock64: the constant 100 MHz counter; the wave sleeps between
  // polls.  ticks is capped by the host (<= 1 s), so every wave exits.
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// Fills the LDS of every CU with one 32-bit pattern (a NaN, say): run before
// a kernel, it makes any read of LDS that the kernel did not write first show
// up in its outputs instead of depending on what ran there before.
__global__ __launch_bounds__(256) void lds_poison_kernel(unsigned bits) {
  extern __shared__ unsigned lds_words[];
  constexpr int WORDS = 80 * 1024 / 4;
  for (int i = threadIdx.x; i < WORDS; i += 256)
    __hip_atomic_store(&lds_words[i], bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
}

// dst[i] = src[i] over n float4s: 16 B per lane per access, grid-stride,
// non-temporal stores (the copy's output is not re-read), 8 accesses in
// flight per lane
__global__ __launch_bounds__(256) void copy_f4_kernel(const float4* __restrict__ src,
                                                      float4* __restrict__ dst, long n) {
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 7 * stride < n; i += 8 * stride) {
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = src[i + k * stride];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      __builtin_nontemporal_store(*reinterpret_cast<floatx4*>(&v[k]),
                                  reinterpret_cast<floatx4*>(dst + i + k * stride));
  }
  for (; i < n; i += stride)
    __builtin_nontemporal_store(*reinterpret_cast<const floatx4*>(src + i),
                                reinterpret_cast<floatx4*>(dst + i));
}

// one float4 per lane, one grid pass, plain or nt stores
template <bool NT>
__global__ __launch_bounds__(256) void copy_f4_flat_kernel(const float4* __restrict__ src,
                                                           float4* __restrict__ dst, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    if (NT) __builtin_nontemporal_store(*reinterpret_cast<const floatx4*>(src + i),
                                        reinterpret_cast<floatx4*>(dst + i));
    else dst[i] = src[i];
  }
}

// U float4 per lane, lane-interleaved within a workgroup chunk, plain stores
template <int U>
__global__ __launch_bounds__(256) void copy_f4_chunk_kernel(const float4* __restrict__ src,
                                                            float4* __restrict__ dst, long n) {
  const long base = (long)blockIdx.x * 256 * U + threadIdx.x;
  float4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) v[k] = base + k * 256 < n ? src[base + k * 256] : float4{};
#pragma unroll
  for (int k = 0; k < U; ++k)
    if (base + k * 256 < n) dst[base + k * 256] = v[k];
}

}  // namespace

extern "C" int mog_copy_f4(const float* src, float* dst, long n4, void* stream) {
  MOG_CHECK_ARG(src && dst && n4 >= 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0 &&
                (reinterpret_cast<uintptr_t>(dst) & 15) == 0);
  if (n4 == 0) return 0;
  const float4* s4 = reinterpret_cast<const float4*>(src);
  float4* d4 = reinterpret_cast<float4*>(dst);
  hipStream_t s = mog_stream(stream);
  static const int variant = getenv("MOG_COPY_VARIANT") ? atoi(getenv("MOG_COPY_VARIANT")) : 0;
  switch (variant) {
    case 1: copy_f4_flat_kernel<false><<<mog_cdiv(n4, 256), 256, 0, s>>>(s4, d4, n4); break;
    case 2: copy_f4_flat_kernel<true><<<mog_cdiv(n4, 256), 256, 0, s>>>(s4, d4, n4); break;
    case 3: copy_f4_chunk_kernel<4><<<mog_cdiv(n4, 1024), 256, 0, s>>>(s4, d4, n4); break;
    case 4: copy_f4_chunk_kernel<8><<<mog_cdiv(n4, 2048), 256, 0, s>>>(s4, d4, n4); break;
    case 5: copy_f4_kernel<<<256 * 32, 256, 0, s>>>(s4, d4, n4); break;
    default: copy_f4_kernel<<<256 * 8, 256, 0, s>>>(s4, d4, n4); break;
  }
  MOG_LAUNCH_RET();
}

extern "C" int mog_lds_poison(unsigned bits, void* stream) {
  // 80 KiB per workgroup (two fill a CU's 160 KiB), eight rounds of them
  lds_poison_kernel<<<256 * 2 * 8, 256, 80 * 1024, mog_stream(stream)>>>(bits);
  MOG_LAUNCH_RET();
}

extern "C" int mog_spin(long long ticks, void* stream) {
  MOG_CHECK_ARG(ticks >= 0 && ticks <= 100000000LL);
  if (ticks == 0) return 0;
  spin_kernel<<<1, 64, 0, mog_stream(stream)>>>(ticks);
  MOG_LAUNCH_RET();
}
