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

// dst[i] = src[i] over n float4s: one 16-byte load and one non-temporal
// 16-byte store per lane, one pass of the grid (measured on MI355X against a
// grid-stride loop with 8 accesses in flight per lane, plain-store and 4- / 8-
// per-lane chunked forms: 6.31 TB/s for this form, 4.4-6.2 for the others;
// the guide's float4 copy: 6.29)
__global__ __launch_bounds__(256) void copy_f4_kernel(const float4* __restrict__ src,
                                                      float4* __restrict__ dst, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n)
    __builtin_nontemporal_store(*reinterpret_cast<const floatx4*>(src + i),
                                reinterpret_cast<floatx4*>(dst + i));
}

}  // namespace

extern "C" int mog_copy_f4(const float* src, float* dst, long n4, void* stream) {
  MOG_CHECK_ARG(src && dst && n4 >= 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0 &&
                (reinterpret_cast<uintptr_t>(dst) & 15) == 0);
  if (n4 == 0) return 0;
  copy_f4_kernel<<<mog_cdiv(n4, 256), 256, 0, mog_stream(stream)>>>(
      reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(dst), n4);
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
