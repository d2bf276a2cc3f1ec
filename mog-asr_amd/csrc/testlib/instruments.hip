// Test-only instruments (include/mog_air_test.h), built into
// mog_air/_lib/libmog_air_test.so -- not part of the product library.
//
// mog_spin: one wave that occupies `stream` for a wall-clock interval.
// tests/test_gpu_streams.py launches it at the head of one stream of a forked
// train step, so that a cross-stream dependency the host code forgot (a fork
// without its wait, a join without its event, a buffer the other stream still
// reads) turns from a rare timing accident into a failure on every run.
//
// mog_lds_poison: every CU's LDS filled with one pattern before a kernel, so
// that a read of LDS the kernel did not write first shows in its outputs.
#include "../mog_common.h"
#include "../../../include/mog_air_test.h"

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

}  // namespace

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
