// Measurement instrument (no reference counterpart).
//
// mog_copy_f4: the device's copy bandwidth, the yardstick the bench quotes
// next to the 8 TB/s spec for the HBM-bound fused step.
// (The test-only instruments are in csrc/testlib/instruments.hip.)
#include "mog_common.h"

namespace {

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
