// Counter-based noise for perf mode (replaces the reference's tf.random_normal /
// tf.random_uniform sites: air_model.py:191, vae.py:29,44, concrete.py:23).
// Philox4x32-10; each thread emits 4 values.  Parity tests inject noise
// tensors instead (TF's RNG stream is not reproducible; SURVEY.md §7 'RNG').
#include "philox.h"

namespace {

__global__ __launch_bounds__(256) void rng_kernel(float* out, long n, uint64_t seed,
                                                  uint64_t offset, int normal) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;  // quad index
  const long i0 = q * 4;
  if (i0 >= n) return;
  float v[4];
  mog_philox_quad(seed, offset + (uint64_t)q, normal != 0, v);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (i0 + k < n) out[i0 + k] = v[k];
}

}  // namespace

extern "C" int mog_rng_fill(float* out, long n, unsigned long long seed,
                            unsigned long long offset, int normal, void* stream) {
  MOG_CHECK_ARG(out && n >= 0);
  if (n == 0) return 0;
  rng_kernel<<<mog_cdiv((n + 3) / 4, 256), 256, 0, mog_stream(stream)>>>(out, n, seed, offset,
                                                                        normal);
  MOG_LAUNCH_RET();
}
