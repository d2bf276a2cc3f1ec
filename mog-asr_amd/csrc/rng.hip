// Counter-based noise for perf mode (replaces the reference's tf.random_normal /
// tf.random_uniform sites: air_model.py:191, vae.py:29,44, concrete.py:23).
// Philox4x32-10; each thread emits 4 values.  Parity tests inject noise
// tensors instead (TF's RNG stream is not reproducible; SURVEY.md §7 'RNG').
#include "mog_common.h"

namespace {

__device__ __forceinline__ void philox_round(uint32_t c[4], uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint64_t p0 = (uint64_t)M0 * c[0];
  const uint64_t p1 = (uint64_t)M1 * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
  c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}

__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__global__ __launch_bounds__(256) void rng_kernel(float* out, long n, uint64_t seed,
                                                  uint64_t offset, int normal) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;  // quad index
  const long i0 = q * 4;
  if (i0 >= n) return;
  const uint64_t ctr = offset + (uint64_t)q;
  uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  float v[4];
  if (normal) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float u1 = ((float)(c[2 * h] >> 8) + 1.0f) * 5.9604644775390625e-08f;  // (0,1]
      const float u2 = (float)(c[2 * h + 1] >> 8) * 5.9604644775390625e-08f;        // [0,1)
      const float r = sqrtf(-2.0f * logf(u1));
      float sn, cs;
      sincosf(6.2831853071795865f * u2, &sn, &cs);
      v[2 * h] = r * cs;
      v[2 * h + 1] = r * sn;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (float)(c[k] >> 8) * 5.9604644775390625e-08f;
  }
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
