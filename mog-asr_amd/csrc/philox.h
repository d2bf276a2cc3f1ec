// Philox4x32-10 noise quads shared by the stand-alone fill kernel (rng.hip) and
// the fused step kernel's in-kernel eps_x generation (vae_step.hip), so both
// produce identical bits for the same (seed, counter).  Quad q of a fill with
// base counter `offset` covers elements 4q .. 4q+3.
#pragma once
#include "mog_common.h"

__device__ __forceinline__ void mog_philox_round(uint32_t c[4], uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint64_t p0 = (uint64_t)M0 * c[0];
  const uint64_t p1 = (uint64_t)M1 * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
  c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}

// four values for counter `ctr`: standard normals (Box-Muller) or U[0,1)
__device__ __forceinline__ void mog_philox_quad(uint64_t seed, uint64_t ctr, bool normal,
                                                float v[4]) {
  uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u};
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    mog_philox_round(c, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  if (normal) {
    // Box-Muller on the hardware transcendentals: v_log_f32 (log2), v_sqrt_f32
    // and v_sin/v_cos_f32, whose argument is in revolutions (sin(2 pi u2)).
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float u1 = ((float)(c[2 * h] >> 8) + 1.0f) * 5.9604644775390625e-08f;  // (0,1]
      const float u2 = (float)(c[2 * h + 1] >> 8) * 5.9604644775390625e-08f;        // [0,1)
      const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
      v[2 * h] = r * __builtin_amdgcn_cosf(u2);
      v[2 * h + 1] = r * __builtin_amdgcn_sinf(u2);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (float)(c[k] >> 8) * 5.9604644775390625e-08f;
  }
}
