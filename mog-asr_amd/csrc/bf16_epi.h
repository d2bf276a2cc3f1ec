// Element-wise epilogues of the bf16 configuration's VAE layers, shared by the
// fused step kernel (vae_step.hip) and the stand-alone bf16 GEMM
// (gemm_bf16.hip) so both produce identical bits.  Hardware transcendentals
// (v_exp_f32 = 2^x, v_log_f32 = log2, v_rcp_f32; ~1 ulp), branch-free: every
// arm is computed and selected, so an epilogue never diverges.  The
// bit-exact spec functions (include/mog_math.h) stay reserved for the fp32
// parity path.
#pragma once
#include "mog_common.h"

// TF softplus (vae.py:18-19,36-37): x above -T, exp(x) below T, log(exp(x) + 1)
// between the thresholds.
__device__ __forceinline__ float mog_softplus_hw(float v) {
  const float e = __builtin_amdgcn_exp2f(v * 1.44269504088896341f);
  const float l = __builtin_amdgcn_logf(e + 1.0f) * 0.693147180559945309f;
  const float r = v < MOG_SOFTPLUS_T ? e : l;
  return v > -MOG_SOFTPLUS_T ? v : r;
}

// sigmoid(y) = 1 / (1 + exp(-y)) (vae.py:44-46)
__device__ __forceinline__ float mog_sigmoid_hw(float y) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(y * -1.44269504088896341f));
}
