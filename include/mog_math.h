/*
 * mog_math.h — the framework's DEFINITION of the fp32 elementary functions
 * used on the AIR hot path (exp, log, expm1, tanh, sigmoid, TF softplus).
 *
 * Why this exists: TF-1.12 evaluates exp/log/tanh/sigmoid through Eigen's
 * vectorised approximations, whose bits are not reproducible outside TF
 * (TensorFlow is not installed here).  The reference's loss is
 * also bit-fragile: the STN write leaves a ~1e-8 cancellation residue outside
 * the window (transformer.py:108-116) which then passes through
 * log(r + 1e-10) (air_model.py:873-880).  To make GPU-vs-oracle parity a
 * bit-level statement instead of a tolerance argument, every elementwise
 * transcendental on the hot path is defined HERE, once, with only IEEE
 * add/sub/mul/div/sqrt/fma/rint and bit casts, so the HIP kernels (hipcc) and
 * the C oracle (gcc) produce identical bits.  Accuracy against libm is pinned
 * by tests/test_math_spec.py (<= 2 ulp on the tested ranges).
 *
 * Rules for this file: no FP contraction (each function body disables it), no
 * library math except sqrtf/rintf/fmaf/floorf (IEEE-exact on host and device).
 */
#ifndef MOG_MATH_H
#define MOG_MATH_H

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP_DEVICE_COMPILE__)
#define MOG_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define MOG_HD static inline
#endif

#ifdef __clang__
#define MOG_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define MOG_NOCONTRACT
#endif

MOG_HD float mog_bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
MOG_HD uint32_t mog_f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* 2^k for k in [-126, 127] as an exact float. */
MOG_HD float mog_pow2i(int k) { return mog_bits2f((uint32_t)(k + 127) << 23); }

/* exp(x): Cody-Waite reduction x = k ln2 + r, |r| <= ln2/2, degree-7 Taylor. */
MOG_HD float mog_expf(float x) {
  MOG_NOCONTRACT
  if (x != x) return x;
  if (x > 88.72283935546875f) return mog_bits2f(0x7f800000u);
  if (x < -103.972084045410156f) return 0.0f;
  const float kf = rintf(x * 1.44269502162933349609375f);
  float r = fmaf(kf, -0.693145751953125f, x);           /* ln2 hi (exact product) */
  r = fmaf(kf, -1.428606765330187045e-06f, r);           /* ln2 lo */
  float p = 1.98412698412698413e-04f;                     /* 1/7! */
  p = fmaf(p, r, 1.38888888888888889e-03f);               /* 1/6! */
  p = fmaf(p, r, 8.33333333333333333e-03f);               /* 1/5! */
  p = fmaf(p, r, 4.16666666666666667e-02f);               /* 1/4! */
  p = fmaf(p, r, 1.66666666666666667e-01f);               /* 1/3! */
  p = fmaf(p, r, 0.5f);
  p = fmaf(p, r, 1.0f);
  p = fmaf(p, r, 1.0f);
  int k = (int)kf;
  if (k > 127) { p = p * 2.0f; k -= 1; }
  if (k < -126) { p = p * mog_pow2i(-126); k += 126; }   /* gradual underflow */
  return p * mog_pow2i(k);
}

/* log(x): x = m 2^e, m in [sqrt(1/2), sqrt(2)), log1p(f) = 2 atanh(f/(2+f)). */
MOG_HD float mog_logf(float x) {
  MOG_NOCONTRACT
  if (x != x) return x;
  if (x < 0.0f) return mog_bits2f(0x7fc00000u);
  if (x == 0.0f) return mog_bits2f(0xff800000u);
  if (x == mog_bits2f(0x7f800000u)) return x;
  int e = 0;
  if (x < 1.17549435e-38f) { x = x * 8388608.0f; e = -23; } /* subnormal */
  uint32_t u = mog_f2bits(x);
  e += (int)((u >> 23) & 0xffu) - 127;
  u = (u & 0x007fffffu) | 0x3f800000u;                 /* m in [1,2) */
  float m = mog_bits2f(u);
  if (m > 1.41421353816986083984375f) { m = m * 0.5f; e += 1; }
  const float f = m - 1.0f;
  const float s = f / (2.0f + f);
  const float s2 = s * s;
  float p = 1.0f / 13.0f;
  p = fmaf(p, s2, 1.0f / 11.0f);
  p = fmaf(p, s2, 1.0f / 9.0f);
  p = fmaf(p, s2, 1.0f / 7.0f);
  p = fmaf(p, s2, 1.0f / 5.0f);
  p = fmaf(p, s2, 1.0f / 3.0f);
  const float l1p = fmaf(2.0f * s, s2 * p, 2.0f * s);  /* 2s + 2s^3 p */
  const float ef = (float)e;
  return fmaf(ef, 0.693145751953125f, fmaf(ef, 1.428606765330187045e-06f, l1p));
}

/* expm1(x): Taylor on |x| <= ln2/2, exp(x)-1 elsewhere. */
MOG_HD float mog_expm1f(float x) {
  MOG_NOCONTRACT
  if (x != x) return x;
  if (x > -0.3465735912322998046875f && x < 0.3465735912322998046875f) {
    float p = 2.75573192239858907e-06f;                   /* 1/9! */
    p = fmaf(p, x, 2.48015873015873016e-05f);             /* 1/8! */
    p = fmaf(p, x, 1.98412698412698413e-04f);
    p = fmaf(p, x, 1.38888888888888889e-03f);
    p = fmaf(p, x, 8.33333333333333333e-03f);
    p = fmaf(p, x, 4.16666666666666667e-02f);
    p = fmaf(p, x, 1.66666666666666667e-01f);
    p = fmaf(p, x, 0.5f);
    return fmaf(p * x, x, x);                              /* x + x^2 p */
  }
  if (x < -17.0f) return -1.0f;
  return mog_expf(x) - 1.0f;
}

/* tanh(x) = e/(e+2) with e = expm1(2x); saturates at |x| > 9.1. */
MOG_HD float mog_tanhf(float x) {
  MOG_NOCONTRACT
  if (x != x) return x;
  const float ax = x < 0.0f ? -x : x;
  float t;
  if (ax > 9.1f) {
    t = 1.0f;
  } else {
    const float e = mog_expm1f(2.0f * ax);
    t = e / (e + 2.0f);
  }
  return x < 0.0f ? -t : t;
}

/* logistic sigmoid 1/(1+exp(-x)). */
MOG_HD float mog_sigmoidf(float x) {
  MOG_NOCONTRACT
  return 1.0f / (1.0f + mog_expf(-x));
}

/* TF-1.12 Softplus (Eigen functor): x > -t -> x ; x < t -> exp(x) ;
 * else log(exp(x) + 1), t = log(FLT_EPSILON) + 2.  (vae.py:11,18-19,36-37) */
#define MOG_SOFTPLUS_T (-13.9423847198486328125f)
MOG_HD float mog_softplusf(float x) {
  MOG_NOCONTRACT
  if (x > -MOG_SOFTPLUS_T) return x;
  const float ex = mog_expf(x);
  if (x < MOG_SOFTPLUS_T) return ex;
  return mog_logf(ex + 1.0f);
}

/* log1p(x) for x > -1: log(u) * x / (u - 1) with u = 1 + x (exact when
 * u == 1), the rounding-compensated form; used by the ASR sigmoid
 * cross-entropy (tf.nn.sigmoid_cross_entropy_with_logits: log1p(exp(-|x|))). */
MOG_HD float mog_log1pf(float x) {
  MOG_NOCONTRACT
  if (x != x) return x;
  const float u = 1.0f + x;
  if (u == 1.0f) return x;
  if (u == mog_bits2f(0x7f800000u)) return u;
  return mog_logf(u) * (x / (u - 1.0f));
}

/* d softplus / dx = sigmoid(x), the gradient TF uses (SoftplusGrad). */
MOG_HD float mog_softplus_grad_from_pre(float x) {
  MOG_NOCONTRACT
  return mog_sigmoidf(x);
}

#endif /* MOG_MATH_H */
