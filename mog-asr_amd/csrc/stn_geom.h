// Bilinear-sampler geometry shared by the STN kernels (stn.hip) and the fused
// step kernel (vae_step.hip): air/transformer.py:75-116 op for op (no
// contraction), so every consumer produces bit-identical samples.
#pragma once
#include "mog_common.h"

struct Tap {
  float x, y, x0f, x1f, y0f, y1f;
  int ia, ib, ic, id;
  bool degenerate;  // corners coincide on at least one axis: all gradients are exactly 0
  bool dead;        // corners coincide on both axes: the sample is +0 exactly
};

__device__ __forceinline__ Tap stn_tap(const float* th, int Hin, int Win, float xt, float yt) {
#pragma clang fp contract(off)
  Tap s;
  const float xs = (th[0] * xt + th[1] * yt) + th[2] * 1.0f;
  const float ys = (th[3] * xt + th[4] * yt) + th[5] * 1.0f;
  s.x = ((xs + 1.0f) * ((float)Win - 1.001f)) / 2.0f;
  s.y = ((ys + 1.0f) * ((float)Hin - 1.001f)) / 2.0f;
  const float fx = fminf(fmaxf(floorf(s.x), -1073741824.0f), 1073741824.0f);
  const float fy = fminf(fmaxf(floorf(s.y), -1073741824.0f), 1073741824.0f);
  int x0 = (int)fx, y0 = (int)fy;
  int x1 = x0 + 1, y1 = y0 + 1;
  x0 = min(max(x0, 0), Win - 1);
  x1 = min(max(x1, 0), Win - 1);
  y0 = min(max(y0, 0), Hin - 1);
  y1 = min(max(y1, 0), Hin - 1);
  s.degenerate = (x0 == x1) || (y0 == y1);
  s.dead = (x0 == x1) && (y0 == y1);
  s.x0f = (float)x0; s.x1f = (float)x1; s.y0f = (float)y0; s.y1f = (float)y1;
  s.ia = y0 * Win + x0; s.ib = y1 * Win + x0; s.ic = y0 * Win + x1; s.id = y1 * Win + x1;
  return s;
}

__device__ __forceinline__ float tap_value(const Tap& s, float Ia, float Ib, float Ic, float Id) {
#pragma clang fp contract(off)
  const float wa = (s.x1f - s.x) * (s.y1f - s.y);
  const float wb = (s.x1f - s.x) * (s.y - s.y0f);
  const float wc = (s.x - s.x0f) * (s.y1f - s.y);
  const float wd = (s.x - s.x0f) * (s.y - s.y0f);
  return ((wa * Ia + wb * Ib) + wc * Ic) + wd * Id;
}

__device__ __forceinline__ float tap_value(const Tap& s, const float* U) {
  return tap_value(s, U[s.ia], U[s.ib], U[s.ic], U[s.id]);
}

// Axis-aligned transforms (theta01 == theta10 == 0, always so in AIR) make the
// geometry separable: x depends on the output column only and y on the row only
// (th1*yt is +-0, and adding it leaves the sum bit-identical), so the
// coordinate and the clipped corner pair are tabulated once per column / row
// as {coordinate, lo | hi << 16}.
__device__ __forceinline__ bool stn_separable(const float* th) {
  return th[1] == 0.0f && th[3] == 0.0f;
}

__device__ __forceinline__ float2 axis_entry(float c, float lo_f, float hi_f) {
  return make_float2(c, __int_as_float((int)lo_f | ((int)hi_f << 16)));
}

__device__ __forceinline__ int axis_lo(float2 e) { return __float_as_int(e.y) & 0xffff; }
__device__ __forceinline__ int axis_hi(float2 e) { return __float_as_int(e.y) >> 16; }

// column entry j (of Wout) / row entry i (of Hout) of an axis-aligned transform
__device__ __forceinline__ float2 axis_col(const float* th, int Hin, int Win, int Hout, int Wout,
                                           int j) {
  const Tap t = stn_tap(th, Hin, Win, mog_linspace(j, Wout), mog_linspace(0, Hout));
  return axis_entry(t.x, t.x0f, t.x1f);
}
__device__ __forceinline__ float2 axis_row(const float* th, int Hin, int Win, int Hout, int Wout,
                                           int i) {
  const Tap t = stn_tap(th, Hin, Win, mog_linspace(0, Wout), mog_linspace(i, Hout));
  return axis_entry(t.y, t.y0f, t.y1f);
}

__device__ __forceinline__ Tap tap_from(float2 ex, float2 ey, int Win) {
  Tap s;
  const int x0 = axis_lo(ex), x1 = axis_hi(ex), y0 = axis_lo(ey), y1 = axis_hi(ey);
  s.x = ex.x; s.y = ey.x;
  s.x0f = (float)x0; s.x1f = (float)x1; s.y0f = (float)y0; s.y1f = (float)y1;
  s.ia = y0 * Win + x0; s.ib = y1 * Win + x0; s.ic = y0 * Win + x1; s.id = y1 * Win + x1;
  s.degenerate = (x0 == x1) || (y0 == y1);
  s.dead = (x0 == x1) && (y0 == y1);
  return s;
}

// Expanded axis entry for table-driven sampling: {lo * scale, hi * scale}
// (int bits; scale = source row pitch for the y axis, 1 for x) and the two
// interpolation weights {hi - c, c - lo}, computed exactly as tap_value does.
__device__ __forceinline__ float4 axis4(float2 e, int scale) {
  const int lo = axis_lo(e), hi = axis_hi(e);
  return make_float4(__int_as_float(lo * scale), __int_as_float(hi * scale), (float)hi - e.x,
                     e.x - (float)lo);
}

// Bilinear sample from expanded column (ex) and row (ey) entries:
// bit-identical to tap_value(stn_tap(...)), +0 when dead.
__device__ __forceinline__ bool axis4_dead(float4 ex, float4 ey) {
  return __float_as_int(ex.x) == __float_as_int(ex.y) && __float_as_int(ey.x) == __float_as_int(ey.y);
}
__device__ __forceinline__ float sample4(float4 ex, float4 ey, float Ia, float Ib, float Ic,
                                         float Id) {
#pragma clang fp contract(off)
  const float wa = ex.z * ey.z, wb = ex.z * ey.w, wc = ex.w * ey.z, wd = ex.w * ey.w;
  return ((wa * Ia + wb * Ib) + wc * Ic) + wd * Id;
}
