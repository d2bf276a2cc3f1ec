// Spatial-transformer bilinear sampler (air/transformer.py:18-175) for gfx950.
//
// One workgroup (4 waves) per image: lanes walk output columns (the x-part of
// the affine grid is per-lane), waves walk output rows — no per-pixel integer
// division, no meshgrid / BatchMatMul tensors (transformer.py:119-163).  The
// four corners are gathered from the (L1/L2-resident, <= 16 KB) source image.
// Arithmetic is op-for-op the reference's (no contraction) so outputs are
// bit-identical to the oracle, including the out-of-window cancellation
// residue.
//
// A sample whose four clipped corners coincide (x0 == x1 AND y0 == y1) has the
// value +0 exactly (wa*I + wb*I cancels to 0, then -wa*I + wa*I = +0), so it is
// written as 0 without gathering, and in the canvas-accumulate mode skipped:
// c + z*0 == c bit-for-bit.  That removes the canvas read-modify-write outside
// the write window's cross-shaped support.
//
// The write direction (glimpse -> canvas, air_model.py:580-588) fuses the
// masked canvas accumulation of air_model.py:665-675:
//      canvas += active ? z * w : 0.
//
// Backward: one wave per image (see stn_bwd_kernel).  A sample whose clipped
// corners coincide on an axis (x0 == x1 or y0 == y1) contributes an exact
// mathematical zero to both dU and dtheta (its weights cancel pairwise), so it
// is skipped — the deterministic form of TF's gradient, which leaves
// order-dependent rounding residue there.  dot = sum_p G w still includes the
// singly-degenerate residue samples, so it is the exact adjoint of the forward
// value.  dU replaces TF's UnsortedSegmentSum (transformer.py:96-116).
#include "stn_geom.h"

namespace {

// Lane/row mapping: columns per pass CW = 32 (Wout <= 32, two rows per wave)
// or 64 (one row per wave); Wout > 64 falls back to a column loop.
struct RowMap {
  int cw, rw, sub, j;
};
__device__ __forceinline__ RowMap row_map(int Wout) {
  RowMap r;
  const int lane = threadIdx.x & 63;
  r.cw = Wout <= 32 ? 32 : 64;
  r.rw = 64 / r.cw;
  r.sub = lane / r.cw;
  r.j = lane % r.cw;
  return r;
}

// mode 0: out = v ; mode 1: out = mask ? out + z*v : out   (canvas accumulate)
// mode 2: out (bf16) = v  (glimpse as the bf16 A operand of the VAE GEMM)
template <int MODE>
__global__ __launch_bounds__(256) void stn_fwd_kernel(const float* __restrict__ U, int Hin,
                                                      int Win, const float* __restrict__ theta,
                                                      int Hout, int Wout, void* outv,
                                                      const float* __restrict__ z,
                                                      const float* __restrict__ mask) {
#pragma clang fp contract(off)
  const int n = blockIdx.x;
  const int P = Hout * Wout;
  if (MODE == 1 && !(mask[n] != 0.0f)) return;
  float th[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) th[k] = theta[n * 6 + k];
  const float* Un = U + (size_t)n * Hin * Win;
  const float zn = MODE == 1 ? z[n] : 0.0f;
  const RowMap rm = row_map(Wout);
  const int w = threadIdx.x >> 6;
  for (int j0 = 0; j0 < Wout; j0 += rm.cw) {
    const int j = j0 + rm.j;
    if (j >= Wout) continue;
    const float xt = mog_linspace(j, Wout);
    for (int i = w * rm.rw + rm.sub; i < Hout; i += 4 * rm.rw) {
      const float yt = mog_linspace(i, Hout);
      const Tap s = stn_tap(th, Hin, Win, xt, yt);
      const size_t o = (size_t)n * P + (size_t)i * Wout + j;
      if (MODE == 1) {
        if (s.dead) continue;  // contribution is exactly +0
        float* out = reinterpret_cast<float*>(outv);
        out[o] = out[o] + zn * tap_value(s, Un);
      } else {
        const float v = s.dead ? 0.0f : tap_value(s, Un);
        if (MODE == 2) reinterpret_cast<__bf16*>(outv)[o] = (__bf16)v;
        else reinterpret_cast<float*>(outv)[o] = v;
      }
    }
  }
}

// Backward, one wave per image (no workgroup barriers): lanes walk output
// columns (the column geometry stays in registers), the wave walks output
// rows with the cotangent rows prefetched one batch ahead.  The source image
// is staged in the wave's LDS slice; dU accumulates there with LDS atomics
// (one wave owns an image, so the accumulation order is fixed).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(256) void stn_bwd_kernel(
    const float* __restrict__ U, int N, int Hin, int Win, const float* __restrict__ theta,
    int Hout, int Wout, const float* __restrict__ G, const float* __restrict__ gscale, float* dU,
    float* dtheta, float* dot) {
#pragma clang fp contract(off)
  extern __shared__ float smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = blockIdx.x * (blockDim.x >> 6) + wv;
  if (n >= N) return;  // no workgroup barriers below
  const int HWin = Hin * Win, P = Hout * Wout;
  const bool want_dU = dU != nullptr;
  const int slice = (HWin * (want_dU ? 2 : 1) + 3) & ~3;
  float* sU = smem + wv * slice;
  float* sD = sU + HWin;
  float th[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) th[k] = theta[n * 6 + k];
  const bool sep = stn_separable(th) && Hin < 32768 && Win < 32768;
  const float* Un = U + (size_t)n * HWin;
  if ((HWin & 3) == 0) {
    const floatx4* src = reinterpret_cast<const floatx4*>(Un);
    for (int q = lane; q < HWin / 4; q += 64) reinterpret_cast<floatx4*>(sU)[q] = src[q];
  } else {
    for (int i = lane; i < HWin; i += 64) sU[i] = Un[i];
  }
  if (want_dU)
    for (int i = lane; i < HWin; i += 64) sD[i] = 0.0f;
  wave_sync();
  const float sc = gscale ? gscale[n] : 1.0f;
  const float wm2 = ((float)Win - 1.001f) / 2.0f;
  const float hm2 = ((float)Hin - 1.001f) / 2.0f;
  const bool grads = sc != 0.0f && (want_dU || dtheta != nullptr);
  float a[7] = {0, 0, 0, 0, 0, 0, 0};
  const float* Gn = G + (size_t)n * P;
  // Wout <= 32: two output rows per pass (lane halves), else one
  const int cw = Wout <= 32 ? 32 : 64, rp = 64 / cw;
  const int sub = lane / cw, jl = lane - sub * cw;
  for (int j0 = 0; j0 < Wout; j0 += cw) {
    const int j = j0 + jl;
    const bool jv = j < Wout;
    const int jc = jv ? j : Wout - 1;
    const float xt = mog_linspace(jc, Wout);
    const float4 ex_sep = axis4(axis_col(th, Hin, Win, Hout, Wout, jc), 1);
    // Cotangent rows are loaded unpredicated from clamped (always valid)
    // addresses, so the waitcnt pass can count the one-batch prefetch exactly
    // (a predicated load makes it wait for everything outstanding).
    constexpr int BR = 4;  // passes per batch
    float gq[BR], gn[BR];
#pragma unroll
    for (int u = 0; u < BR; ++u) gn[u] = Gn[min(sub + rp * u, Hout - 1) * Wout + jc];
    for (int i0 = 0; i0 < Hout; i0 += rp * BR) {
#pragma unroll
      for (int u = 0; u < BR; ++u) gq[u] = gn[u];
#pragma unroll
      for (int u = 0; u < BR; ++u)  // prefetch the next batch
        gn[u] = Gn[min(i0 + rp * BR + sub + rp * u, Hout - 1) * Wout + jc];
#pragma unroll
      for (int u = 0; u < BR; ++u) {
        const int i = i0 + sub + rp * u;
        if (!jv || i >= Hout) continue;
        const float yt = mog_linspace(i, Hout);
        float4 ex, ey;
        if (sep) {
          ex = ex_sep;
          ey = axis4(axis_row(th, Hin, Win, Hout, Wout, i), Win);
        } else {
          const Tap t = stn_tap(th, Hin, Win, xt, yt);
          ex = make_float4(__int_as_float((int)t.x0f), __int_as_float((int)t.x1f), t.x1f - t.x,
                           t.x - t.x0f);
          ey = make_float4(__int_as_float((int)t.y0f * Win), __int_as_float((int)t.y1f * Win),
                           t.y1f - t.y, t.y - t.y0f);
        }
        const int x0 = __float_as_int(ex.x), x1 = __float_as_int(ex.y);
        const int y0 = __float_as_int(ey.x), y1 = __float_as_int(ey.y);
        if (x0 == x1 && y0 == y1) continue;  // value and all gradients exactly 0
        const float Ia = sU[y0 + x0], Ib = sU[y1 + x0], Ic = sU[y0 + x1], Id = sU[y1 + x1];
        const float gout = gq[u];
        if (dot != nullptr) a[6] += gout * sample4(ex, ey, Ia, Ib, Ic, Id);
        const float g = gout * sc;
        if (!grads || x0 == x1 || y0 == y1 || g == 0.0f) continue;
        const float ax = ex.z, bx = ex.w, ay = ey.z, by = ey.w;
        if (want_dU) {
          atomicAdd(&sD[y0 + x0], ax * ay * g);
          atomicAdd(&sD[y1 + x0], ax * by * g);
          atomicAdd(&sD[y0 + x1], bx * ay * g);
          atomicAdd(&sD[y1 + x1], bx * by * g);
        }
        const float dx = g * (ay * (Ic - Ia) + by * (Id - Ib)) * wm2;
        const float dy = g * (ax * (Ib - Ia) + bx * (Id - Ic)) * hm2;
        a[0] += dx * xt; a[1] += dx * yt; a[2] += dx;
        a[3] += dy * xt; a[4] += dy * yt; a[5] += dy;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 7; ++k) a[k] = mog_wave_sum(a[k]);
  if (lane == 0) {
    if (dtheta)
      for (int k = 0; k < 6; ++k) dtheta[n * 6 + k] = a[k];
    if (dot) dot[n] = a[6];
  }
  if (!want_dU) return;
  wave_sync();
  float* dUn = dU + (size_t)n * HWin;
  if ((HWin & 3) == 0) {
    for (int q = lane; q < HWin / 4; q += 64)
      reinterpret_cast<floatx4*>(dUn)[q] = reinterpret_cast<const floatx4*>(sD)[q];
  } else {
    for (int i = lane; i < HWin; i += 64) dUn[i] = sD[i];
  }
}

}  // namespace

// transformer(U, theta, out_size) forward; see include/mog_air.h
extern "C" int mog_stn_forward(const float* U, int N, int Hin, int Win, const float* theta,
                               int Hout, int Wout, void* out, const float* z,
                               const float* mask, int mode, void* stream) {
  MOG_CHECK_ARG(U && theta && out && N >= 0 && Hin > 0 && Win > 0 && Hout > 0 && Wout > 0);
  MOG_CHECK_ARG(mode >= 0 && mode <= 2 && (mode != 1 || (z && mask)));
  if (N == 0) return 0;
  hipStream_t s = mog_stream(stream);
  if (mode == 1)
    stn_fwd_kernel<1><<<N, 256, 0, s>>>(U, Hin, Win, theta, Hout, Wout, out, z, mask);
  else if (mode == 2)
    stn_fwd_kernel<2><<<N, 256, 0, s>>>(U, Hin, Win, theta, Hout, Wout, out, nullptr, nullptr);
  else
    stn_fwd_kernel<0><<<N, 256, 0, s>>>(U, Hin, Win, theta, Hout, Wout, out, nullptr, nullptr);
  MOG_LAUNCH_RET();
}

extern "C" int mog_stn_backward(const float* U, int N, int Hin, int Win, const float* theta,
                                int Hout, int Wout, const float* G, const float* gscale,
                                float* dU, float* dtheta, float* dot, void* stream) {
  MOG_CHECK_ARG(U && theta && G && N >= 0 && Hin > 0 && Win > 0 && Hout > 0 && Wout > 0);
  MOG_CHECK_ARG(Hin * Win <= 16384);
  if (N == 0) return 0;
  const size_t slice = ((size_t)Hin * Win * (dU ? 2 : 1) + 3) & ~(size_t)3;
  int wpb = 4;  // waves (images) per workgroup, within 64 KiB of LDS
  while (wpb > 1 && slice * sizeof(float) * wpb > 64 * 1024) wpb >>= 1;
  MOG_CHECK_ARG(slice * sizeof(float) * wpb <= 160 * 1024);
  stn_bwd_kernel<<<mog_cdiv(N, wpb), 64 * wpb, slice * sizeof(float) * wpb,
                   mog_stream(stream)>>>(U, N, Hin, Win, theta, Hout, Wout, G, gscale, dU, dtheta,
                                         dot);
  MOG_LAUNCH_RET();
}
