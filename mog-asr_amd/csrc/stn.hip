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
// Backward: one workgroup per image.  dU is accumulated in LDS (no global
// atomics; replaces TF's UnsortedSegmentSum), dtheta is block-reduced.  A
// sample whose clipped corners coincide on an axis (x0 == x1 or y0 == y1)
// contributes an exact mathematical zero to both dU and dtheta (its weights
// cancel pairwise), so it is skipped — the deterministic form of TF's
// gradient, which leaves order-dependent rounding residue there.  dot =
// sum_p G w still includes the singly-degenerate residue samples, so it is the
// exact adjoint of the forward value.
#include "mog_common.h"

namespace {

struct Samp {
  float x, y, x0f, x1f, y0f, y1f;
  int ia, ib, ic, id;
  bool degenerate;  // corners coincide on at least one axis
  bool dead;        // corners coincide on both axes: value is +0 exactly
};

__device__ __forceinline__ Samp stn_sample(const float* th, int Hin, int Win, float xt,
                                           float yt) {
#pragma clang fp contract(off)
  Samp s;
  const float xs = (th[0] * xt + th[1] * yt) + th[2] * 1.0f;
  const float ys = (th[3] * xt + th[4] * yt) + th[5] * 1.0f;
  const float wm = (float)Win - 1.001f;
  const float hm = (float)Hin - 1.001f;
  s.x = ((xs + 1.0f) * wm) / 2.0f;
  s.y = ((ys + 1.0f) * hm) / 2.0f;
  const float fx = fminf(fmaxf(floorf(s.x), -1073741824.0f), 1073741824.0f);
  const float fy = fminf(fmaxf(floorf(s.y), -1073741824.0f), 1073741824.0f);
  int x0 = (int)fx, y0 = (int)fy;
  int x1 = x0 + 1, y1 = y0 + 1;
  x0 = min(max(x0, 0), Win - 1);
  x1 = min(max(x1, 0), Win - 1);
  y0 = min(max(y0, 0), Hin - 1);
  y1 = min(max(y1, 0), Hin - 1);
  s.x0f = (float)x0; s.x1f = (float)x1; s.y0f = (float)y0; s.y1f = (float)y1;
  s.ia = y0 * Win + x0; s.ib = y1 * Win + x0; s.ic = y0 * Win + x1; s.id = y1 * Win + x1;
  s.degenerate = (x0 == x1) || (y0 == y1);
  s.dead = (x0 == x1) && (y0 == y1);
  return s;
}

__device__ __forceinline__ float stn_value(const Samp& s, const float* U) {
#pragma clang fp contract(off)
  const float Ia = U[s.ia], Ib = U[s.ib], Ic = U[s.ic], Id = U[s.id];
  const float wa = (s.x1f - s.x) * (s.y1f - s.y);
  const float wb = (s.x1f - s.x) * (s.y - s.y0f);
  const float wc = (s.x - s.x0f) * (s.y1f - s.y);
  const float wd = (s.x - s.x0f) * (s.y - s.y0f);
  return ((wa * Ia + wb * Ib) + wc * Ic) + wd * Id;
}

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
      const Samp s = stn_sample(th, Hin, Win, xt, yt);
      const size_t o = (size_t)n * P + (size_t)i * Wout + j;
      if (MODE == 1) {
        if (s.dead) continue;  // contribution is exactly +0
        float* out = reinterpret_cast<float*>(outv);
        out[o] = out[o] + zn * stn_value(s, Un);
      } else {
        const float v = s.dead ? 0.0f : stn_value(s, Un);
        if (MODE == 2) reinterpret_cast<__bf16*>(outv)[o] = (__bf16)v;
        else reinterpret_cast<float*>(outv)[o] = v;
      }
    }
  }
}

// One block (256 threads) per image.
__global__ __launch_bounds__(256) void stn_bwd_kernel(
    const float* __restrict__ U, int Hin, int Win, const float* __restrict__ theta, int Hout,
    int Wout, const float* __restrict__ G, const float* __restrict__ gscale, float* dU,
    float* dtheta, float* dot) {
#pragma clang fp contract(off)
  extern __shared__ float sU[];
  __shared__ float red[8][4];
  const int n = blockIdx.x;
  const int HWin = Hin * Win, P = Hout * Wout;
  const bool want_dU = dU != nullptr;
  if (want_dU)
    for (int i = threadIdx.x; i < HWin; i += 256) sU[i] = 0.0f;
  __syncthreads();
  float th[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) th[k] = theta[n * 6 + k];
  const float sc = gscale ? gscale[n] : 1.0f;
  const float* Un = U + (size_t)n * HWin;
  const float* Gn = G + (size_t)n * P;
  const float wm2 = ((float)Win - 1.001f) / 2.0f;
  const float hm2 = ((float)Hin - 1.001f) / 2.0f;
  float a[7] = {0, 0, 0, 0, 0, 0, 0};
  const bool grads = sc != 0.0f && (want_dU || dtheta != nullptr);
  const RowMap rm = row_map(Wout);
  const int wv = threadIdx.x >> 6;
  for (int j0 = 0; j0 < Wout; j0 += rm.cw) {
    const int j = j0 + rm.j;
    if (j >= Wout) continue;
    const float xt = mog_linspace(j, Wout);
    for (int i = wv * rm.rw + rm.sub; i < Hout; i += 4 * rm.rw) {
      const float yt = mog_linspace(i, Hout);
      const Samp s = stn_sample(th, Hin, Win, xt, yt);
      if (s.dead) continue;  // value and all gradients are exactly 0
      const float gout = Gn[i * Wout + j];
      if (dot != nullptr) a[6] += gout * stn_value(s, Un);
      const float g = gout * sc;
      if (!grads || s.degenerate || g == 0.0f) continue;
      const float Ia = Un[s.ia], Ib = Un[s.ib], Ic = Un[s.ic], Id = Un[s.id];
      const float ax = s.x1f - s.x, bx = s.x - s.x0f, ay = s.y1f - s.y, by = s.y - s.y0f;
      if (want_dU) {
        atomicAdd(&sU[s.ia], ax * ay * g);
        atomicAdd(&sU[s.ib], ax * by * g);
        atomicAdd(&sU[s.ic], bx * ay * g);
        atomicAdd(&sU[s.id], bx * by * g);
      }
      const float dx = g * (ay * (Ic - Ia) + by * (Id - Ib)) * wm2;
      const float dy = g * (ax * (Ib - Ia) + bx * (Id - Ic)) * hm2;
      a[0] += dx * xt; a[1] += dx * yt; a[2] += dx;
      a[3] += dy * xt; a[4] += dy * yt; a[5] += dy;
    }
  }
  // block reduce 7 accumulators
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    float v = mog_wave_sum(a[k]);
    if (l == 0) red[k][wv] = v;
  }
  __syncthreads();
  if (threadIdx.x < 7) {
    const int k = threadIdx.x;
    const float v = (red[k][0] + red[k][1]) + (red[k][2] + red[k][3]);
    if (k < 6) {
      if (dtheta) dtheta[n * 6 + k] = v;
    } else if (dot) {
      dot[n] = v;
    }
  }
  if (want_dU)
    for (int i = threadIdx.x; i < HWin; i += 256) dU[(size_t)n * HWin + i] = sU[i];
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
  const size_t lds = dU ? (size_t)Hin * Win * sizeof(float) : 0;
  stn_bwd_kernel<<<N, 256, lds, mog_stream(stream)>>>(U, Hin, Win, theta, Hout, Wout, G, gscale,
                                                      dU, dtheta, dot);
  MOG_LAUNCH_RET();
}
