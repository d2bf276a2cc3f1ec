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
#include <stdio.h>

#include <algorithm>
#include <vector>

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
                                                      const float* __restrict__ mask,
                                                      int u_period) {
#pragma clang fp contract(off)
  const int n = blockIdx.x;
  const int P = Hout * Wout;
  if (MODE == 1 && !(mask[n] != 0.0f)) return;
  float th[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) th[k] = theta[n * 6 + k];
  const float* Un = U + (size_t)(u_period > 0 ? n % u_period : n) * Hin * Win;
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

// STN write of one image into its canvas part (the fp32 counterpart of the
// fused step kernel's write phase): part = mask ? z * STN(U, theta) : 0,
// stored only on the rows whose clipped corner rows differ (the others are
// exactly +0: their y weights cancel on one source row), widened to even
// bounds; part_rows[n] = lo | hi << 16 records them (0: inactive image, nothing
// stored).  mog_recon_loss sums the parts in step order, bit-identical to the
// running canvas accumulation (mode 1 above), so all T steps' writes run as
// one launch and the canvas is never read-modified-written.
__global__ __launch_bounds__(256) void stn_part_kernel(const float* __restrict__ U, int Hin,
                                                       int Win, const float* __restrict__ theta,
                                                       int Hout, int Wout, float* parts,
                                                       int* part_rows, const float* __restrict__ z,
                                                       const float* __restrict__ mask) {
#pragma clang fp contract(off)
  __shared__ int srange;
  const int n = blockIdx.x;
  const int P = Hout * Wout;
  if (!(mask[n] != 0.0f)) {
    if (threadIdx.x == 0) part_rows[n] = 0;
    return;
  }
  float th[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) th[k] = theta[n * 6 + k];
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int lo = 0, hi = Hout;
    if (stn_separable(th) && Hout <= 64 && (Hout & 1) == 0) {
      const float2 e = axis_row(th, Hin, Win, Hout, Wout, min(lane, Hout - 1));
      const unsigned long long lm =
          __builtin_amdgcn_ballot_w64(lane < Hout && axis_lo(e) != axis_hi(e));
      lo = lm ? (__builtin_ctzll(lm) & ~1) : 0;
      hi = lm ? min(Hout, (64 - __builtin_clzll(lm) + 1) & ~1) : 0;
    }
    if (lane == 0) {
      srange = lo | (hi << 16);
      part_rows[n] = lo | (hi << 16);
    }
  }
  __syncthreads();
  const int lo = srange & 0xffff, hi = srange >> 16;
  const float* Un = U + (size_t)n * Hin * Win;
  const float zn = z[n];
  const RowMap rm = row_map(Wout);
  const int w = threadIdx.x >> 6;
  float* out = parts + (size_t)n * P;
  for (int j0 = 0; j0 < Wout; j0 += rm.cw) {
    const int j = j0 + rm.j;
    if (j >= Wout) continue;
    const float xt = mog_linspace(j, Wout);
    for (int i = lo + w * rm.rw + rm.sub; i < hi; i += 4 * rm.rw) {
      const float yt = mog_linspace(i, Hout);
      const Tap s = stn_tap(th, Hin, Win, xt, yt);
      out[i * Wout + j] = s.dead ? 0.0f : zn * tap_value(s, Un);
    }
  }
}

// Backward, one wave per image (no workgroup barriers): lanes walk output
// columns (the column geometry stays in registers), the wave walks output
// rows with the cotangent rows prefetched one batch ahead.  The source image
// is staged in the wave's LDS slice.  For axis-aligned transforms (AIR's) the
// scaled cotangent g is kept as an LDS tile and dU is contracted separably,
// T = g Wx then dU = Wy^T T, each sum over the contiguous range of canvas
// columns / rows whose corner pair touches the source column / row (found
// with wave ballots) — no atomics (LDS float atomics cost ~40 LDS cycles per
// wave-instruction).  Other transforms accumulate dU with LDS atomics (one
// wave owns an image, so the order is fixed).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifdef MOG_STN_DEBUG
// diagnosis build only: every pixel's operands of the read backward
__device__ float* mog_stn_dbg = nullptr;
extern "C" int mog_stn_debug_set(float* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(mog_stn_dbg), &p, sizeof(p));
}
#endif

// The per-pixel loop of stn_bwd_kernel, specialised so the hot body has no
// branches: SEP (axis-aligned: geometry from the tables), DU (0 none,
// 1 separable g tile, 2 LDS atomics).
template <bool SEP, int DU>
__device__ __forceinline__ void bwd_pixels(const float* th, int Hin, int Win, int Hout, int Wout,
                                           const float* __restrict__ Gn, float sc, bool grads,
                                           bool want_dot, const float* sU, float* sD, float* sg,
                                           float4* coltab, const float4* rowtab, float* a) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const float wm2 = ((float)Win - 1.001f) / 2.0f;
  const float hm2 = ((float)Hin - 1.001f) / 2.0f;
  const float ystep = Hout > 1 ? 2.0f / (float)(Hout - 1) : 0.0f;
  // lane i holds the geometry of output row i (SEP: Hout <= 64)
  const float4 ry = SEP ? rowtab[min(lane, Hout - 1)] : make_float4(0.f, 0.f, 0.f, 0.f);
  // Wout <= 32: two output rows per pass (lane halves), else one
  const int cw = Wout <= 32 ? 32 : 64, rp = 64 / cw;
  const int sub = lane / cw, jl = lane - sub * cw;
  // SEP: only the rows whose clipped corner rows differ are walked.  A row
  // with y0 == y1 samples exactly +0 (its y weights are exact negatives on one
  // source row) and is degenerate, so it adds exactly nothing to dtheta or to
  // dot for a finite cotangent; those rows are a prefix and a suffix (the
  // row map increases).
  int ilo = 0, ihi = Hout;
  if (SEP) {
    const unsigned long long lm = __builtin_amdgcn_ballot_w64(
        lane < Hout && __float_as_int(ry.x) != __float_as_int(ry.y));
    ilo = lm ? (__builtin_ctzll(lm) / rp) * rp : 0;
    ihi = lm ? 64 - __builtin_clzll(lm) : 0;
  }
  for (int j0 = 0; j0 < Wout; j0 += cw) {
    const int j = j0 + jl;
    const bool jv = j < Wout;
    const int jc = jv ? j : Wout - 1;
    const float xt = mog_linspace(jc, Wout);
    float sdx = 0.0f, sdy = 0.0f;
    const float4 ex_sep = axis4(axis_col(th, Hin, Win, Hout, Wout, jc), 1);
    if (DU == 1 && jv) coltab[j] = ex_sep;
    // Cotangent rows are loaded unpredicated from clamped (always valid)
    // addresses, so the waitcnt pass can count the one-batch prefetch exactly
    // (a predicated load makes it wait for everything outstanding).
    constexpr int BR = 4;  // passes per batch
    float gq[BR], gn[BR];
#pragma unroll
    for (int u = 0; u < BR; ++u) gn[u] = Gn[min(ilo + sub + rp * u, Hout - 1) * Wout + jc];
    for (int i0 = ilo; i0 < ihi; i0 += rp * BR) {
#pragma unroll
      for (int u = 0; u < BR; ++u) gq[u] = gn[u];
#pragma unroll
      for (int u = 0; u < BR; ++u)  // prefetch the next batch
        gn[u] = Gn[min(i0 + rp * BR + sub + rp * u, Hout - 1) * Wout + jc];
      // Branch-free row bodies (masks instead of `continue`): the four rows'
      // LDS gathers can be in flight together.  Every gather index is a
      // valid clipped corner, so unmasked loads are safe.
#pragma unroll
      for (int u = 0; u < BR; ++u) {
        const int i = i0 + sub + rp * u;
        const bool valid = jv && i < Hout;
        const int ic = min(i, Hout - 1);
        const float yt = Hout == 1 ? -1.0f
                         : (ic == Hout - 1 ? 1.0f : -1.0f + ystep * (float)ic);  // = mog_linspace
        float4 ex, ey;
        if (SEP) {
          ex = ex_sep;
          // row geometry from the lane that owns the row (scalar broadcast, no LDS)
          const int ia = min(i0 + rp * u, Hout - 1), ib = min(i0 + 1 + rp * u, Hout - 1);
          const float4 ea = make_float4(
              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.x), ia)),
              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.y), ia)),
              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.z), ia)),
              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.w), ia)));
          if (rp == 1) {
            ey = ea;
          } else {
            const float4 eb = make_float4(
                __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.x), ib)),
                __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.y), ib)),
                __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.z), ib)),
                __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.w), ib)));
            ey = sub ? eb : ea;
          }
        } else {
          const Tap t = stn_tap(th, Hin, Win, xt, yt);
          ex = make_float4(__int_as_float((int)t.x0f), __int_as_float((int)t.x1f), t.x1f - t.x,
                           t.x - t.x0f);
          ey = make_float4(__int_as_float((int)t.y0f * Win), __int_as_float((int)t.y1f * Win),
                           t.y1f - t.y, t.y - t.y0f);
        }
        const int x0 = __float_as_int(ex.x), x1 = __float_as_int(ex.y);
        const int y0 = __float_as_int(ey.x), y1 = __float_as_int(ey.y);
        const bool dead = x0 == x1 && y0 == y1;
        const bool degen = x0 == x1 || y0 == y1;
        const float Ia = sU[y0 + x0], Ib = sU[y1 + x0], Ic = sU[y0 + x1], Id = sU[y1 + x1];
        const float gout = gq[u];
        const float pv = gout * sample4(ex, ey, Ia, Ib, Ic, Id);
        a[6] += (want_dot && valid && !dead) ? pv : 0.0f;
        const float g0 = gout * sc;
        const bool use = valid && grads && !degen && g0 != 0.0f;
        const float g = use ? g0 : 0.0f;  // value and gradients exactly 0 where !use
        const float ax = ex.z, bx = ex.w, ay = ey.z, by = ey.w;
        if (DU == 2 && use) {
          atomicAdd(&sD[y0 + x0], ax * ay * g);
          atomicAdd(&sD[y1 + x0], ax * by * g);
          atomicAdd(&sD[y0 + x1], bx * ay * g);
          atomicAdd(&sD[y1 + x1], bx * by * g);
        }
        const float dx = g * (ay * (Ic - Ia) + by * (Id - Ib)) * wm2;
        const float dy = g * (ax * (Ib - Ia) + bx * (Id - Ic)) * hm2;
#ifdef MOG_STN_DEBUG
        if (mog_stn_dbg != nullptr && valid && SEP && DU == 0) {
          const int nn = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
          float* d = mog_stn_dbg + (((size_t)nn * Hout + i) * Wout + j) * 16;
          d[0] = gout; d[1] = Ia; d[2] = Ib; d[3] = Ic; d[4] = Id; d[5] = ax; d[6] = bx;
          d[7] = ay; d[8] = by; d[9] = __int_as_float(x0); d[10] = __int_as_float(x1);
          d[11] = __int_as_float(y0); d[12] = __int_as_float(y1); d[13] = dx; d[14] = dy;
          d[15] = g;
        }
#endif
        // the column coordinate xt is constant per lane: sum_rows dx, scaled once
        sdx += dx; a[1] += dx * yt;
        sdy += dy; a[4] += dy * yt;
      }
    }
    a[0] += sdx * xt; a[2] += sdx;
    a[3] += sdy * xt; a[5] += sdy;
  }
}

// Axis-aligned transform, 32 < Wout <= 64 (one output row per pass: the STN
// write backward, canvas -> glimpse): every live cotangent row of the lane's
// column is loaded up front into registers gv[] (one memory latency per
// image instead of one per 4-row batch), the row bodies then run from
// registers, and gv[] stays live for the separable dU pass (lanes exchange
// it with ds_bpermute, no second read of the cotangent).  The per-row body,
// its order and its masks are bwd_pixels<true, DU>'s.
constexpr int GV = 64;  // rows held per lane (Hout <= 64)

// Row geometry of the lane's output row (lane i -> row i) and the live row
// range [ilo, ihi): rows whose clipped corner rows differ (a prefix and a
// suffix of the rows are degenerate; they add exactly nothing).
__device__ __forceinline__ float4 live_rows(const float* th, int Hin, int Win, int Hout, int Wout,
                                            int& ilo, int& ihi) {
  const int lane = threadIdx.x & 63;
  const float4 ry = axis4(axis_row(th, Hin, Win, Hout, Wout, min(lane, Hout - 1)), Win);
  const unsigned long long lm = __builtin_amdgcn_ballot_w64(
      lane < Hout && __float_as_int(ry.x) != __float_as_int(ry.y));
  ilo = lm ? __builtin_ctzll(lm) : 0;
  ihi = lm ? 64 - __builtin_clzll(lm) : 0;
  return ry;
}

// all live cotangent rows of the lane's column into gv[] (clamped rows:
// unpredicated loads, 16 per chunk), issued before the image is staged so
// the two latencies overlap
__device__ __forceinline__ void load_rows(const float* __restrict__ Gn, int Hout, int Wout, int ilo,
                                          int ihi, float (&gv)[GV]) {
  const int lane = threadIdx.x & 63;
  const int jc = lane < Wout ? lane : Wout - 1;
#pragma unroll
  for (int c = 0; c < GV / 16; ++c) {
    if (16 * c < ihi - ilo) {
#pragma unroll
      for (int r = 16 * c; r < 16 * c + 16; ++r) gv[r] = Gn[min(ilo + r, Hout - 1) * Wout + jc];
    }
  }
}

template <int DU>
__device__ __forceinline__ void bwd_rows_reg(const float* th, int Hin, int Win, int Hout,
                                             int Wout, float sc, bool grads, bool want_dot,
                                             const float* sU, float4* coltab, const float4 ry,
                                             int ilo, int ihi, float* a, const float (&gv)[GV]) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const float wm2 = ((float)Win - 1.001f) / 2.0f;
  const float hm2 = ((float)Hin - 1.001f) / 2.0f;
  const float ystep = Hout > 1 ? 2.0f / (float)(Hout - 1) : 0.0f;
  const int j = lane;
  const bool jv = j < Wout;
  const int jc = jv ? j : Wout - 1;
  const float xt = mog_linspace(jc, Wout);
  const float4 ex = axis4(axis_col(th, Hin, Win, Hout, Wout, jc), 1);
  if (DU == 1 && jv) coltab[j] = ex;
  const int x0 = __float_as_int(ex.x), x1 = __float_as_int(ex.y);
  const float ax = ex.z, bx = ex.w;
  float sdx = 0.0f, sdy = 0.0f;
  // rows in groups of four: one uniform branch per group, so the four rows'
  // LDS gathers are in flight together (rows past ihi are clamped and masked)
#pragma unroll
  for (int r = 0; r < GV; ++r) {
    if (r % 4 == 0 && ilo + r >= ihi) break;
    const bool rv = ilo + r < ihi;
    const int i = min(ilo + r, ihi - 1);
    const float yt = Hout == 1 ? -1.0f : (i == Hout - 1 ? 1.0f : -1.0f + ystep * (float)i);
    const float4 ey = make_float4(
        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.x), i)),
        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.y), i)),
        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.z), i)),
        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry.w), i)));
    const int y0 = __float_as_int(ey.x), y1 = __float_as_int(ey.y);
    const bool dead = x0 == x1 && y0 == y1;
    const bool degen = x0 == x1 || y0 == y1;
    const float Ia = sU[y0 + x0], Ib = sU[y1 + x0], Ic = sU[y0 + x1], Id = sU[y1 + x1];
    const float gout = gv[r];
    const float pv = gout * sample4(ex, ey, Ia, Ib, Ic, Id);
    a[6] += (want_dot && jv && rv && !dead) ? pv : 0.0f;
    const float g0 = gout * sc;
    const bool use = jv && rv && grads && !degen && g0 != 0.0f;
    const float g = use ? g0 : 0.0f;
    const float ay = ey.z, by = ey.w;
    const float dx = g * (ay * (Ic - Ia) + by * (Id - Ib)) * wm2;
    const float dy = g * (ax * (Ib - Ia) + bx * (Id - Ic)) * hm2;
    sdx += dx; a[1] += dx * yt;
    sdy += dy; a[4] += dy * yt;
  }
  a[0] += sdx * xt; a[2] += sdx;
  a[3] += sdy * xt; a[5] += sdy;
}

// floats of one wave's LDS slice (max over the atomic and separable layouts)
__host__ __device__ inline int stn_bwd_slice(int Hin, int Win, int Hout, int Wout, bool dU) {
  const int hw4 = (Hin * Win + 3) & ~3;
  const int atomic_l = hw4 * (dU ? 2 : 1) + 4 * Hout;
  const int sep_l = ((hw4 > ((Hout * Win + 3) & ~3)) ? hw4 : ((Hout * Win + 3) & ~3)) +
                    4 * 64 + 4 * 64 + 2 * 64;
  return dU && atomic_l < sep_l ? sep_l : atomic_l;
}

#define TS(k) if (ts && lane == 0) ts[(size_t)n * 8 + (k)] = wall_clock64()
// One image of stn_bwd_kernel.  REGS: the rows-in-registers form (see
// bwd_rows_reg), a separate instantiation so the other forms' register
// allocation never sees its 64 cotangent registers.
template <bool REGS>
__device__ __forceinline__ void stn_bwd_image(
    const float* __restrict__ U, int Hin, int Win, const float* th, int Hout, int Wout,
    const float* __restrict__ G, const float* __restrict__ gscale, float* dU, float* dtheta,
    float* dot, int u_period, int g_period, long long* ts, int du_mode, int n, int lane, int wv,
    bool sep, bool sdu) {
#pragma clang fp contract(off)
  extern __shared__ float smem[];
  const int HWin = Hin * Win, P = Hout * Wout;
  const bool want_dU = dU != nullptr;
  const int slice = stn_bwd_slice(Hin, Win, Hout, Wout, want_dU);
  const int hw4 = (HWin + 3) & ~3;
  float* sU = smem + wv * slice;
  // atomic path: [U | dU | rows];  separable path: [U, then T | g | cols | rows | ranges]
  float* sD = sU + hw4;
  float* sT = sU;
  float* sg = sU + max(hw4, (Hout * Win + 3) & ~3);
  float4* coltab = reinterpret_cast<float4*>(sg);
  float4* rowtab = sdu ? coltab + 64 : reinterpret_cast<float4*>(sU + hw4 * (want_dU ? 2 : 1));
  int2* vrange = reinterpret_cast<int2*>(rowtab + 64);
  const float* Un = U + (size_t)(u_period > 0 ? n % u_period : n) * HWin;
  const float* Gn = G + (size_t)(g_period > 0 ? n % g_period : n) * P;
  // rows in registers: axis-aligned, one output row per pass, separable or no
  // dU, image staged by 16-byte loads (the write backward, canvas <- glimpse)
  const int mode = __builtin_amdgcn_readfirstlane((sep ? 1 : 0) | (sdu ? 2 : 0) | (want_dU ? 4 : 0));
  constexpr bool regs = REGS;
  float gv[GV];
  int rlo = 0, rhi = 0;
  float4 ry = make_float4(0.f, 0.f, 0.f, 0.f);
  if (regs) {
    // image -> registers, cotangent rows -> registers, then image -> LDS: the
    // write to LDS waits only for the image loads (issued first)
    const floatx4* src = reinterpret_cast<const floatx4*>(Un);
    floatx4 us[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) us[k] = src[min(lane + 64 * k, HWin / 4 - 1)];
    ry = live_rows(th, Hin, Win, Hout, Wout, rlo, rhi);
    load_rows(Gn, Hout, Wout, rlo, rhi, gv);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (lane + 64 * k < HWin / 4) reinterpret_cast<floatx4*>(sU)[lane + 64 * k] = us[k];
    if (lane < Hout) rowtab[lane] = ry;
  } else if ((HWin & 3) == 0) {
    // axis-aligned without dU (the STN read backward, glimpse <- canvas):
    // only the source rows between the clipped corner rows of output rows 0
    // and Hout - 1 (the map is monotonic, so every row's corners lie there)
    // are staged -- the window's rows, not the whole canvas
    int q0 = 0, q1 = HWin / 4;
    if (mode == 1) {
      const float2 ea = axis_row(th, Hin, Win, Hout, Wout, 0);
      const float2 eb = axis_row(th, Hin, Win, Hout, Wout, Hout - 1);
      const int ylo = min(min(axis_lo(ea), axis_hi(ea)), min(axis_lo(eb), axis_hi(eb)));
      const int yhi = max(max(axis_lo(ea), axis_hi(ea)), max(axis_lo(eb), axis_hi(eb)));
      q0 = (ylo * Win) >> 2;
      q1 = min(HWin / 4, ((yhi + 1) * Win + 3) >> 2);
    }
    const floatx4* src = reinterpret_cast<const floatx4*>(Un);
    for (int q = q0 + lane; q < q1; q += 64) reinterpret_cast<floatx4*>(sU)[q] = src[q];
  } else {
    for (int i = lane; i < HWin; i += 64) sU[i] = Un[i];
  }
  if (want_dU && !sdu)
    for (int i = lane; i < HWin; i += 64) sD[i] = 0.0f;
  if (sep && !regs)  // row geometry once per image (lane i -> row i)
    for (int i = lane; i < Hout; i += 64) rowtab[i] = axis4(axis_row(th, Hin, Win, Hout, Wout, i), Win);
  wave_sync();
  TS(1);
  const float sc = gscale ? gscale[n] : 1.0f;
  const bool grads = sc != 0.0f && (want_dU || dtheta != nullptr);
  float a[7] = {0, 0, 0, 0, 0, 0, 0};
  if (regs) {
    if (mode == 1)
      bwd_rows_reg<0>(th, Hin, Win, Hout, Wout, sc, grads, dot != nullptr, sU, coltab, ry, rlo,
                      rhi, a, gv);
    else
      bwd_rows_reg<1>(th, Hin, Win, Hout, Wout, sc, grads, dot != nullptr, sU, coltab, ry, rlo,
                      rhi, a, gv);
  } else if (mode == 3 || mode == 7)
    bwd_pixels<true, 1>(th, Hin, Win, Hout, Wout, Gn, sc, grads, dot != nullptr, sU, sD, sg, coltab, rowtab, a);
  else if (mode == 5)
    bwd_pixels<true, 2>(th, Hin, Win, Hout, Wout, Gn, sc, grads, dot != nullptr, sU, sD, sg, coltab, rowtab, a);
  else if (mode == 1)
    bwd_pixels<true, 0>(th, Hin, Win, Hout, Wout, Gn, sc, grads, dot != nullptr, sU, sD, sg, coltab, rowtab, a);
  else if (mode & 4)
    bwd_pixels<false, 2>(th, Hin, Win, Hout, Wout, Gn, sc, grads, dot != nullptr, sU, sD, sg, coltab, rowtab, a);
  else
    bwd_pixels<false, 0>(th, Hin, Win, Hout, Wout, Gn, sc, grads, dot != nullptr, sU, sD, sg, coltab, rowtab, a);
#pragma unroll
  for (int k = 0; k < 7; ++k) a[k] = mog_wave_sum(a[k]);
  if (lane == 0) {
    if (dtheta)
      for (int k = 0; k < 6; ++k) dtheta[n * 6 + k] = a[k];
    if (dot) dot[n] = a[6];
  }
  TS(2);
  if (!want_dU) return;
  wave_sync();
  // du_mode 1 / 2: the glimpse gradient leaves through the VAE output
  // sigmoid (vae.py:44-46; TF SigmoidGrad dm = (dr * r) * (1 - r), r = U) as
  // bf16 / fp32 -- bit-identical to dU followed by mog_sigmoid_backward
  float* dUn = dU + (size_t)n * HWin;
  __bf16* dMn = reinterpret_cast<__bf16*>(dU) + (size_t)n * HWin;
  auto put_u = [&](int idx, float d, float v) {
    if (du_mode) {
      const float m = (d * v) * (1.0f - v);
      if (du_mode == 1) dMn[idx] = (__bf16)m;
      else dUn[idx] = m;
    } else {
      dUn[idx] = d;
    }
  };
  auto put = [&](int idx, float d) {
    if (du_mode) {
      const float v = Un[idx];
      const float m = (d * v) * (1.0f - v);
      if (du_mode == 1) dMn[idx] = (__bf16)m;
      else dUn[idx] = m;
    } else {
      dUn[idx] = d;
    }
  };
  if (sdu) {
    // contiguous index ranges (the maps increase): canvas columns j whose
    // corner pair touches source column u, canvas rows i touching source row v
    // Degenerate (clipped, x0 == x1) columns carry g == 0: give them sentinel
    // corners before (left clip) or after (right clip) every source column so
    // no range includes them — otherwise the ranges of the edge columns 0 and
    // W-1 would span every clipped canvas column.
    int x0l = 1 << 30, x1l = 1 << 30, y0l = 1 << 30, y1l = 1 << 30;
    if (lane < Wout) {
      const float4 e = coltab[lane];
      x0l = __float_as_int(e.x);
      x1l = __float_as_int(e.y);
      if (x0l == x1l) x0l = x1l = (x0l == 0) ? -1 : (1 << 30);
    }
    if (lane < Hout) {
      const float4 e = rowtab[lane];
      y0l = __float_as_int(e.x) / Win;
      y1l = __float_as_int(e.y) / Win;
      if (y0l == y1l) y0l = y1l = (y0l == 0) ? -1 : (1 << 30);
    }
    const int cwi = Win <= 32 ? 32 : 64, rpi = 64 / cwi;
    const int ul = lane % cwi, half = lane / cwi;
    constexpr int UV = 16;  // dU outputs per lane held up front (Hin <= 16 rpi)
    const bool upre = du_mode != 0 && rpi * UV >= Hin;
    float uv[UV];
    int jlo = 0, jhi = -1;
    for (int u = 0; u < Win; ++u) {
      const int lo = __popcll(__ballot(x1l < u));
      const int hi = __popcll(__ballot(x0l <= u)) - 1;
      if (ul == u) { jlo = lo; jhi = hi; }
    }
    for (int v = 0; v < Hin; ++v) {
      const int lo = __popcll(__ballot(y1l < v));
      const int hi = __popcll(__ballot(y0l <= v)) - 1;
      if (lane == 0) vrange[v] = make_int2(lo, hi);
    }
    // T[i][u] = sum_j g[i][j] * (x0(j) == u ? x1 - x : x - x0)   (U is dead: T reuses it)
    // j outer, the lane's rows inner: the row reads are independent (ILP).
    // g is recomputed from the (L1/L2-resident) cotangent exactly as the pixel
    // loop forms it -- g = G * sc where the sample is not degenerate, else 0;
    // the columns of [jlo, jhi] are never degenerate, so only the row test
    // remains -- instead of being staged in LDS (a 10 KB tile per wave that
    // held the kernel to two waves per SIMD).
    // The rows with y0 == y1 (a prefix and a suffix) are never read by the dU
    // pass (no row range includes them): T is formed for the live rows only.
    // (Ballot over the whole wave, before the lane test below.)
    const unsigned long long lmr = __builtin_amdgcn_ballot_w64(
        lane < Hout && __float_as_int(rowtab[min(lane, Hout - 1)].x) !=
                           __float_as_int(rowtab[min(lane, Hout - 1)].y));
    // the cotangent through a buffer descriptor (built in uniform control flow
    // from uniform values, so it lives in SGPRs: no waterfall loop per load):
    // 32-bit offsets, no 64-bit address registers per load
    const unsigned long long gp = reinterpret_cast<unsigned long long>(Gn);
    const unsigned glo = __builtin_amdgcn_readfirstlane((unsigned)gp);
    const unsigned ghi = __builtin_amdgcn_readfirstlane((unsigned)(gp >> 32));
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<float*>(((unsigned long long)ghi << 32) | glo), 0,
        __builtin_amdgcn_readfirstlane(P * 4), 0x00020000);
    const int tlo = lmr ? (__builtin_ctzll(lmr) / rpi) * rpi : Hout;
    const int thi = lmr ? 64 - __builtin_clzll(lmr) : Hout;
    if (regs) {
      // T[i][u] = sum_{j = jlo(u)..jhi(u)} g[i][j] w_j(u), j ascending (the order
      // of the loop below); lane j's g[i][j] arrives by ds_bpermute, so every
      // lane takes part in each exchange and lanes u >= Win discard theirs.
      // The live rows [rlo, rhi) are exactly [tlo, thi) for one row per pass.
      constexpr int JM = 8;  // canvas columns per source column (<= 8: scale <= ~2)
      const bool uact = ul < Win && half == 0;
      const int nj = uact ? jhi - jlo + 1 : 0;
      int jmax = nj;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) jmax = max(jmax, __shfl_xor(jmax, o, 64));
      jmax = __builtin_amdgcn_readfirstlane(jmax);
      if (jmax <= JM) {
        float wj[JM];
        int src[JM];
#pragma unroll
        for (int d = 0; d < JM; ++d) {
          const int jj = min(jlo + d, Wout - 1);
          const float4 e = coltab[max(jj, 0)];
          wj[d] = d < nj ? (__float_as_int(e.x) == ul ? e.z : e.w) : 0.0f;
          src[d] = max(jj, 0) * 4;
        }
        // rows in groups of RG (one uniform branch per group), the column
        // offset d outermost: the group's RG exchanges of one d are
        // independent and in flight together (per row the sum still runs
        // over d ascending)
        constexpr int RG = 8;
#pragma unroll
        for (int r0 = 0; r0 < GV; r0 += RG) {
          if (rlo + r0 >= rhi) break;
          float gt[RG], acc[RG];
#pragma unroll
          for (int r = 0; r < RG; ++r) {
            const float g0 = gv[r0 + r] * sc;
            gt[r] = grads && g0 != 0.0f ? g0 : 0.0f;
            acc[r] = 0.0f;
          }
#pragma unroll
          for (int d = 0; d < JM; ++d) {
            if (d >= jmax) break;
            float gj[RG];
#pragma unroll
            for (int r = 0; r < RG; ++r)
              gj[r] = __int_as_float(__builtin_amdgcn_ds_bpermute(src[d], __float_as_int(gt[r])));
#pragma unroll
            for (int r = 0; r < RG; ++r)
              if (d < nj) acc[r] += gj[r] * wj[d];
          }
#pragma unroll
          for (int r = 0; r < RG; ++r)
            if (uact && rlo + r0 + r < rhi) sT[(rlo + r0 + r) * Win + ul] = acc[r];
        }
        wave_sync();
        TS(3);
        goto du_pass;
      }
    }
    if (ul < Win) {
      constexpr int RMAX = 32;  // rows per lane (ceil(Hout / rpi) <= 32, see sdu)
      constexpr int RC = 16;    // rows per chunk (register budget: occupancy)
      const int rb = tlo + half;  // the lane's first row
      const int nr = rb < thi ? (thi - rb + rpi - 1) / rpi : 0;

#pragma unroll 1
      for (int r0 = 0; r0 < RMAX; r0 += RC) {
        if (r0 >= nr) break;
        float acc[RC];
        unsigned ylive = 0;  // bit r: the lane's row r0 + r has distinct corner rows
#pragma unroll
        for (int r = 0; r < RC; ++r) {
          acc[r] = 0.0f;
          const float4 e = rowtab[min(rb + rpi * (r0 + r), Hout - 1)];
          ylive |= (__float_as_int(e.x) != __float_as_int(e.y) ? 1u : 0u) << r;
        }
        for (int j = jlo; j <= jhi; ++j) {
          const float4 e = coltab[j];
          const float w = __float_as_int(e.x) == ul ? e.z : e.w;
#pragma unroll
          for (int r = 0; r < RC; ++r) {  // unpredicated (clamped row): loads stay in flight
            const float g0 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                                 gr, (min(rb + rpi * (r0 + r), Hout - 1) * Wout + j) * 4, 0, 0)) *
                             sc;
            const float g = ((ylive >> r) & 1u) && grads && g0 != 0.0f ? g0 : 0.0f;
            acc[r] += g * w;
          }
        }
#pragma unroll
        for (int r = 0; r < RC; ++r)
          if (r0 + r < nr) sT[(rb + rpi * (r0 + r)) * Win + ul] = acc[r];
      }
    }
    wave_sync();
    TS(3);
  du_pass:
    // the output sigmoid's r = U at the lane's dU outputs, all loaded up
    // front (the T pass overwrote the staged image): one memory latency
    // instead of one dependent round trip per output
    if (upre) {
#pragma unroll
      for (int k = 0; k < UV; ++k)
        uv[k] = Un[min(half + rpi * k, Hin - 1) * Win + min(ul, Win - 1)];
    }
    // dU[v][u] = sum_i T[i][u] * (y0(i) == v ? y1 - y : y - y0)
    if (upre) {
      if (ul < Win) {
        // outputs in groups of VG, the first IM rows of every range read
        // together (clamped, masked); longer ranges finish in a loop.  Per
        // output the sum runs over i ascending, as before.
        constexpr int VG = 4, IM = 4;
#pragma unroll
        for (int k0 = 0; k0 < UV; k0 += VG) {
          if (half + rpi * k0 >= Hin) break;
          int2 rr[VG];
#pragma unroll
          for (int q = 0; q < VG; ++q) rr[q] = vrange[min(half + rpi * (k0 + q), Hin - 1)];
          float tv[VG][IM], wv[VG][IM];
#pragma unroll
          for (int q = 0; q < VG; ++q) {
            const int v = half + rpi * (k0 + q);
#pragma unroll
            for (int j = 0; j < IM; ++j) {
              const int i = max(min(rr[q].x + j, rr[q].y), 0);
              const float4 e = rowtab[i];
              tv[q][j] = sT[i * Win + ul];
              wv[q][j] = __float_as_int(e.x) == v * Win ? e.z : e.w;
            }
          }
#pragma unroll
          for (int q = 0; q < VG; ++q) {
            const int k = k0 + q, v = half + rpi * k;
            if (v >= Hin) break;
            float acc = 0.0f;
#pragma unroll
            for (int j = 0; j < IM; ++j)
              if (rr[q].x + j <= rr[q].y) acc += tv[q][j] * wv[q][j];
            for (int i = rr[q].x + IM; i <= rr[q].y; ++i) {
              const float4 e = rowtab[i];
              acc += sT[i * Win + ul] * (__float_as_int(e.x) == v * Win ? e.z : e.w);
            }
            put_u(v * Win + ul, acc, uv[k]);
          }
        }
      }
    } else if (ul < Win)
      for (int v = half; v < Hin; v += rpi) {
        const int2 r = vrange[v];
        float acc = 0.0f;
        for (int i = r.x; i <= r.y; ++i) {
          const float4 e = rowtab[i];
          acc += sT[i * Win + ul] * (__float_as_int(e.x) == v * Win ? e.z : e.w);
        }
        put(v * Win + ul, acc);
      }
    TS(4);
    return;
  }
  if ((HWin & 3) == 0 && !du_mode) {
    for (int q = lane; q < HWin / 4; q += 64)
      reinterpret_cast<floatx4*>(dUn)[q] = reinterpret_cast<const floatx4*>(sD)[q];
  } else {
    for (int i = lane; i < HWin; i += 64) put(i, sD[i]);
  }
}

__global__ __launch_bounds__(256, 4) void stn_bwd_kernel(
    const float* __restrict__ U, int N, int Hin, int Win, const float* __restrict__ theta,
    int Hout, int Wout, const float* __restrict__ G, const float* __restrict__ gscale, float* dU,
    float* dtheta, float* dot, int u_period, int g_period, long long* ts, int du_mode) {
#pragma clang fp contract(off)
  // wave-uniform image index (readfirstlane): the cotangent's buffer
  // descriptor below is then provably uniform -- otherwise hipcc wraps every
  // buffer load of the T pass in a waterfall loop and serialises them
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = blockIdx.x * (blockDim.x >> 6) + wv;
  if (q >= N) return;  // no workgroup barriers below
  // rows sharing a periodic operand (AIR's T loop steps of one image: the
  // canvas cotangent of the write backward, the input canvas of the read
  // backward) run back to back on neighbouring waves, so the shared image is
  // read from HBM once and from L2 by the other steps; each row is still
  // computed by one wave alone, so the results do not change
  const int per = u_period > 0 ? u_period : g_period;
  const int nt = per > 0 && N % per == 0 ? N / per : 1;
  const int n = nt > 1 ? (q % nt) * per + q / nt : q;
  TS(0);
  const int HWin = Hin * Win;
  const bool want_dU = dU != nullptr;
  float th[6];  // wave-uniform (scalar registers): the branches below are uniform
#pragma unroll
  for (int k = 0; k < 6; ++k)
    th[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(theta[n * 6 + k])));
  const bool sep = stn_separable(th) && Hin < 32768 && Win < 32768 && Hout <= 64;
  // separable dU (no atomics): axis-aligned, increasing maps, extents <= 64
  const bool sdu = want_dU && sep && th[0] > 0.0f && th[4] > 0.0f && Hin <= 64 && Win <= 64 &&
                   Hout <= (Win <= 32 ? 64 : 32) && Wout <= 64;
  const int mode = (sep ? 1 : 0) | (sdu ? 2 : 0) | (want_dU ? 4 : 0);
  const bool regs = sep && Wout > 32 && Wout <= 64 && (HWin & 3) == 0 && HWin <= 1024 &&
                    (mode == 1 || mode == 3 || mode == 7);
  if (regs)
    stn_bwd_image<true>(U, Hin, Win, th, Hout, Wout, G, gscale, dU, dtheta, dot, u_period,
                        g_period, ts, du_mode, n, lane, wv, sep, sdu);
  else
    stn_bwd_image<false>(U, Hin, Win, th, Hout, Wout, G, gscale, dU, dtheta, dot, u_period,
                         g_period, ts, du_mode, n, lane, wv, sep, sdu);
}

}  // namespace

extern "C" int mog_stn_write_parts(const float* U, int N, int Hin, int Win, const float* theta,
                                   int Hout, int Wout, const float* z, const float* mask,
                                   float* parts, int* part_rows, void* stream) {
  MOG_CHECK_ARG(U && theta && z && mask && parts && part_rows && N >= 0);
  MOG_CHECK_ARG(Hin > 0 && Win > 0 && Hout > 0 && Wout > 0 && Hout < 65536);
  if (N == 0) return 0;
  stn_part_kernel<<<N, 256, 0, mog_stream(stream)>>>(U, Hin, Win, theta, Hout, Wout, parts,
                                                      part_rows, z, mask);
  MOG_LAUNCH_RET();
}

// transformer(U, theta, out_size) forward; see include/mog_air.h
extern "C" int mog_stn_forward_periodic(const float* U, int u_period, int N, int Hin, int Win,
                                        const float* theta, int Hout, int Wout, void* out,
                                        const float* z, const float* mask, int mode,
                                        void* stream) {
  MOG_CHECK_ARG(U && theta && out && N >= 0 && Hin > 0 && Win > 0 && Hout > 0 && Wout > 0);
  MOG_CHECK_ARG(mode >= 0 && mode <= 2 && (mode != 1 || (z && mask)) && u_period >= 0);
  if (N == 0) return 0;
  hipStream_t s = mog_stream(stream);
  if (mode == 1)
    stn_fwd_kernel<1><<<N, 256, 0, s>>>(U, Hin, Win, theta, Hout, Wout, out, z, mask, u_period);
  else if (mode == 2)
    stn_fwd_kernel<2><<<N, 256, 0, s>>>(U, Hin, Win, theta, Hout, Wout, out, nullptr, nullptr,
                                        u_period);
  else
    stn_fwd_kernel<0><<<N, 256, 0, s>>>(U, Hin, Win, theta, Hout, Wout, out, nullptr, nullptr,
                                        u_period);
  MOG_LAUNCH_RET();
}

extern "C" int mog_stn_forward(const float* U, int N, int Hin, int Win, const float* theta,
                               int Hout, int Wout, void* out, const float* z,
                               const float* mask, int mode, void* stream) {
  return mog_stn_forward_periodic(U, 0, N, Hin, Win, theta, Hout, Wout, out, z, mask, mode,
                                  stream);
}

static int stn_backward_launch(const float* U, int N, int Hin, int Win, const float* theta,
                               int Hout, int Wout, const float* G, const float* gscale, float* dU,
                               float* dtheta, float* dot, int u_period, int g_period, int du_mode,
                               void* stream) {
  MOG_CHECK_ARG(U && theta && G && N >= 0 && Hin > 0 && Win > 0 && Hout > 0 && Wout > 0);
  MOG_CHECK_ARG(u_period >= 0 && g_period >= 0);
  MOG_CHECK_ARG(Hin * Win <= 16384);
  if (N == 0) return 0;
  const size_t slice = (size_t)stn_bwd_slice(Hin, Win, Hout, Wout, dU != nullptr);
  int wpb = 4;  // waves (images) per workgroup, within 80 KiB of LDS
  while (wpb > 1 && slice * sizeof(float) * wpb > 80 * 1024) --wpb;
  MOG_CHECK_ARG(slice * sizeof(float) * wpb <= 160 * 1024);
  // MOG_STN_TIMING=1 (profiling build): per-wave phase durations to stderr
  static long long* tbuf = nullptr;
  static size_t tcap = 0;
  long long* ts = nullptr;
  if (mog_prof_env("MOG_STN_TIMING")) {
    if (tcap < (size_t)N * 8) {
      if (tbuf) (void)hipFree(tbuf);
      tcap = (size_t)N * 8;
      if (hipMalloc(&tbuf, tcap * sizeof(long long)) != hipSuccess) return MOG_ERR_INVALID;
    }
    (void)hipMemset(tbuf, 0, tcap * sizeof(long long));
    ts = tbuf;
  }
  stn_bwd_kernel<<<mog_cdiv(N, wpb), 64 * wpb, slice * sizeof(float) * wpb,
                   mog_stream(stream)>>>(U, N, Hin, Win, theta, Hout, Wout, G, gscale, dU, dtheta,
                                         dot, u_period, g_period, ts, du_mode);
  if (ts) {
    std::vector<long long> h((size_t)N * 8);
    (void)hipStreamSynchronize(mog_stream(stream));
    (void)hipMemcpy(h.data(), tbuf, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
    double acc[4] = {0, 0, 0, 0};
    int cnt[4] = {0, 0, 0, 0};
    long long t0 = h[0], t1 = 0;
    for (int b = 0; b < N; ++b) {
      for (int k = 0; k < 4; ++k)
        if (h[b * 8 + k + 1] && h[b * 8 + k]) {
          acc[k] += (double)(h[b * 8 + k + 1] - h[b * 8 + k]);
          ++cnt[k];
        }
      t0 = std::min(t0, h[b * 8]);
      for (int k = 0; k < 5; ++k) t1 = std::max(t1, h[b * 8 + k]);
    }
    fprintf(stderr, "stn_bwd wave phases (us): stage %.2f main %.2f Tpass %.2f dUpass %.2f | span %.2f\n",
            cnt[0] ? acc[0] / cnt[0] / 100 : 0.0, cnt[1] ? acc[1] / cnt[1] / 100 : 0.0,
            cnt[2] ? acc[2] / cnt[2] / 100 : 0.0, cnt[3] ? acc[3] / cnt[3] / 100 : 0.0,
            (t1 - t0) / 100.0);
  }
  MOG_LAUNCH_RET();
}

extern "C" int mog_stn_backward(const float* U, int N, int Hin, int Win, const float* theta,
                                int Hout, int Wout, const float* G, const float* gscale,
                                float* dU, float* dtheta, float* dot, int u_period, int g_period,
                                void* stream) {
  return stn_backward_launch(U, N, Hin, Win, theta, Hout, Wout, G, gscale, dU, dtheta, dot,
                             u_period, g_period, 0, stream);
}

extern "C" int mog_stn_backward_sigmoid_bf16(const float* U, int N, int Hin, int Win,
                                             const float* theta, int Hout, int Wout,
                                             const float* G, const float* gscale, void* dm,
                                             float* dtheta, float* dot, int u_period, int g_period,
                                             void* stream) {
  MOG_CHECK_ARG(dm != nullptr && u_period == 0);
  return stn_backward_launch(U, N, Hin, Win, theta, Hout, Wout, G, gscale,
                             reinterpret_cast<float*>(dm), dtheta, dot, u_period, g_period, 1,
                             stream);
}

extern "C" int mog_stn_backward_sigmoid_f32(const float* U, int N, int Hin, int Win,
                                            const float* theta, int Hout, int Wout,
                                            const float* G, const float* gscale, float* dm,
                                            float* dtheta, float* dot, int u_period, int g_period,
                                            void* stream) {
  MOG_CHECK_ARG(dm != nullptr && u_period == 0);
  return stn_backward_launch(U, N, Hin, Win, theta, Hout, Wout, G, gscale, dm, dtheta, dot,
                             u_period, g_period, 2, stream);
}
