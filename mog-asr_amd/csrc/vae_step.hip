// Fused per-object step: STN read -> glimpse VAE -> latent sample + KL ->
// STN write, one launch per loop step (air_model.py:500-588 + :718-736,
// vae.py:5-48, transformer.py:18-175).  This is the kernel SURVEY.md §8 D.3
// prices at 30,024 algorithmic HBM bytes per image-step.
//
// One workgroup = 8 waves = MB (32) images, two workgroups per CU (70.5 KB of
// LDS each), so one workgroup's gathers and stores overlap the other's MFMA
// phases.  Activations stay in LDS between the six dense layers (bf16, rows
// padded against bank conflicts), reusing one region: a layer whose output
// lands on its own input waits for the whole workgroup after its k loop.  The
// bf16 weights (W^T in MFMA B-fragment order: one 1-KiB contiguous wave load
// per fragment) stream from L2 straight into the MFMA B operand (four k-steps
// of register prefetch); the A operand is read from LDS with ds_read_b128.
// Activations the backward needs (glimpse, softplus outputs, mu/logvar/z, r)
// are flushed to HBM with 16-byte stores.  The output layer's tiles are
// transposed through LDS so that the bias + noise + sigmoid epilogue works on
// four consecutive pixels (one Philox quad of eps_x) and r leaves with 16-byte
// stores; the STN write then stages r back from L2 sixteen images at a time
// and stores this step's canvas contribution z * w (0 where inactive or where
// the sample is exactly +0, i.e. x0 == x1 && y0 == y1); mog_recon_loss sums
// the parts in step order, so the canvas is bit-identical to the running
// accumulation of air_model.py:665-675 and this kernel never waits on a
// canvas read.
//
// Precision: bf16 MFMA operands, fp32 accumulation and epilogues with
// hardware transcendentals (the bf16 configuration, BASELINE configs[1]).
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "philox.h"
#include "stn_geom.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int MB = 32;        // images per workgroup
constexpr int NW = 8;         // waves per workgroup
constexpr int NTHR = NW * 64;
constexpr int W2 = 784;       // 28 x 28 glimpse
constexpr int KG = 800;       // glimpse k extent padded to a multiple of 32 (25 k-steps)
constexpr int SG = KG + 8;    // LDS row strides (bf16), +16 B against bank conflicts
constexpr int S512 = 512 + 8, S256 = 256 + 8, SZ = 64 + 8;
// One LDS arena: region A [0, A_BYTES) then region H [A_BYTES, ARENA).
//   A: glimpse [32][808] -> a1 [32][520] -> mu | lv | kl fp32, z bf16 -> d2
//      [32][520] (+ the output layer's transpose scratch behind it)
//   H: read tables -> a2 [32][264] -> d1 [32][264]
//   A+H: r staging for 16 images [16][784] fp32 + their write tables
constexpr int A_BYTES = MB * SG * 2;                     // 51,712
constexpr int H_BYTES = MB * S256 * 2;                   // 16,896
constexpr int ARENA = A_BYTES + H_BYTES;                 // 68,608
constexpr int TABR = 28 + 28;                            // read tables: 28 columns + 28 rows
constexpr int OFF_MU = 0, OFF_LV = MB * 50 * 4, OFF_KL = 2 * MB * 50 * 4, OFF_Z = 3 * MB * 50 * 4;
constexpr int OFF_XP = MB * S512 * 2;                    // transpose scratch behind d2
constexpr int XP_STRIDE = 20;                            // floats per scratch row (conflict-free)
constexpr int XP_WAVE = 32 * XP_STRIDE * 4;              // 2,560 B per wave
constexpr int RH = 16;                                   // images per r-staging half
constexpr int OFF_TABW = RH * W2 * 4;                    // 50,176
constexpr int CTAB_MAX = 64;                             // write tables for canvases up to 64 x 64
static_assert(MB * TABR * 8 <= H_BYTES, "read tables");
static_assert(OFF_Z + MB * SZ * 2 <= A_BYTES, "mu/lv/kl/z");
static_assert(MB * S512 * 2 <= A_BYTES && MB * S256 * 2 <= H_BYTES, "activations");
static_assert(OFF_XP + NW * XP_WAVE <= ARENA, "transpose scratch");
static_assert(OFF_TABW + RH * 2 * CTAB_MAX * 8 <= ARENA, "write tables");

struct StepArgs {
  const float* x;            // [B, C*C] canvas input
  const float* theta_f;      // [B, 6]
  const float* theta_b;      // [B, 6]
  const float* mask;         // [B] active (new stopping sum < thr)
  const float* zval;         // [B] z_pres
  const float* eps_z;        // [B, Z]
  const float* eps_x;        // [B, 784] (read when eps_gen == 0)
  unsigned long long eps_seed, eps_offset;  // eps_gen: Philox quad (eps_offset + b*196 + k/4)
  int eps_gen;
  const __bf16* wt[7];       // W^T in B-fragment order: r1 [512][800], r2 [256][512],
                             // mu, lv [64][256], g1 [256][64], g2 [512][256], go [784][512]
  const float* bias[7];
  float* part;               // [B, C*C] this step's canvas contribution (written)
  float* runloss;            // [B]
  float* vkl;                // [B]
  __bf16* gb;                // [B, 784]   saved for the backward
  __bf16* a1b;               // [B, 512]
  __bf16* a2b;               // [B, 256]
  float* mu;                 // [B, 50]
  float* lv;                 // [B, 50]
  float* z;                  // [B, 50]
  __bf16* zb;                // [B, 56]
  __bf16* d1b;               // [B, 256]
  __bf16* d2b;               // [B, 512]
  float* r;                  // [B, 784]
  int B, C;
  float lik_std, v_pm, v_pv, v_plv;
  int phases;               // profiling aid: bit mask of the phases to run (all by default)
  long long* tstamp;        // profiling aid: per-block phase timestamps (or null)
};

// Workgroup barrier for LDS hand-offs only: unlike __syncthreads() it does not
// drain the wave's global stores (activation flushes, canvas parts), which stay
// in flight across phases.  The one global hand-off (r, go layer -> STN write)
// waits for its stores explicitly.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ float softplus_fast(float v) {
  return v > -MOG_SOFTPLUS_T ? v : (v < MOG_SOFTPLUS_T ? __expf(v) : __logf(__expf(v) + 1.0f));
}

// Axis tables of `nimg` images' transforms (th at sth[m0 + m][th_off]):
// tab[m*per + n], n < Wout columns then Hout rows, as {coordinate, lo | hi<<16}.
__device__ __forceinline__ void build_tables(float2* tab, const float (*sth)[12], int m0, int nimg,
                                             int th_off, int Hin, int Win, int Hout, int Wout) {
  const int per = Wout + Hout;
  for (int i = threadIdx.x; i < nimg * per; i += NTHR) {
    const int m = i / per, n = i - (i / per) * per;
    const float* th = &sth[m0 + m][th_off];
    tab[i] = n < Wout ? axis_col(th, Hin, Win, Hout, Wout, n)
                      : axis_row(th, Hin, Win, Hout, Wout, n - Wout);
  }
}

// Column tiles tile_base + (w + nw*c + rot) % (nw*TPW) of one dense layer
// over the MB rows held in LDS, for waves wbase .. wbase+nw-1.  A: LDS
// [MB][lda] bf16, zero-padded to K.  W: the layer's W^T in B-fragment order
// (mog_cvt_bf16_batch transpose 2; N padded to 16, K to 32, zeros outside),
// so each B fragment is one 1-KiB contiguous wave load streamed from L2
// straight into the MFMA, with a register prefetch ring of D k-steps (rolled,
// branch-free body so the compiler keeps the distance; the ragged tail is
// peeled at compile time).  SYNC: the whole workgroup meets after the k loop
// (the epilogue overwrites A; requires nw == NW).  epi(ct, acc[2][4] per tile).
template <int K, int TPW, bool SYNC, class Epi>
__device__ __forceinline__ void dense_tiles(const __bf16* A, int lda, const __bf16* __restrict__ W,
                                            int tile_base, int wbase, int nw, Epi epi) {
  constexpr int KS = K / 32;
  static_assert(K % 32 == 0, "K padding");
  const int rot = (int)(blockIdx.x >> 3);  // spread the CUs of one XCD over the weight columns
  const int lane = threadIdx.x & 63, w = (threadIdx.x >> 6) - wbase;
  const bool on = w >= 0 && w < nw;
  const int li = lane & 15, g = lane >> 4;
  int ct[TPW];
  const bf16x8* wf[TPW];
#pragma unroll
  for (int c = 0; c < TPW; ++c) {
    ct[c] = tile_base + (w + nw * c + rot) % (nw * TPW);
    wf[c] = reinterpret_cast<const bf16x8*>(W) + (size_t)ct[c] * KS * 64 + lane;
  }
  floatx4 acc[2][TPW];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int c = 0; c < TPW; ++c) acc[rt][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto loadB = [&](int ks, bf16x8* b) {
#pragma unroll
    for (int c = 0; c < TPW; ++c) b[c] = wf[c][ks * 64];
  };
  auto step = [&](int ks, const bf16x8* b) {
    const int k = ks * 32 + 8 * g;
    const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&A[li * lda + k]);
    const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&A[(16 + li) * lda + k]);
#pragma unroll
    for (int c = 0; c < TPW; ++c) {
      acc[0][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b[c], acc[0][c], 0, 0, 0);
      acc[1][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b[c], acc[1][c], 0, 0, 0);
    }
  };
  // ring depth: four k-steps of B fragments in flight, two for four-tile waves
  // (register budget of two workgroups per CU)
  constexpr int D = TPW >= 4 ? 2 : 4;
  if (on) {
    if constexpr (KS < D) {
      bf16x8 q[TPW];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        loadB(ks, q);
        step(ks, q);
      }
    } else {
      constexpr int NI = (KS - D) / D;   // ring iterations with D refills each
      constexpr int K0 = D * NI;         // first k-step of the peeled tail
      bf16x8 q[D][TPW];
#pragma unroll
      for (int d = 0; d < D; ++d) loadB(d, q[d]);
#pragma unroll 1
      for (int ks = 0; ks < K0; ks += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
          step(ks + d, q[d]);
          loadB(ks + d + D, q[d]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int d = 0; d < D; ++d) {
        step(K0 + d, q[d]);
        if (K0 + d + D < KS) loadB(K0 + d + D, q[d]);
      }
#pragma unroll
      for (int d = 0; d < D; ++d)
        if (K0 + D + d < KS) step(K0 + D + d, q[d]);
    }
  }
  if constexpr (SYNC) lds_barrier();
  if (!on) return;
#pragma unroll
  for (int c = 0; c < TPW; ++c) {
    floatx4 a[2] = {acc[0][c], acc[1][c]};
    epi(ct[c], a);
  }
}

// element-wise epilogue into an LDS tile: out[row][col] = f(acc, col) for the
// lane's 8 accumulators of column tile ct (rows rt*16 + g*4 + r, col ct*16 + li)
template <class F>
__device__ __forceinline__ void epi_rows(int ct, const floatx4* a, int N, F f) {
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  const int col = ct * 16 + li;
  if (col >= N) return;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) f(rt * 16 + g * 4 + r, col, a[rt][r]);
}

// LDS tile [nb][lds] -> HBM rows [nb][ldg] with 16-byte stores (ncols * sizeof(T) % 16 == 0).
template <class T>
__device__ __forceinline__ void flush_rows(const T* s, int lds, T* g, int ldg, int ncols, int nb) {
  constexpr int V = 16 / sizeof(T);
  const int cpr = ncols / V;
  for (int i = threadIdx.x; i < nb * cpr; i += NTHR) {
    const int m = i / cpr, c = i - (i / cpr) * cpr;
    *reinterpret_cast<u32x4*>(g + (size_t)m * ldg + c * V) =
        *reinterpret_cast<const u32x4*>(s + m * lds + c * V);
  }
}

#define STAMP(k) \
  if (p.tstamp && threadIdx.x == 0) p.tstamp[blockIdx.x * 16 + (k)] = wall_clock64()

__global__ __launch_bounds__(NTHR, 4) void stn_vae_step_bf16_kernel(StepArgs p) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) unsigned char arena[ARENA];
  __shared__ float sth[MB][12];
  __shared__ float szv[MB];
  __shared__ int smask[MB];
  __shared__ int ssep[MB];  // bit 0: theta_f axis-aligned, bit 1: theta_b (and tables fit)
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int b0 = blockIdx.x * MB;
  const int nb = min(MB, p.B - b0);
  const int C = p.C, C2 = C * C;
  unsigned char* sA = arena;
  unsigned char* sHb = arena + A_BYTES;
  __bf16* sG = reinterpret_cast<__bf16*>(sA);
  __bf16* sA1 = reinterpret_cast<__bf16*>(sA);
  __bf16* sD2 = reinterpret_cast<__bf16*>(sA);
  float* sMu = reinterpret_cast<float*>(sA + OFF_MU);
  float* sLv = reinterpret_cast<float*>(sA + OFF_LV);
  float* sKl = reinterpret_cast<float*>(sA + OFF_KL);
  __bf16* sZ = reinterpret_cast<__bf16*>(sA + OFF_Z);
  float2* tabR = reinterpret_cast<float2*>(sHb);
  __bf16* sA2 = reinterpret_cast<__bf16*>(sHb);
  __bf16* sD1 = reinterpret_cast<__bf16*>(sHb);
  float* sR = reinterpret_cast<float*>(arena);
  float2* tabW = reinterpret_cast<float2*>(arena + OFF_TABW);
  STAMP(11);

  for (int i = tid; i < MB * 12; i += NTHR) {
    const int m = i / 12, k = i % 12;
    float v = 0.0f;
    if (m < nb) v = k < 6 ? p.theta_f[(size_t)(b0 + m) * 6 + k] : p.theta_b[(size_t)(b0 + m) * 6 + k - 6];
    sth[m][k] = v;
  }
  if (tid < MB) {
    const bool act = tid < nb && p.mask[b0 + tid] != 0.0f;
    smask[tid] = act;
    szv[tid] = act ? p.zval[b0 + tid] : 0.0f;
  }
  lds_barrier();
  bool sep_f = true;
  if (tid < MB) {
    sep_f = stn_separable(&sth[tid][0]);
    ssep[tid] = (sep_f ? 1 : 0) | (stn_separable(&sth[tid][6]) && C <= CTAB_MAX ? 2 : 0);
  }
  build_tables(tabR, sth, 0, MB, 0, C, C, 28, 28);
  const bool all_sep = __syncthreads_and(sep_f) != 0;  // (no global stores issued yet)
  STAMP(0);

  // ---- 1. STN read (transformer.py:18-175): glimpse -> LDS bf16 ---------
  // Half-wave per glimpse row (lane = column).  Axis-aligned transforms (every
  // AIR theta): 14 rows per pass, 56 gathers per lane in flight, the bilinear
  // weights re-read from the LDS axis tables once the gathers have landed
  // (only the gathered values are live across the wait).  General affine
  // transforms: eight rows per pass with per-sample geometry.
  if ((p.phases & 1) && all_sep) {
    // half-wave hw owns images 2hw and 2hw+1 (its row entries are broadcast
    // LDS reads, the column pair per lane is fixed per image); 14 rows per
    // pass, gathers through a buffer descriptor over this block's images
    // (32-bit offsets).
    static_assert(MB == 32 && NTHR == 512, "two images per half-wave");
    const int hw = tid >> 5, j = tid & 31, jc = min(j, 27);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.x) + (size_t)b0 * C2, 0, nb * C2 * 4, 0x00020000);
    const int C4 = C * 4;
#pragma unroll 1
    for (int h = 0; h < 4; ++h) {
      const int m = 2 * hw + (h >> 1), i0 = (h & 1) * 14;
      const int mc = m < nb ? m : 0;
      const float2* tr = tabR + mc * TABR;
      const float2 cx = tr[jc];
      const int xo = mc * C2 * 4;
      const int xa = xo + axis_lo(cx) * 4, xb = xo + axis_hi(cx) * 4;
      float I[14][4];
#pragma unroll
      for (int u = 0; u < 14; ++u) {
        const float2 cy = tr[28 + i0 + u];
        const int ya = __mul24(axis_lo(cy), C4), yb = __mul24(axis_hi(cy), C4);
        I[u][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, xa + ya, 0, 0));
        I[u][1] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, xa + yb, 0, 0));
        I[u][2] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, xb + ya, 0, 0));
        I[u][3] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, xb + yb, 0, 0));
      }
      asm volatile("" ::: "memory");  // re-read the tables below instead of keeping them live
      const float2 cx2 = tr[jc];
      const float4 ex = axis4(cx2, 1);
      const bool xlive = m < nb && axis_lo(cx2) != axis_hi(cx2);
      // branch-free: every lane samples; lanes 28..31 store into the unused
      // row padding [800, 804) (beyond the GEMM's k extent)
      __bf16* dst = sG + m * SG + (j < 28 ? i0 * 28 + j : KG + j - 28);
      const int ustep = j < 28 ? 28 : 0;
#pragma unroll
      for (int u = 0; u < 14; ++u) {
        const float2 cy = tr[28 + i0 + u];
        const float4 ey = axis4(cy, C);
        const bool live = xlive || (m < nb && axis_lo(cy) != axis_hi(cy));  // not both axes dead
        const float sv = sample4(ex, ey, I[u][0], I[u][1], I[u][2], I[u][3]);
        dst[u * ustep] = (__bf16)(live ? sv : 0.0f);
      }
    }
    for (int i = tid; i < MB * (KG - W2); i += NTHR) {  // zero k padding
      const int m = i / (KG - W2);
      sG[m * SG + W2 + (i - m * (KG - W2))] = (__bf16)0.0f;
    }
  } else if (p.phases & 1) {
    constexpr int UR = 8;
    const int hw = tid >> 5, j = tid & 31;
    for (int rr0 = hw; rr0 < MB * 28; rr0 += 16 * UR) {
      float I[UR][4];
      float4 ex[UR], ey[UR];
      bool live[UR];
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const int rr = rr0 + 16 * u;
        const int m = rr / 28, i = rr - (rr / 28) * 28;
        live[u] = rr < MB * 28 && m < nb && j < 28;
        const int mc = live[u] ? m : 0, jc = min(j, 27);
        const float* U = p.x + (size_t)(b0 + mc) * C2;
        if (ssep[mc] & 1) {
          ex[u] = axis4(tabR[mc * TABR + jc], 1);
          ey[u] = axis4(tabR[mc * TABR + 28 + i], C);
        } else {  // general affine transform: per-sample geometry
          const Tap t = stn_tap(sth[mc], C, C, mog_linspace(jc, 28), mog_linspace(i, 28));
          ex[u] = make_float4(__int_as_float((int)t.x0f), __int_as_float((int)t.x1f),
                              t.x1f - t.x, t.x - t.x0f);
          ey[u] = make_float4(__int_as_float((int)t.y0f * C), __int_as_float((int)t.y1f * C),
                              t.y1f - t.y, t.y - t.y0f);
        }
        live[u] = live[u] && !axis4_dead(ex[u], ey[u]);
        const int x0 = __float_as_int(ex[u].x), x1 = __float_as_int(ex[u].y);
        const int y0 = __float_as_int(ey[u].x), y1 = __float_as_int(ey[u].y);
        // unpredicated (all indices are valid clipped corners of a real
        // image) so the waitcnt pass keeps the 32 gathers in flight
        I[u][0] = U[y0 + x0];
        I[u][1] = U[y1 + x0];
        I[u][2] = U[y0 + x1];
        I[u][3] = U[y1 + x1];
      }
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const int rr = rr0 + 16 * u;
        if (rr >= MB * 28 || j >= 28) continue;
        const int m = rr / 28, i = rr - (rr / 28) * 28;
        const float v = live[u] ? sample4(ex[u], ey[u], I[u][0], I[u][1], I[u][2], I[u][3]) : 0.0f;
        sG[m * SG + i * 28 + j] = (__bf16)v;
      }
    }
    for (int i = tid; i < MB * (KG - W2); i += NTHR) {  // zero k padding
      const int m = i / (KG - W2);
      sG[m * SG + W2 + (i - m * (KG - W2))] = (__bf16)0.0f;
    }
  }
  lds_barrier();
  STAMP(1);
  if (p.phases & 16) flush_rows(sG, SG, p.gb + (size_t)b0 * W2, W2, W2, nb);

  // ---- 2. a1 = softplus(g W1 + b1)  [MB x 512], over the glimpse ----------
  if (p.phases & 2) {
    const float* bias = p.bias[0];
    dense_tiles<KG, 4, true>(sG, SG, p.wt[0], 0, 0, NW, [&](int ct, const floatx4* a) {
      epi_rows(ct, a, 512, [&](int m, int n, float v) {
        sA1[m * S512 + n] = (__bf16)softplus_fast(v + bias[n]);
      });
    });
  }
  lds_barrier();
  STAMP(2);
  if (p.phases & 16) flush_rows(sA1, S512, p.a1b + (size_t)b0 * 512, 512, 512, nb);
  // ---- 3. a2 = softplus(a1 W2 + b2)  [MB x 256] -> H ----------------------
  if (p.phases & 2) {
    const float* bias = p.bias[1];
    dense_tiles<512, 2, false>(sA1, S512, p.wt[1], 0, 0, NW, [&](int ct, const floatx4* a) {
      epi_rows(ct, a, 256, [&](int m, int n, float v) {
        sA2[m * S256 + n] = (__bf16)softplus_fast(v + bias[n]);
      });
    });
  }
  lds_barrier();
  STAMP(3);
  if (p.phases & 16) flush_rows(sA2, S256, p.a2b + (size_t)b0 * 256, 256, 256, nb);
  // ---- 4. mu | lv = a2 W + b  [MB x 50] fp32 -> A (waves 0-3 | 4-7) ------
  if (p.phases & 2) {
    const float* bm = p.bias[2];
    dense_tiles<256, 1, false>(sA2, S256, p.wt[2], 0, 0, 4, [&](int ct, const floatx4* a) {
      epi_rows(ct, a, 50, [&](int m, int n, float v) { sMu[m * 50 + n] = v + bm[n]; });
    });
    const float* bl = p.bias[3];
    dense_tiles<256, 1, false>(sA2, S256, p.wt[3], 0, 4, 4, [&](int ct, const floatx4* a) {
      epi_rows(ct, a, 50, [&](int m, int n, float v) { sLv[m * 50 + n] = v + bl[n]; });
    });
  }
  lds_barrier();
  STAMP(4);
  // ---- 5. z = mu + eps sqrt(exp(lv)); VAE KL -> runloss (vae.py:27-30) ---
  for (int i = tid; i < MB * 64; i += NTHR) {
    const int m = i >> 6, k = i & 63;
    float zv = 0.0f;
    if (k < 50 && m < nb) {
      const size_t o = (size_t)(b0 + m) * 50 + k;
      const float l = sLv[m * 50 + k];
      const float mv = sMu[m * 50 + k];
      const float var = mog_expf(l);
      zv = mv + p.eps_z[o] * sqrtf(var);
      p.mu[o] = mv;
      p.lv[o] = l;
      p.z[o] = zv;
      p.zb[(size_t)(b0 + m) * 56 + k] = (__bf16)zv;
      const float d = mv - p.v_pm;
      sKl[m * 50 + k] = (((p.v_plv - l) - 1.0f) + var / p.v_pv) + (d * d) / p.v_pv;
    }
    sZ[m * SZ + k] = (__bf16)zv;
  }
  lds_barrier();
  if (tid < nb) {  // sequential KL sum per image (k order, as vae_sample_fwd_kernel)
    const int m = tid;
    float t[50];
#pragma unroll
    for (int k = 0; k < 50; ++k) t[k] = sKl[m * 50 + k];
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < 50; ++k) sum = sum + t[k];
    const float vkl = 0.5f * sum;
    p.vkl[b0 + m] = vkl;
    if (smask[m]) p.runloss[b0 + m] = p.runloss[b0 + m] + vkl;
  }
  STAMP(5);
  // ---- 6. d1 = softplus(z Wg1 + b)  [MB x 256] -> H -----------------------
  if (p.phases & 2) {
    const float* bias = p.bias[4];
    dense_tiles<64, 2, false>(sZ, SZ, p.wt[4], 0, 0, NW, [&](int ct, const floatx4* a) {
      epi_rows(ct, a, 256, [&](int m, int n, float v) {
        sD1[m * S256 + n] = (__bf16)softplus_fast(v + bias[n]);
      });
    });
  }
  lds_barrier();
  STAMP(6);
  if (p.phases & 16) flush_rows(sD1, S256, p.d1b + (size_t)b0 * 256, 256, 256, nb);
  // ---- 7. d2 = softplus(d1 Wg2 + b)  [MB x 512] -> A ----------------------
  if (p.phases & 2) {
    const float* bias = p.bias[5];
    dense_tiles<256, 4, false>(sD1, S256, p.wt[5], 0, 0, NW, [&](int ct, const floatx4* a) {
      epi_rows(ct, a, 512, [&](int m, int n, float v) {
        sD2[m * S512 + n] = (__bf16)softplus_fast(v + bias[n]);
      });
    });
  }
  lds_barrier();
  STAMP(7);
  if (p.phases & 16) flush_rows(sD2, S512, p.d2b + (size_t)b0 * 512, 512, 512, nb);
  // ---- 8. r = sigmoid(d2 Wgo + b + std eps)  [MB x 784] fp32 -> HBM -------
  // Each 32 x 16 accumulator tile goes through the wave's LDS scratch so that
  // a lane owns four consecutive pixels of one row: one Philox quad of eps_x
  // (generated in-kernel exactly as mog_rng_fill would, or loaded), one
  // 16-byte store of r.  49 column tiles: 32 (4 per wave) + 16 (2) + 1 (wave 0).
  if (p.phases & 2) {
    const float* bias = p.bias[6];
    const float sd = p.lik_std;
    float* xp = reinterpret_cast<float*>(arena + OFF_XP + wv * XP_WAVE);
    auto epi = [&](int ct, const floatx4* a) {
      const int li = lane & 15, g = lane >> 4;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) xp[(rt * 16 + g * 4 + r) * XP_STRIDE + li] = a[rt][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int cq = lane & 3, n = ct * 16 + 4 * cq;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int m = h * 16 + (lane >> 2);
        const float4 v = *reinterpret_cast<const float4*>(&xp[m * XP_STRIDE + 4 * cq]);
        if (m < nb && n < W2) {
          float e[4];
          const size_t q = (size_t)(b0 + m) * (W2 / 4) + (n >> 2);
          if (p.eps_gen) {
            mog_philox_quad(p.eps_seed, p.eps_offset + q, true, e);
          } else {
            const float4 e4 = reinterpret_cast<const float4*>(p.eps_x)[q];
            e[0] = e4.x; e[1] = e4.y; e[2] = e4.z; e[3] = e4.w;
          }
          const float vv[4] = {v.x, v.y, v.z, v.w};
          float o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float y = __builtin_fmaf(e[k], sd, vv[k] + bias[n + k]);
            o[k] = 1.0f / (1.0f + __expf(-y));
          }
          reinterpret_cast<float4*>(p.r)[q] = make_float4(o[0], o[1], o[2], o[3]);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // scratch reads before the next tile
    };
    dense_tiles<512, 4, false>(sD2, S512, p.wt[6], 0, 0, NW, epi);
    dense_tiles<512, 2, false>(sD2, S512, p.wt[6], 32, 0, NW, epi);
    dense_tiles<512, 1, false>(sD2, S512, p.wt[6], 48, 0, 1, epi);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // r stores done before other waves read it
  lds_barrier();
  STAMP(8);
  STAMP(9);
  // ---- 9. STN write (air_model.py:580-588): this step's canvas part -------
  // part = active ? z * w : 0 for every pixel (write-only; mog_recon_loss sums
  // the parts in step order).  r is staged back from L2 sixteen images at a
  // time; one wave per image; each lane produces four consecutive canvas
  // pixels (flat order) and stores them with one 16-byte store.  Dead samples
  // (clipped corners coincide on both axes) are exactly +0 and are selected,
  // not branched.
  if (p.phases & 8) {
    const bool vec = (C2 & 3) == 0;  // even C: 16-byte aligned image rows of parts
    for (int h0 = 0; h0 < nb; h0 += RH) {
      const int nh = min(RH, nb - h0);
      {
        const float4* src = reinterpret_cast<const float4*>(p.r + (size_t)(b0 + h0) * W2);
        float4* dst = reinterpret_cast<float4*>(sR);
        for (int i = tid; i < nh * (W2 / 4); i += NTHR) dst[i] = src[i];
      }
      if (C <= CTAB_MAX) build_tables(tabW, sth, h0, nh, 6, 28, 28, C, C);
      lds_barrier();
      for (int mm = wv; mm < nh; mm += NW) {
        const int m = h0 + mm;
        float* om = p.part + (size_t)(b0 + m) * C2;
        float4* om4 = reinterpret_cast<float4*>(om);
        const float* U = sR + mm * W2;
        const bool act = smask[m] != 0, tab = (ssep[m] & 2) != 0;
        const float zn = szv[m];
        const float2* tcol = tabW + mm * 2 * C;
        const float2* trow = tcol + C;
        if (!act) {  // inactive: the whole part is +0
          const int nq = vec ? C2 / 4 : C2;
          for (int q = lane; q < nq; q += 64) {
            if (vec) om4[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            else om[q] = 0.0f;
          }
        } else if (tab && vec && C <= 128) {
          // Two-row bands of C/2 16-byte quads: a lane keeps the same four
          // columns (its x entries stay in registers) across every band and
          // reads only the two row entries per band.
          const int QB = C >> 1, NBW = 64 / QB;
          const bool ln = lane < NBW * QB;
          const int k = ln ? lane % QB : 0, bs = lane / QB;
          float4 ex[4];
          bool br[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int pp = 4 * k + e;
            br[e] = pp >= C;
            ex[e] = axis4(tcol[br[e] ? pp - C : pp], 1);
          }
          for (int bb = 0; bb < QB; bb += NBW) {
            const int b = bb + bs;
            const bool on = ln && b < QB;
            const float4 ey0 = axis4(trow[on ? 2 * b : 0], 28), ey1 = axis4(trow[on ? 2 * b + 1 : 0], 28);
            // A row whose clipped corner rows coincide samples exactly +0 at
            // every column (the y weights are exact negatives on one source
            // row, so the four products cancel pairwise in summation order):
            // bands where the whole wave sees only such rows store zeros.
            const bool rows_live = on && (__float_as_int(ey0.x) != __float_as_int(ey0.y) ||
                                          __float_as_int(ey1.x) != __float_as_int(ey1.y));
            if (__builtin_amdgcn_ballot_w64(rows_live) == 0) {
              if (on) om4[b * QB + k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
              continue;
            }
            if (!on) continue;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float4 ey = br[e] ? ey1 : ey0;
              const int x0 = __float_as_int(ex[e].x), x1 = __float_as_int(ex[e].y);
              const int y0 = __float_as_int(ey.x), y1 = __float_as_int(ey.y);
              const float sv = zn * sample4(ex[e], ey, U[y0 + x0], U[y1 + x0], U[y0 + x1],
                                            U[y1 + x1]);
              v[e] = axis4_dead(ex[e], ey) ? 0.0f : sv;
            }
            om4[b * QB + k] = make_float4(v[0], v[1], v[2], v[3]);
          }
        } else {  // general transform or odd C: per-pixel geometry, flat order
          const int nq = vec ? C2 / 4 : C2;
          const int per = vec ? 4 : 1;
          for (int q = lane; q < nq; q += 64) {
            float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            int pix = q * per;
            int i = pix / C, j = pix - (pix / C) * C;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              if (e < per) {
                const Tap t = stn_tap(&sth[m][6], 28, 28, mog_linspace(j, C), mog_linspace(i, C));
                v[e] = t.dead ? 0.0f : zn * tap_value(t, U);
                if (++j == C) { j = 0; ++i; }
              }
            }
            if (vec) om4[q] = make_float4(v[0], v[1], v[2], v[3]);
            else om[q] = v[0];
          }
        }
      }
      lds_barrier();
    }
  }
  if (p.tstamp) {
    lds_barrier();
    STAMP(10);
  }
}

}  // namespace

extern "C" int mog_stn_vae_step_forward(int B, int C, int W, int R1, int R2, int Z, int G1,
                                        int G2, const float* x, const float* theta_f,
                                        const float* theta_b, const float* mask,
                                        const float* zval, const float* eps_z,
                                        const float* eps_x, int eps_gen,
                                        unsigned long long eps_seed,
                                        unsigned long long eps_offset, const void* const* wt,
                                        const float* const* bias, float lik_std, float v_pm,
                                        float v_pv, float v_plv, float* canvas_part,
                                        float* runloss, float* vkl, void* gb, void* a1b,
                                        void* a2b, float* mu, float* lv, float* z, void* zb,
                                        void* d1b, void* d2b, float* r, void* stream) {
  MOG_CHECK_ARG(B >= 0 && C > 0 && C * C <= 16384);
  // the tile shapes are compiled for the reference's default VAE
  MOG_CHECK_ARG(W == 28 && R1 == 512 && R2 == 256 && Z == 50 && G1 == 256 && G2 == 512);
  MOG_CHECK_ARG(x && theta_f && theta_b && mask && zval && eps_z && (eps_x || eps_gen) && wt && bias);
  MOG_CHECK_ARG(canvas_part && runloss && vkl && gb && a1b && a2b && mu && lv && z && zb);
  MOG_CHECK_ARG(d1b && d2b && r);
  if (B == 0) return 0;
  StepArgs p;
  p.x = x; p.theta_f = theta_f; p.theta_b = theta_b; p.mask = mask; p.zval = zval;
  p.eps_z = eps_z; p.eps_x = eps_x;
  p.eps_gen = eps_gen; p.eps_seed = eps_seed; p.eps_offset = eps_offset;
  for (int i = 0; i < 7; ++i) {
    MOG_CHECK_ARG(wt[i] && bias[i]);
    p.wt[i] = reinterpret_cast<const __bf16*>(wt[i]);
    p.bias[i] = bias[i];
  }
  p.part = canvas_part; p.runloss = runloss; p.vkl = vkl;
  p.gb = reinterpret_cast<__bf16*>(gb); p.a1b = reinterpret_cast<__bf16*>(a1b);
  p.a2b = reinterpret_cast<__bf16*>(a2b); p.mu = mu; p.lv = lv; p.z = z;
  p.zb = reinterpret_cast<__bf16*>(zb); p.d1b = reinterpret_cast<__bf16*>(d1b);
  p.d2b = reinterpret_cast<__bf16*>(d2b); p.r = r;
  const char* ph = getenv("MOG_VS_PHASES");
  p.phases = ph ? atoi(ph) : 31;
  p.B = B; p.C = C; p.lik_std = lik_std; p.v_pm = v_pm; p.v_pv = v_pv; p.v_plv = v_plv;
  // MOG_VS_TIMING=1 (profiling aid): per-phase durations, averaged over
  // blocks, printed to stderr (synchronizes the stream)
  static long long* tbuf = nullptr;
  static size_t tcap = 0;
  const unsigned nblk = mog_cdiv(B, MB);
  p.tstamp = nullptr;
  if (getenv("MOG_VS_TIMING")) {
    if (tcap < (size_t)nblk * 16) {
      if (tbuf) (void)hipFree(tbuf);
      tcap = (size_t)nblk * 16;
      if (hipMalloc(&tbuf, tcap * sizeof(long long)) != hipSuccess) return MOG_ERR_INVALID;
    }
    p.tstamp = tbuf;
  }
  stn_vae_step_bf16_kernel<<<nblk, NTHR, 0, mog_stream(stream)>>>(p);
  if (p.tstamp) {
    std::vector<long long> h((size_t)nblk * 16);
    (void)hipStreamSynchronize(mog_stream(stream));
    (void)hipMemcpy(h.data(), tbuf, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
    static const char* names[10] = {"stn_read", "L1", "L2", "mu_lv", "sample",
                                    "g1", "g2", "go", "-", "write"};
    double acc[11] = {0}, pro = 0;
    long long t0 = h[0], t1 = h[10];
    for (unsigned b = 0; b < nblk; ++b) {
      for (int k = 0; k < 10; ++k) acc[k] += (double)(h[b * 16 + k + 1] - h[b * 16 + k]);
      acc[10] += (double)(h[b * 16 + 10] - h[b * 16]);
      pro += (double)(h[b * 16] - h[b * 16 + 11]);
      t0 = std::min(t0, h[b * 16]);
      t1 = std::max(t1, h[b * 16 + 10]);
    }
    fprintf(stderr, "stn_vae_step phases (us, mean over %u blocks; 100 MHz clock): prologue %.2f",
            nblk, pro / nblk / 100.0);
    for (int k = 0; k < 10; ++k) fprintf(stderr, " %s %.2f", names[k], acc[k] / nblk / 100.0);
    fprintf(stderr, " | block %.2f | span %.2f\n", acc[10] / nblk / 100.0, (t1 - t0) / 100.0);
  }
  MOG_LAUNCH_RET();
}
