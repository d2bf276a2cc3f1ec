// Fused per-object step: STN read -> glimpse VAE -> latent sample + KL ->
// STN write, one launch per loop step (air_model.py:500-588 + :718-736,
// vae.py:5-48, transformer.py:18-175).  This is the kernel SURVEY.md §8 D.3
// prices at 30,024 algorithmic HBM bytes per image-step.
//
// One workgroup = 8 waves = MB (32) images.  Activations stay in LDS between
// the six dense layers (bf16, rows padded against bank conflicts); the packed
// bf16 weights (W^T in MFMA B-fragment order: one 1-KiB contiguous load per
// fragment) stream from L2 straight into the MFMA B operand (four k-steps of
// register prefetch); the A operand is
// read from LDS with ds_read_b128.  Activations the backward needs (glimpse,
// softplus outputs, mu/logvar/z, r) are flushed to HBM with 16-byte stores.
// The STN write samples r from LDS (fp32) and stores this step's canvas
// contribution z * w (0 where inactive or where the sample is exactly +0,
// i.e. x0 == x1 && y0 == y1); mog_recon_loss sums the parts in step order, so
// the canvas is bit-identical to the running accumulation of
// air_model.py:665-675 and this kernel never waits on a canvas read.
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
// LDS region A (bytes): glimpse tile + read tables, then a2 | mu | lv | kl | z | d1,
// then r (fp32).  Region H: a1, then d2, then the write tables.
constexpr int REGION_A = MB * W2 * 4;
constexpr int OFF_TABR = MB * SG * 2;
constexpr int TABR = 28 + 28;                 // read tables: 28 columns + 28 rows per image
constexpr int OFF_MU = MB * S256 * 2;
constexpr int OFF_LV = OFF_MU + MB * 50 * 4;
constexpr int OFF_KL = OFF_LV + MB * 50 * 4;
constexpr int OFF_Z = OFF_KL + MB * 50 * 4;
constexpr int OFF_D1 = OFF_Z + MB * SZ * 2;
constexpr int CTAB_MAX = 52;                  // write tables for canvases up to 52 x 52
constexpr int REGION_H = MB * 2 * CTAB_MAX * 16;
static_assert(OFF_TABR + MB * TABR * 16 <= REGION_A, "read tables");
static_assert(OFF_D1 + MB * S256 * 2 <= REGION_A, "LDS layout");
static_assert(MB * S512 * 2 <= REGION_H, "region H");

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

__device__ __forceinline__ float softplus_fast(float v) {
  return v > -MOG_SOFTPLUS_T ? v : (v < MOG_SOFTPLUS_T ? __expf(v) : __logf(__expf(v) + 1.0f));
}

// Expanded axis tables of every image's transform (th at sth[m][th_off]):
// tab[m][0..Wout) columns, tab[m][Wout..Wout+Hout) rows (row entries carry
// the source pitch Win).  Only read for axis-aligned transforms.
__device__ __forceinline__ void build_tables(float4* tab, int stride, const float (*sth)[12],
                                             int th_off, int Hin, int Win, int Hout, int Wout) {
  const int per = Wout + Hout;
  for (int i = threadIdx.x; i < MB * per; i += NTHR) {
    const int m = i / per, n = i - (i / per) * per;
    const float* th = &sth[m][th_off];
    tab[m * stride + n] = n < Wout ? axis4(axis_col(th, Hin, Win, Hout, Wout, n), 1)
                                   : axis4(axis_row(th, Hin, Win, Hout, Wout, n - Wout), Win);
  }
}

// Column tiles tile_base + (w + nw*c + rot) % (nw*TPW) of one dense layer
// over the MB rows held in LDS, for waves wbase .. wbase+nw-1:
// epi(row, col, acc, aux).  A: LDS [MB][lda] bf16, zero-padded to K.  W: the
// layer's W^T in B-fragment order (mog_cvt_bf16_batch transpose 2; N padded
// to 16, K to 32, zeros outside), so each B fragment is one 1-KiB contiguous
// wave load streamed from L2 straight into the MFMA, with a four-k-step
// register prefetch ring (rolled, branch-free body so the compiler keeps the
// distance; the ragged tail is peeled at compile time).  With AUX the
// epilogue operand aux[row][col] is loaded before the k loop.
template <int N, int K, int TPW, bool AUX, class Epi>
__device__ __forceinline__ void dense_tiles(const __bf16* A, int lda, const __bf16* __restrict__ W,
                                            int tile_base, int wbase, int nw,
                                            const float* __restrict__ aux, int ldaux, int nb,
                                            Epi epi) {
  constexpr int KS = K / 32;
  static_assert(K % 32 == 0, "K padding");
  const int rot = (int)(blockIdx.x >> 3);  // spread the CUs of one XCD over the weight columns
  const int lane = threadIdx.x & 63, w = (threadIdx.x >> 6) - wbase;
  if (w < 0 || w >= nw) return;
  const int li = lane & 15, g = lane >> 4;
  int ct[TPW];
  const bf16x8* wf[TPW];
#pragma unroll
  for (int c = 0; c < TPW; ++c) {
    ct[c] = tile_base + (w + nw * c + rot) % (nw * TPW);
    wf[c] = reinterpret_cast<const bf16x8*>(W) + (size_t)ct[c] * KS * 64 + lane;
  }
  float av[2][TPW][4];
  if constexpr (AUX) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int c = 0; c < TPW; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rt * 16 + g * 4 + r, col = ct[c] * 16 + li;
          av[rt][c][r] = aux[(size_t)min(row, nb - 1) * ldaux + min(col, N - 1)];  // unpredicated
        }
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
  if constexpr (KS < 4) {
    bf16x8 q[TPW];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      loadB(ks, q);
      step(ks, q);
    }
  } else {
    constexpr int NI = (KS - 4) / 4;   // ring iterations with four refills each
    constexpr int K0 = 4 * NI;         // first k-step of the peeled tail
    constexpr int R = KS - K0;         // 4 .. 7 tail steps
    bf16x8 q0[TPW], q1[TPW], q2[TPW], q3[TPW];
    loadB(0, q0);
    loadB(1, q1);
    loadB(2, q2);
    loadB(3, q3);
#pragma unroll 1
    for (int ks = 0; ks < K0; ks += 4) {
      step(ks, q0);
      loadB(ks + 4, q0);
      __builtin_amdgcn_sched_barrier(0);
      step(ks + 1, q1);
      loadB(ks + 5, q1);
      __builtin_amdgcn_sched_barrier(0);
      step(ks + 2, q2);
      loadB(ks + 6, q2);
      __builtin_amdgcn_sched_barrier(0);
      step(ks + 3, q3);
      loadB(ks + 7, q3);
      __builtin_amdgcn_sched_barrier(0);
    }
    step(K0, q0);
    if constexpr (R > 4) loadB(K0 + 4, q0);
    step(K0 + 1, q1);
    if constexpr (R > 5) loadB(K0 + 5, q1);
    step(K0 + 2, q2);
    if constexpr (R > 6) loadB(K0 + 6, q2);
    step(K0 + 3, q3);
    if constexpr (R > 4) step(K0 + 4, q0);
    if constexpr (R > 5) step(K0 + 5, q1);
    if constexpr (R > 6) step(K0 + 6, q2);
  }
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int c = 0; c < TPW; ++c) {
      const int col = ct[c] * 16 + li;
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        epi(rt * 16 + g * 4 + r, col, acc[rt][c][r], AUX ? av[rt][c][r] : 0.0f);
    }
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

__global__ __launch_bounds__(NTHR) void stn_vae_step_bf16_kernel(StepArgs p) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) unsigned char sA[REGION_A];
  __shared__ __attribute__((aligned(16))) unsigned char sHb[REGION_H];
  __shared__ float sth[MB][12];
  __shared__ float szv[MB];
  __shared__ int smask[MB];
  __shared__ int ssep[MB];  // bit 0: theta_f axis-aligned, bit 1: theta_b (and tables fit)
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b0 = blockIdx.x * MB;
  const int nb = min(MB, p.B - b0);
  const int C = p.C, C2 = C * C;
  __bf16* sG = reinterpret_cast<__bf16*>(sA);
  float4* tabR = reinterpret_cast<float4*>(sA + OFF_TABR);
  __bf16* sA2 = reinterpret_cast<__bf16*>(sA);
  float* sMu = reinterpret_cast<float*>(sA + OFF_MU);
  float* sLv = reinterpret_cast<float*>(sA + OFF_LV);
  float* sKl = reinterpret_cast<float*>(sA + OFF_KL);
  __bf16* sZ = reinterpret_cast<__bf16*>(sA + OFF_Z);
  __bf16* sD1 = reinterpret_cast<__bf16*>(sA + OFF_D1);
  float* sR = reinterpret_cast<float*>(sA);
  __bf16* sH = reinterpret_cast<__bf16*>(sHb);
  float4* tabW = reinterpret_cast<float4*>(sHb);

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
  __syncthreads();
  if (tid < MB)
    ssep[tid] = (stn_separable(&sth[tid][0]) ? 1 : 0) |
                (stn_separable(&sth[tid][6]) && C <= CTAB_MAX ? 2 : 0);
  build_tables(tabR, TABR, sth, 0, C, C, 28, 28);
  __syncthreads();
  STAMP(0);

  // ---- 1. STN read (transformer.py:18-175): glimpse -> LDS bf16 ---------
  // Half-wave per glimpse row (lane = column), eight rows per pass so 32
  // gathers per lane are in flight.
  if (p.phases & 1) {
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
          ex[u] = tabR[mc * TABR + jc];
          ey[u] = tabR[mc * TABR + 28 + i];
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
  __syncthreads();
  STAMP(1);
  if (p.phases & 16) flush_rows(sG, SG, p.gb + (size_t)b0 * W2, W2, W2, nb);

  // ---- 2. a1 = softplus(g W1 + b1)  [MB x 512] -> H -----------------------
  if (p.phases & 2) {
    const float* bias = p.bias[0];
    dense_tiles<512, KG, 4, false>(sG, SG, p.wt[0], 0, 0, NW, nullptr, 0, nb,
                                       [&](int m, int n, float v, float) {
      sH[m * S512 + n] = (__bf16)softplus_fast(v + bias[n]);
    });
  }
  __syncthreads();
  STAMP(2);
  if (p.phases & 16) flush_rows(sH, S512, p.a1b + (size_t)b0 * 512, 512, 512, nb);
  // ---- 3. a2 = softplus(a1 W2 + b2)  [MB x 256] -> A ----------------------
  if (p.phases & 2) {
    const float* bias = p.bias[1];
    dense_tiles<256, 512, 2, false>(sH, S512, p.wt[1], 0, 0, NW, nullptr, 0, nb,
                                         [&](int m, int n, float v, float) {
      sA2[m * S256 + n] = (__bf16)softplus_fast(v + bias[n]);
    });
  }
  __syncthreads();
  STAMP(3);
  if (p.phases & 16) flush_rows(sA2, S256, p.a2b + (size_t)b0 * 256, 256, 256, nb);
  // ---- 4. mu | lv = a2 W + b  [MB x 50] fp32 (waves 0-3 | 4-7) ------------
  if (p.phases & 2) {
    const float* bm = p.bias[2];
    dense_tiles<50, 256, 1, false>(sA2, S256, p.wt[2], 0, 0, 4, nullptr, 0, nb,
                                        [&](int m, int n, float v, float) {
      sMu[m * 50 + n] = v + bm[n];
    });
    const float* bl = p.bias[3];
    dense_tiles<50, 256, 1, false>(sA2, S256, p.wt[3], 0, 4, 4, nullptr, 0, nb,
                                        [&](int m, int n, float v, float) {
      sLv[m * 50 + n] = v + bl[n];
    });
  }
  __syncthreads();
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
  __syncthreads();
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
  // ---- 6. d1 = softplus(z Wg1 + b)  [MB x 256] ----------------------------
  if (p.phases & 2) {
    const float* bias = p.bias[4];
    dense_tiles<256, 64, 2, false>(sZ, SZ, p.wt[4], 0, 0, NW, nullptr, 0, nb,
                                       [&](int m, int n, float v, float) {
      sD1[m * S256 + n] = (__bf16)softplus_fast(v + bias[n]);
    });
  }
  __syncthreads();
  STAMP(6);
  if (p.phases & 16) flush_rows(sD1, S256, p.d1b + (size_t)b0 * 256, 256, 256, nb);
  // ---- 7. d2 = softplus(d1 Wg2 + b)  [MB x 512] -> H ----------------------
  if (p.phases & 2) {
    const float* bias = p.bias[5];
    dense_tiles<512, 256, 4, false>(sD1, S256, p.wt[5], 0, 0, NW, nullptr, 0, nb,
                                         [&](int m, int n, float v, float) {
      sH[m * S512 + n] = (__bf16)softplus_fast(v + bias[n]);
    });
  }
  __syncthreads();
  STAMP(7);
  if (p.phases & 16) flush_rows(sH, S512, p.d2b + (size_t)b0 * 512, 512, 512, nb);
  // ---- 8. r = sigmoid(d2 Wgo + b + std eps)  [MB x 784] fp32 -> A ---------
  // eps_x is staged in the r tile first (generated in-kernel with the same
  // Philox quads mog_rng_fill would write, or loaded with 16-byte reads); each
  // epilogue lane reads its eps and overwrites it with r.  49 column tiles:
  // 32 (4 per wave) + 16 (2 per wave) + 1 (wave 0).
  if (p.phases & 2) {
    float4* sR4 = reinterpret_cast<float4*>(sR);
    constexpr int QPR = W2 / 4;  // 196 quads per image
    if (p.eps_gen) {
      for (int i = tid; i < nb * QPR; i += NTHR) {
        const int m = i / QPR, q = i - (i / QPR) * QPR;
        float v[4];
        mog_philox_quad(p.eps_seed, p.eps_offset + (unsigned long long)(b0 + m) * QPR + q, true,
                        v);
        sR4[i] = make_float4(v[0], v[1], v[2], v[3]);
      }
    } else {
      const float4* ex4 = reinterpret_cast<const float4*>(p.eps_x + (size_t)b0 * W2);
      for (int i = tid; i < nb * QPR; i += NTHR) sR4[i] = ex4[i];
    }
    __syncthreads();
    const float* bias = p.bias[6];
    const float sd = p.lik_std;
    auto epi = [&](int m, int n, float v, float) {
      const float e = sR[m * W2 + n];
      const float y = __builtin_fmaf(e, sd, v + bias[n]);
      sR[m * W2 + n] = 1.0f / (1.0f + __expf(-y));
    };
    dense_tiles<784, 512, 4, false>(sH, S512, p.wt[6], 0, 0, NW, nullptr, 0, nb, epi);
    dense_tiles<784, 512, 2, false>(sH, S512, p.wt[6], 32, 0, NW, nullptr, 0, nb, epi);
    dense_tiles<784, 512, 1, false>(sH, S512, p.wt[6], 48, 0, 1, nullptr, 0, nb, epi);
  }
  __syncthreads();
  STAMP(8);
  if (p.phases & 16) flush_rows(sR, W2, p.r + (size_t)b0 * W2, W2, W2, nb);
  if (C <= CTAB_MAX) build_tables(tabW, 2 * C, sth, 6, 28, 28, C, C);  // d2 is dead
  __syncthreads();
  STAMP(9);
  // ---- 9. STN write (air_model.py:580-588): this step's canvas part -------
  // part = active ? z * w : 0 for every pixel (write-only; mog_recon_loss sums
  // the parts in step order).  One wave per image; each lane produces four
  // consecutive canvas pixels (flat order) and stores them with one 16-byte
  // store.  Dead samples (clipped corners coincide on both axes) are exactly
  // +0 and are selected, not branched.
  if (p.phases & 8) {
    const int lane = tid & 63;
    const bool vec = (C2 & 3) == 0;  // even C: 16-byte aligned image rows of parts
    for (int m = wv; m < nb; m += NW) {
      float* om = p.part + (size_t)(b0 + m) * C2;
      const float* U = sR + m * W2;
      const bool act = smask[m] != 0, tab = (ssep[m] & 2) != 0;
      const float zn = szv[m];
      const float4* tcol = tabW + m * 2 * C;
      const float4* trow = tcol + C;
      const int nq = vec ? C2 / 4 : C2;
      const int per = vec ? 4 : 1;
      for (int q = lane; q < nq; q += 64) {
        float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (act) {
          int pix = q * per;
          int i = pix / C, j = pix - (pix / C) * C;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (e < per) {
              if (tab) {
                const float4 ex = tcol[j], ey = trow[i];
                const int x0 = __float_as_int(ex.x), x1 = __float_as_int(ex.y);
                const int y0 = __float_as_int(ey.x), y1 = __float_as_int(ey.y);
                const float s = zn * sample4(ex, ey, U[y0 + x0], U[y1 + x0], U[y0 + x1],
                                             U[y1 + x1]);
                v[e] = axis4_dead(ex, ey) ? 0.0f : s;
              } else {
                const Tap t = stn_tap(&sth[m][6], 28, 28, mog_linspace(j, C), mog_linspace(i, C));
                v[e] = t.dead ? 0.0f : zn * tap_value(t, U);
              }
              if (++j == C) { j = 0; ++i; }
            }
          }
        }
        if (vec)
          reinterpret_cast<float4*>(om)[q] = make_float4(v[0], v[1], v[2], v[3]);
        else
          om[q] = v[0];
      }
    }
  }
  if (p.tstamp) {
    __syncthreads();
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
                                    "g1", "g2", "go", "flush_r+tables", "write"};
    double acc[11] = {0};
    long long t0 = h[0], t1 = h[10];
    for (unsigned b = 0; b < nblk; ++b) {
      for (int k = 0; k < 10; ++k) acc[k] += (double)(h[b * 16 + k + 1] - h[b * 16 + k]);
      acc[10] += (double)(h[b * 16 + 10] - h[b * 16]);
      t0 = std::min(t0, h[b * 16]);
      t1 = std::max(t1, h[b * 16 + 10]);
    }
    fprintf(stderr, "stn_vae_step phases (us, mean over %u blocks; 100 MHz clock):", nblk);
    for (int k = 0; k < 10; ++k) fprintf(stderr, " %s %.2f", names[k], acc[k] / nblk / 100.0);
    fprintf(stderr, " | block %.2f | span %.2f\n", acc[10] / nblk / 100.0, (t1 - t0) / 100.0);
  }
  MOG_LAUNCH_RET();
}
