// Fused per-object step: STN read -> glimpse VAE -> latent sample + KL ->
// STN write + masked canvas accumulation, one launch per loop step
// (air_model.py:500-588 + :665-675 + :718-736, vae.py:5-48,
// transformer.py:18-175).  This is the kernel SURVEY.md §8 D.3 prices at
// 30,024 algorithmic HBM bytes per image-step.
//
// One workgroup = 4 waves = MB (32) images.  Activations stay in LDS between
// the six dense layers (bf16, rows padded to kill bank conflicts); the packed
// bf16 weights (W^T, [out][in8]) stream from L2 straight into the MFMA B
// operand (16 B per lane, one k-step of register prefetch); the A operand is
// read from LDS with ds_read_b128.  Activations needed by the backward pass
// (glimpse, softplus outputs, mu/logvar/z, r) are written to HBM as they are
// produced.  The STN write re-reads r (fp32) that this workgroup just stored
// (L2-resident, never cached in this CU's L1 before: the launch invalidates
// L1) and accumulates into the canvas only where the sample is not exactly
// zero (x0 == x1 && y0 == y1 gives +0; skipping keeps the canvas
// bit-identical).
//
// Precision: bf16 MFMA operands, fp32 accumulation and epilogues with
// hardware transcendentals (the bf16 configuration, BASELINE configs[1]).
#include "mog_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int MB = 32;        // images per workgroup
constexpr int NW = 8;         // waves per workgroup
constexpr int NTHR = NW * 64;
constexpr int W2 = 784;       // 28 x 28 glimpse
constexpr int KG = 800;       // glimpse k extent padded to a multiple of 32
constexpr int SG = KG + 8;    // LDS row strides (bf16), +16 B against bank conflicts
constexpr int S512 = 512 + 8, S256 = 256 + 8, SZ = 64 + 8;
// LDS region A (bytes): glimpse tile, then a2 | mu | lv | z | d1, then r (fp32)
constexpr int OFF_MU = MB * S256 * 2;
constexpr int OFF_LV = OFF_MU + MB * 50 * 4;
constexpr int OFF_Z = OFF_LV + MB * 50 * 4;
constexpr int OFF_D1 = OFF_Z + MB * SZ * 2;
constexpr int REGION_A = MB * W2 * 4;
constexpr int OFF_TABR = MB * SG * 2;     // read-phase axis tables (after the glimpse tile)
constexpr int TABR = 28 + 28;
constexpr int TABW = 64 + 64;             // write-phase axis tables (in sH), canvas <= 64
static_assert(OFF_TABR + MB * TABR * 8 <= REGION_A && MB * TABW * 8 <= MB * S512 * 2, "tables");
static_assert(MB * SG * 2 <= REGION_A && OFF_D1 + MB * S256 * 2 <= REGION_A, "LDS layout");

struct StepArgs {
  const float* x;            // [B, C*C] canvas input
  const float* theta_f;      // [B, 6]
  const float* theta_b;      // [B, 6]
  const float* mask;         // [B] active (new stopping sum < thr)
  const float* zval;         // [B] z_pres
  const float* eps_z;        // [B, Z]
  const float* eps_x;        // [B, 784]
  const __bf16* wt[7];       // packed W^T: r1 [512][784], r2 [256][512], mu [50][256],
                             //             lv [50][256], g1 [256][56], g2 [512][256], go [784][512]
  const float* bias[7];
  float* canvas;             // [B, C*C] accumulated in place
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
  int phases;  // profiling aid: bit mask of the phases to run (all by default)
};

__device__ __forceinline__ float softplus_fast(float v) {
  return v > -MOG_SOFTPLUS_T ? v : (v < MOG_SOFTPLUS_T ? __expf(v) : __logf(__expf(v) + 1.0f));
}

// Bilinear sample geometry (transformer.py:75-116), op-for-op as stn.hip.
struct Tap {
  float x, y, x0f, x1f, y0f, y1f;
  int ia, ib, ic, id;
  bool dead;  // all four clipped corners coincide: the sample is +0 exactly
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

// Axis-aligned transforms (theta01 == theta10 == 0, always so in AIR) make the
// sample geometry separable: x depends on the output column only, y on the
// row only (th1*yt is +-0 and adding it leaves the sum bit-identical), so the
// coordinate and clipped corner pair are tabulated once per column / row:
// {coordinate, lo | hi << 16}.
__device__ __forceinline__ float2 axis_entry(float c, float lo_f, float hi_f) {
  return make_float2(c, __int_as_float((int)lo_f | ((int)hi_f << 16)));
}

__device__ __forceinline__ Tap tap_from(float2 ex, float2 ey, int Win) {
  Tap s;
  const int px = __float_as_int(ex.y), py = __float_as_int(ey.y);
  const int x0 = px & 0xffff, x1 = px >> 16, y0 = py & 0xffff, y1 = py >> 16;
  s.x = ex.x; s.y = ey.x;
  s.x0f = (float)x0; s.x1f = (float)x1; s.y0f = (float)y0; s.y1f = (float)y1;
  s.ia = y0 * Win + x0; s.ib = y1 * Win + x0; s.ic = y0 * Win + x1; s.id = y1 * Win + x1;
  s.dead = (x0 == x1) && (y0 == y1);
  return s;
}

// Fill tab[m][0..Wout) with column entries and tab[m][Wout..Wout+Hout) with row
// entries for every image m whose transform (th at sth[m][th_off]) is
// axis-aligned.  stride = entries per image.
__device__ __forceinline__ void build_axis_tables(float2* tab, int stride, const float (*sth)[12],
                                                  int th_off, int Hin, int Win, int Hout,
                                                  int Wout) {
  const int per = Wout + Hout;
  for (int i = threadIdx.x; i < MB * per; i += NTHR) {
    const int m = i / per, n = i - (i / per) * per;
    const float* th = &sth[m][th_off];
    if (n < Wout) {
      const Tap t = stn_tap(th, Hin, Win, mog_linspace(n, Wout), mog_linspace(0, Hout));
      tab[m * stride + n] = axis_entry(t.x, t.x0f, t.x1f);
    } else {
      const Tap t = stn_tap(th, Hin, Win, mog_linspace(0, Wout), mog_linspace(n - Wout, Hout));
      tab[m * stride + n] = axis_entry(t.y, t.y0f, t.y1f);
    }
  }
}

// One dense layer over the MB rows held in LDS: epi(row, col, A @ W^T).
// A: LDS [MB][lda] bf16, zero-padded to K (a multiple of 32); W: global
// [N][ldw] bf16, k < KW valid.  Waves wbase .. wbase+nw-1 take column tiles
// round-robin, four per pass; B fragments stream from L2 with a two-k-step
// register prefetch ring (the k loop is unrolled so the ring is static).
template <int N, int K, int KW, class Epi>
__device__ __forceinline__ void dense_layer(const __bf16* A, int lda, const __bf16* __restrict__ W,
                                            int ldw, int wbase, int nw, Epi epi) {
  constexpr int NT = (N + 15) / 16;
  constexpr int KS = K / 32;
  static_assert(K % 32 == 0, "K padded");
  const int lane = threadIdx.x & 63, w = (threadIdx.x >> 6) - wbase;
  if (w < 0 || w >= nw) return;
  const int li = lane & 15, g = lane >> 4;
  const bf16x8 zero8 = {};
  for (int ct0 = w; ct0 < NT; ct0 += 4 * nw) {
    int ct[4];
    bool cv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      ct[c] = ct0 + nw * c;
      cv[c] = ct[c] < NT && ct[c] * 16 + li < N;
    }
    floatx4 acc[2][4];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[rt][c] = floatx4{0.f, 0.f, 0.f, 0.f};
    // Rows past N are clamped to a valid row: those columns are discarded by
    // the epilogue, so their B values never matter.  Past KW (only in the last
    // k-step of a padded layer) the fragment is zeroed: A is zero there too,
    // but the bytes beyond the last row are not ours to read.
    const __bf16* wrow[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) wrow[c] = W + (size_t)min(ct[c] * 16 + li, N - 1) * ldw + 8 * g;
    bf16x8 bq[3][4];
    auto loadB = [&](int ks, bf16x8* b) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (ks * 32 + 32 <= KW)
          b[c] = *reinterpret_cast<const bf16x8*>(wrow[c] + ks * 32);
        else
          b[c] = ks * 32 + 8 * g < KW ? *reinterpret_cast<const bf16x8*>(wrow[c] + ks * 32) : zero8;
      }
    };
    loadB(0, bq[0]);
    if (KS > 1) loadB(1, bq[1]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 2 < KS) loadB(ks + 2, bq[(ks + 2) % 3]);
      const int k = ks * 32 + 8 * g;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&A[li * lda + k]);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&A[(16 + li) * lda + k]);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[0][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bq[ks % 3][c], acc[0][c], 0, 0, 0);
        acc[1][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bq[ks % 3][c], acc[1][c], 0, 0, 0);
      }
    }
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (!cv[c]) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) epi(rt * 16 + g * 4 + r, ct[c] * 16 + li, acc[rt][c][r]);
      }
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

__global__ __launch_bounds__(NTHR) void stn_vae_step_bf16_kernel(StepArgs p) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) unsigned char sA[REGION_A];
  __shared__ __attribute__((aligned(16))) __bf16 sH[MB * S512];
  __shared__ float sth[MB][12];
  __shared__ float szv[MB];
  __shared__ int smask[MB];
  __shared__ int ssep[MB];  // bit 0: theta_f axis-aligned, bit 1: theta_b
  const int tid = threadIdx.x;
  const int b0 = blockIdx.x * MB;
  const int nb = min(MB, p.B - b0);
  const int C = p.C, C2 = C * C;
  __bf16* sG = reinterpret_cast<__bf16*>(sA);
  __bf16* sA2 = reinterpret_cast<__bf16*>(sA);
  float* sMu = reinterpret_cast<float*>(sA + OFF_MU);
  float* sLv = reinterpret_cast<float*>(sA + OFF_LV);
  __bf16* sZ = reinterpret_cast<__bf16*>(sA + OFF_Z);
  __bf16* sD1 = reinterpret_cast<__bf16*>(sA + OFF_D1);
  float* sR = reinterpret_cast<float*>(sA);

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
    ssep[tid] = (sth[tid][1] == 0.0f && sth[tid][3] == 0.0f ? 1 : 0) |
                (sth[tid][7] == 0.0f && sth[tid][9] == 0.0f && C <= 64 ? 2 : 0);
  float2* tabR = reinterpret_cast<float2*>(sA + OFF_TABR);
  build_axis_tables(tabR, TABR, sth, 0, C, C, 28, 28);
  __syncthreads();

  // ---- 1. STN read (transformer.py:18-175): glimpse -> LDS bf16 ---------
  // four samples per thread per pass: 16 independent gathers in flight
  if (p.phases & 1) {
    constexpr int UR = 4;
    for (int base = 0; base < MB * KG; base += NTHR * UR) {
      Tap tp[UR];
      int mm[UR];
      bool live[UR];
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const int idx = base + u * NTHR + tid;
        const int m = idx / KG, k = idx - (idx / KG) * KG;
        mm[u] = idx;
        live[u] = idx < MB * KG && m < nb && k < W2;
        const int i = k / 28, j = k - (k / 28) * 28;
        const int mc = live[u] ? m : 0;
        tp[u] = (ssep[mc] & 1) ? tap_from(tabR[mc * TABR + j], tabR[mc * TABR + 28 + i], C)
                               : stn_tap(sth[mc], C, C, mog_linspace(j, 28), mog_linspace(i, 28));
        live[u] = live[u] && !tp[u].dead;
      }
      float I[UR][4];
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const float* U = p.x + (size_t)(b0 + mm[u] / KG) * C2;
        I[u][0] = live[u] ? U[tp[u].ia] : 0.0f;
        I[u][1] = live[u] ? U[tp[u].ib] : 0.0f;
        I[u][2] = live[u] ? U[tp[u].ic] : 0.0f;
        I[u][3] = live[u] ? U[tp[u].id] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const int idx = mm[u];
        if (idx >= MB * KG) continue;
        const float v = live[u] ? tap_value(tp[u], I[u][0], I[u][1], I[u][2], I[u][3]) : 0.0f;
        const int m = idx / KG, k = idx - (idx / KG) * KG;
        sG[m * SG + k] = (__bf16)v;
      }
    }
  }
  __syncthreads();
  if (p.phases & 16) flush_rows(sG, SG, p.gb + (size_t)b0 * W2, W2, W2, nb);

  // ---- 2. a1 = softplus(g W1 + b1)  [MB x 512] -> sH ---------------------
  if (p.phases & 2) {
    const float* bias = p.bias[0];
    dense_layer<512, KG, W2>(sG, SG, p.wt[0], W2, 0, NW, [&](int m, int n, float v) {
      sH[m * S512 + n] = (__bf16)softplus_fast(v + bias[n]);
    });
  }
  __syncthreads();
  if (p.phases & 16) flush_rows(sH, S512, p.a1b + (size_t)b0 * 512, 512, 512, nb);
  // ---- 3. a2 = softplus(a1 W2 + b2)  [MB x 256] -> region A ---------------
  if (p.phases & 2) {
    const float* bias = p.bias[1];
    dense_layer<256, 512, 512>(sH, S512, p.wt[1], 512, 0, NW, [&](int m, int n, float v) {
      sA2[m * S256 + n] = (__bf16)softplus_fast(v + bias[n]);
    });
  }
  __syncthreads();
  if (p.phases & 16) flush_rows(sA2, S256, p.a2b + (size_t)b0 * 256, 256, 256, nb);
  // ---- 4. mu | lv = a2 W + b  [MB x 50] fp32 (waves 0-3 | 4-7) ------------
  if (p.phases & 2) {
    const float* bm = p.bias[2];
    dense_layer<50, 256, 256>(sA2, S256, p.wt[2], 256, 0, 4, [&](int m, int n, float v) {
      sMu[m * 50 + n] = v + bm[n];
    });
    const float* bl = p.bias[3];
    dense_layer<50, 256, 256>(sA2, S256, p.wt[3], 256, 4, 4, [&](int m, int n, float v) {
      sLv[m * 50 + n] = v + bl[n];
    });
  }
  __syncthreads();
  // ---- 5. z = mu + eps sqrt(exp(lv)); VAE KL -> runloss (vae.py:27-30) ---
  for (int i = tid; i < MB * 64; i += NTHR) {
    const int m = i >> 6, k = i & 63;
    float zv = 0.0f;
    if (k < 50 && m < nb) {
      const size_t o = (size_t)(b0 + m) * 50 + k;
      const float l = sLv[m * 50 + k];
      const float mv = sMu[m * 50 + k];
      zv = mv + p.eps_z[o] * sqrtf(mog_expf(l));
      p.mu[o] = mv;
      p.lv[o] = l;
      p.z[o] = zv;
      p.zb[(size_t)(b0 + m) * 56 + k] = (__bf16)zv;
    }
    sZ[m * SZ + k] = (__bf16)zv;
  }
  if (tid < nb) {  // sequential KL sum per image (k order, as vae_sample_fwd_kernel)
    const int m = tid;
    float sum = 0.0f;
    for (int k = 0; k < 50; ++k) {
      const float l = sLv[m * 50 + k];
      const float var = mog_expf(l);
      const float d = sMu[m * 50 + k] - p.v_pm;
      sum = sum + ((((p.v_plv - l) - 1.0f) + var / p.v_pv) + (d * d) / p.v_pv);
    }
    const float vkl = 0.5f * sum;
    p.vkl[b0 + m] = vkl;
    if (smask[m]) p.runloss[b0 + m] = p.runloss[b0 + m] + vkl;
  }
  __syncthreads();
  // ---- 6. d1 = softplus(z Wg1 + b)  [MB x 256] ----------------------------
  if (p.phases & 2) {
    const float* bias = p.bias[4];
    dense_layer<256, 64, 56>(sZ, SZ, p.wt[4], 56, 0, NW, [&](int m, int n, float v) {
      sD1[m * S256 + n] = (__bf16)softplus_fast(v + bias[n]);
    });
  }
  __syncthreads();
  if (p.phases & 16) flush_rows(sD1, S256, p.d1b + (size_t)b0 * 256, 256, 256, nb);
  // ---- 7. d2 = softplus(d1 Wg2 + b)  [MB x 512] -> sH ---------------------
  if (p.phases & 2) {
    const float* bias = p.bias[5];
    dense_layer<512, 256, 256>(sD1, S256, p.wt[5], 256, 0, NW, [&](int m, int n, float v) {
      sH[m * S512 + n] = (__bf16)softplus_fast(v + bias[n]);
    });
  }
  __syncthreads();
  if (p.phases & 16) flush_rows(sH, S512, p.d2b + (size_t)b0 * 512, 512, 512, nb);
  // ---- 8. r = sigmoid(d2 Wgo + b + std eps)  [MB x 784] fp32 -> region A --
  if (p.phases & 2) {
    const float* bias = p.bias[6];
    const float sd = p.lik_std;
    const float* ex = p.eps_x + (size_t)b0 * W2;
    dense_layer<784, 512, 512>(sH, S512, p.wt[6], 512, 0, NW, [&](int m, int n, float v) {
      const float e = m < nb ? ex[m * W2 + n] : 0.0f;
      const float y = __builtin_fmaf(e, sd, v + bias[n]);
      sR[m * W2 + n] = 1.0f / (1.0f + __expf(-y));
    });
  }
  __syncthreads();
  if (p.phases & 16) flush_rows(sR, W2, p.r + (size_t)b0 * W2, W2, W2, nb);
  float2* tabW = reinterpret_cast<float2*>(sH);  // d2 is dead after the last layer
  if (C <= 64) build_axis_tables(tabW, TABW, sth, 6, 28, 28, C, C);
  __syncthreads();
  // ---- 9. STN write + masked canvas accumulation (air_model.py:580-675) --
  // canvas += z * w only where the sample is not exactly zero; eight pixels
  // per thread per pass so the canvas loads overlap.
  if (p.phases & 8) {
    constexpr int UW = 8;
    const int total = nb * C2;
    const float invC2 = 1.0f / (float)C2, invC = 1.0f / (float)C;
    for (int base = 0; base < total; base += NTHR * UW) {
      float v[UW];
      int off[UW];
      bool live[UW];
#pragma unroll
      for (int u = 0; u < UW; ++u) {
        const int idx = base + u * NTHR + tid;
        // exact: |error| of the float quotient << 0.5 / C2 for idx < 2^21
        const int m = (int)(((float)idx + 0.5f) * invC2);
        const int k = idx - m * C2;
        live[u] = idx < total && smask[min(m, MB - 1)];
        off[u] = idx;
        v[u] = 0.0f;
        if (live[u]) {
          const int i = (int)(((float)k + 0.5f) * invC), j = k - i * C;
          const Tap t = (ssep[m] & 2)
                            ? tap_from(tabW[m * TABW + j], tabW[m * TABW + C + i], 28)
                            : stn_tap(&sth[m][6], 28, 28, mog_linspace(j, C), mog_linspace(i, C));
          live[u] = !t.dead;
          if (live[u]) {
            const float* U = sR + m * W2;
            v[u] = szv[m] * tap_value(t, U[t.ia], U[t.ib], U[t.ic], U[t.id]);
          }
        }
      }
      float* cv = p.canvas + (size_t)b0 * C2;
      float c[UW];
#pragma unroll
      for (int u = 0; u < UW; ++u) c[u] = live[u] ? cv[off[u]] : 0.0f;
#pragma unroll
      for (int u = 0; u < UW; ++u)
        if (live[u]) cv[off[u]] = c[u] + v[u];
    }
  }
}

}  // namespace

extern "C" int mog_stn_vae_step_forward(int B, int C, int W, int R1, int R2, int Z, int G1,
                                        int G2, const float* x, const float* theta_f,
                                        const float* theta_b, const float* mask,
                                        const float* zval, const float* eps_z,
                                        const float* eps_x, const void* const* wt,
                                        const float* const* bias, float lik_std, float v_pm,
                                        float v_pv, float v_plv, float* canvas,
                                        float* runloss, float* vkl, void* gb, void* a1b,
                                        void* a2b, float* mu, float* lv, float* z, void* zb,
                                        void* d1b, void* d2b, float* r, void* stream) {
  MOG_CHECK_ARG(B >= 0 && C > 0 && C * C <= 16384);
  // the tile shapes are compiled for the reference's default VAE
  MOG_CHECK_ARG(W == 28 && R1 == 512 && R2 == 256 && Z == 50 && G1 == 256 && G2 == 512);
  MOG_CHECK_ARG(x && theta_f && theta_b && mask && zval && eps_z && eps_x && wt && bias);
  MOG_CHECK_ARG(canvas && runloss && vkl && gb && a1b && a2b && mu && lv && z && zb);
  MOG_CHECK_ARG(d1b && d2b && r);
  if (B == 0) return 0;
  StepArgs p;
  p.x = x; p.theta_f = theta_f; p.theta_b = theta_b; p.mask = mask; p.zval = zval;
  p.eps_z = eps_z; p.eps_x = eps_x;
  for (int i = 0; i < 7; ++i) {
    MOG_CHECK_ARG(wt[i] && bias[i]);
    p.wt[i] = reinterpret_cast<const __bf16*>(wt[i]);
    p.bias[i] = bias[i];
  }
  p.canvas = canvas; p.runloss = runloss; p.vkl = vkl;
  p.gb = reinterpret_cast<__bf16*>(gb); p.a1b = reinterpret_cast<__bf16*>(a1b);
  p.a2b = reinterpret_cast<__bf16*>(a2b); p.mu = mu; p.lv = lv; p.z = z;
  p.zb = reinterpret_cast<__bf16*>(zb); p.d1b = reinterpret_cast<__bf16*>(d1b);
  p.d2b = reinterpret_cast<__bf16*>(d2b); p.r = r;
  const char* ph = getenv("MOG_VS_PHASES");
  p.phases = ph ? atoi(ph) : 31;
  p.B = B; p.C = C; p.lik_std = lik_std; p.v_pm = v_pm; p.v_pv = v_pv; p.v_plv = v_plv;
  stn_vae_step_bf16_kernel<<<mog_cdiv(B, MB), NTHR, 0, mog_stream(stream)>>>(p);
  MOG_LAUNCH_RET();
}
