// AIR-ASR per-step cells and structural losses:
// air/air_number_bbox_location.py:384-1079.  Everything here is scalar /
// per-image work around the GEMM, LSTM, STN and glimpse-VAE kernels the AIR
// path already has; the forward numerics follow oracle/asr_ref.c op for op
// (k-ordered fma chains, mog_math.h transcendentals, contraction off); the
// backward is hand-derived (TF gradient conventions: Maximum / Minimum pass
// the gradient at ties to the first operand, ReduceMin splits it evenly over
// tied minima, Abs' = sign).
#include "mog_common.h"

namespace {

// step-record slots ([Q_N][B] per step)
enum {
  Q_SM0, Q_SM1, Q_SLV0, Q_SLV1, Q_SL0, Q_SL1, Q_CM, Q_CLV, Q_CL, Q_S, Q_TX, Q_TY,
  Q_GSM0, Q_GSM1, Q_GSLV0, Q_GSLV1, Q_PLO, Q_LO, Q_Y, Q_Z, Q_ACT_OLD, Q_ACT, Q_LIVE,
  Q_ZKL, Q_SKL, Q_SHKL, Q_PRN, Q_ZPROB, Q_N
};
static_assert(Q_N == 28, "record layout is part of the ABI (include/mog_air.h)");

// output-layer weights (TF [in, out]) in the ABI order of w[20]
enum {
  W_IS1, B_IS1, W_IS3, B_IS3,            // inf_shift dense_1 / dense_3  [64,2]
  W_IC0, B_IC0, W_IC1, B_IC1,            // inf_scale dense [258,64] / dense_1 [66,1]
  W_IC2, B_IC2, W_IC3, B_IC3,            // inf_scale dense_2 / dense_3
  W_GS1, B_GS1, W_GS3, B_GS3,            // gen_shift dense_1 / dense_3 [64,2]
  W_ZP1, B_ZP1, W_ZL1, B_ZL1,            // z_pres prior / log-odds dense_1 [64,1]
  W_N
};

// douts slots ([B][12] per step): gradients wrt the output-layer values
enum { D_SM0, D_SM1, D_SLV0, D_SLV1, D_LO, D_GSM0, D_GSM1, D_GSLV0, D_GSLV1, D_PLO, D_CM,
       D_CLV, D_N };

struct AsrCfg {
  int B, step, train, fix_steps;
  float thr, temperature, gcm, gcvar, gclv, g_num, grad_scale;
};

struct AsrW {
  const float* w[W_N];
};
struct AsrHid {
  float* h[8];  // [B,64]: 0 inf_shift m, 1 inf_shift v, 2 z_pres log-odds, 3 gen_shift m,
                // 4 gen_shift v, 5 z_pres prior (or null), 6/7 inf_scale m/v (raw -> finished)
};

constexpr int HS = 64;

// one k-ordered fma chain; the operands of 32 k-steps loaded before their
// fmas (one memory round trip per 32 k, not per k; same bits)
__device__ __forceinline__ float chain64(const float* a, const float* w, int ldw) {
#pragma clang fp contract(off)
  float acc = 0.0f;
#pragma unroll
  for (int k0 = 0; k0 < HS; k0 += 32) {
    float av[32], wv[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      av[i] = a[k0 + i];
      wv[i] = w[(size_t)(k0 + i) * ldw];
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) acc = fmaf(av[i], wv[i], acc);
  }
  return acc;
}

__device__ __forceinline__ float lse0(float a) {
#pragma clang fp contract(off)
  float m = a > 0.0f ? a : 0.0f;
  if (!(m - m == 0.0f)) m = 0.0f;
  return mog_logf(mog_expf(0.0f - m) + mog_expf(a - m)) + m;
}

__device__ __forceinline__ float concrete_kl(float y, float plo, float pT, float qlo, float qT) {
#pragma clang fp contract(off)
  const float eps = 1e-9f;
  const float lse_p = lse0(-y * pT + plo);
  const float log_prior = ((mog_logf(pT + eps) - y * (pT + 1.0f)) + plo) - 2.0f * lse_p;
  const float lse_q = lse0(-y * qT + qlo);
  const float log_post = ((mog_logf(qT + eps) - y * (qT + 1.0f)) + qlo) - 2.0f * lse_q;
  return log_post - log_prior;
}

// U rows [z_prev (Z) | ss_prev (3) | h_prev (H) | 0 pad] (the LSTMCell input
// concat order, :403-412 / :457-463); null sources are zeros (step 0)
// (out2 != null: a second output from h2 in the same launch -- the two cells'
// rows share z and ss)
__global__ __launch_bounds__(256) void asr_pack_kernel(int B, int Z, int H, int ld,
                                                       const float* z, const float* ss,
                                                       const float* h, float* out,
                                                       const float* h2, float* out2) {
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long n = (long)B * ld;
  if (i >= (out2 ? 2 * n : n)) return;
  if (i >= n) {
    i -= n;
    h = h2;
    out = out2;
  }
  const int b = i / ld, k = i - (long)b * ld;
  float v = 0.0f;
  if (k < Z) v = z ? z[(size_t)b * Z + k] : 0.0f;
  else if (k < Z + 3) v = ss ? ss[(size_t)b * 3 + k - Z] : 0.0f;
  else if (k < Z + 3 + H) v = h ? h[(size_t)b * H + k - Z - 3] : 0.0f;
  out[i] = v;
}

// gradient of the packed rows back to its sources: z / ss carries (the two
// LSTMCell inputs add), h_prev += dU[.., Z+3 ..], hg_prev += dUg[.., Z+3 ..]
__global__ __launch_bounds__(256) void asr_unpack_kernel(int B, int Z, int H, int ld,
                                                         const float* dU, const float* dUg,
                                                         float* dz, float* dss, float* dh,
                                                         float* dhg, int acc_dz, int nparts,
                                                         long part_stride) {
#pragma clang fp contract(off)
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * (Z + 3 + H)) return;
  const int n = Z + 3 + H;
  const int b = i / n, k = i - (long)b * n;
  float a = dU[(size_t)b * ld + k], g = dUg[(size_t)b * ld + k];
  if (nparts > 1) {  // dU / dUg as K parts of their GEMM: summed in part order
    float pa[4], pg[4];
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      pa[j] = j < nparts ? dU[j * part_stride + (size_t)b * ld + k] : 0.0f;
      pg[j] = j < nparts ? dUg[j * part_stride + (size_t)b * ld + k] : 0.0f;
    }
#pragma unroll
    for (int j = 1; j < 4; ++j)
      if (j < nparts) {
        a = a + pa[j];
        g = g + pg[j];
      }
  }
  if (k < Z) {
    const size_t o = (size_t)b * Z + k;
    dz[o] = acc_dz ? dz[o] + (a + g) : a + g;  // (the same sum as add_(dz, carry))
  }
  else if (k < Z + 3) dss[(size_t)b * 3 + k - Z] = a + g;
  else {
    const size_t o = (size_t)b * H + k - Z - 3;
    dh[o] = dh[o] + a;
    dhg[o] = dhg[o] + g;
  }
}

struct AsrFwdIO {
  const float* eps_shift;  // [B,2]
  const float* eps_scale;  // [B]
  const float* u;          // [B]
  float* stop;             // [B] state
  int* digits;             // [B] state
  int* live;               // [T+1]
  float* rec;              // [Q_N, B]
  float* theta_fwd;        // [B,6]
  float* theta_back;       // [B,6]
  float* ss;               // [B,3] (shift latent x, y; scale latent)
  float* scale;            // [B]
  float* shift;            // [B,2]
  float* zprob;            // [B]
  float* zmask;            // [B]
  float* zval;             // [B]
  float* zc;               // [B] canvas coefficient active ? z : 0 (STN-write backward scale)
};

// One wave per image (4 per block): head output chains, latent sampling, the
// scale hidden layers finished over the shift latent, theta / theta^-1,
// concrete z_pres, KLs, entropy regulariser, stopping sum, counts, live flag.
__global__ __launch_bounds__(256) void asr_step_fwd_kernel(AsrCfg cfg, AsrW W, AsrHid hp,
                                                           AsrFwdIO io) {
#pragma clang fp contract(off)
  __shared__ float sv[4][16];
  __shared__ float sh6[4][HS], sh7[4][HS];
  const int m = threadIdx.x >> 6, q = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + m;
  const int B = cfg.B;
  const bool ok = b < B;
  const int bc = ok ? b : 0;
  // the later phases' global operands loaded up front, unconditionally (one
  // memory latency for all of them instead of one per phase behind the
  // barriers; clamped image index, as the chains below)
  const size_t r6 = (size_t)bc * HS + q;
  const float es0 = io.eps_shift[(size_t)bc * 2], es1 = io.eps_shift[(size_t)bc * 2 + 1];
  const float h6 = hp.h[6][r6], h7 = hp.h[7][r6];
  const float w6a = W.w[W_IC0][256 * HS + q], w6b = W.w[W_IC0][257 * HS + q], b6 = W.w[B_IC0][q];
  const float w7a = W.w[W_IC2][256 * HS + q], w7b = W.w[W_IC2][257 * HS + q], b7 = W.w[B_IC2][q];
  const float e_s = io.eps_scale[bc], uu = io.u[bc], stop_old = io.stop[bc];
  const int live = io.live[cfg.step], dig = io.digits[bc];
  // phase 1: ten output-layer chains over the 64 hidden units
  if (q < 10) {
    float v = 0.0f;
    const size_t r = (size_t)bc * HS;
    switch (q) {
      case 0: v = chain64(hp.h[0] + r, W.w[W_IS1], 2) + W.w[B_IS1][0]; break;
      case 1: v = chain64(hp.h[0] + r, W.w[W_IS1] + 1, 2) + W.w[B_IS1][1]; break;
      case 2: v = chain64(hp.h[1] + r, W.w[W_IS3], 2) + W.w[B_IS3][0]; break;
      case 3: v = chain64(hp.h[1] + r, W.w[W_IS3] + 1, 2) + W.w[B_IS3][1]; break;
      case 4: v = chain64(hp.h[3] + r, W.w[W_GS1], 2) + W.w[B_GS1][0]; break;
      case 5: v = chain64(hp.h[3] + r, W.w[W_GS1] + 1, 2) + W.w[B_GS1][1]; break;
      case 6: v = chain64(hp.h[4] + r, W.w[W_GS3], 2) + W.w[B_GS3][0]; break;
      case 7: v = chain64(hp.h[4] + r, W.w[W_GS3] + 1, 2) + W.w[B_GS3][1]; break;
      case 8: v = chain64(hp.h[2] + r, W.w[W_ZL1], 1) + W.w[B_ZL1][0]; break;
      default:
        v = cfg.fix_steps >= 0 ? (cfg.step < cfg.fix_steps ? 100.0f : -100.0f)
                               : chain64(hp.h[5] + r, W.w[W_ZP1], 1) + W.w[B_ZP1][0];
    }
    sv[m][q] = v;
  }
  __syncthreads();
  // phase 2: shift latent (:424-427)
  if (q == 0) {
    for (int d = 0; d < 2; ++d) {
      const float svar = mog_expf(sv[m][2 + d]);
      sv[m][10 + d] = sv[m][d] + (d == 0 ? es0 : es1) * sqrtf(svar);
    }
  }
  __syncthreads();
  // phase 3: inf_scale hidden layers on concat([h, shift_latent]) (:429-447):
  // the GEMM left the chain over h; add the two latent terms, bias, relu
  const float sl0 = sv[m][10], sl1 = sv[m][11];
  {
    float a6 = h6, a7 = h7;
    a6 = fmaf(sl0, w6a, a6);
    a6 = fmaf(sl1, w6b, a6);
    a6 = a6 + b6;
    a7 = fmaf(sl0, w7a, a7);
    a7 = fmaf(sl1, w7b, a7);
    a7 = a7 + b7;
    sh6[m][q] = a6 > 0.0f ? a6 : 0.0f;
    sh7[m][q] = a7 > 0.0f ? a7 : 0.0f;
  }
  __syncthreads();
  if (ok) {
    hp.h[6][r6] = sh6[m][q];
    hp.h[7][r6] = sh7[m][q];
  }
  // phase 4: scale mean / log-variance on concat([hidden, shift_latent])
  if (q < 2) {
    const float* hh = q == 0 ? sh6[m] : sh7[m];
    const float* w = W.w[q == 0 ? W_IC1 : W_IC3];
    float acc = chain64(hh, w, 1);
    acc = fmaf(sl0, w[HS], acc);
    acc = fmaf(sl1, w[HS + 1], acc);
    sv[m][12 + q] = acc + W.w[q == 0 ? B_IC1 : B_IC3][0];
  }
  __syncthreads();
  if (q != 0 || !ok) return;
  // phase 5: everything per image (:424-772)
  const float sm0 = sv[m][0], sm1 = sv[m][1], slv0 = sv[m][2], slv1 = sv[m][3];
  const float gsm0 = sv[m][4], gsm1 = sv[m][5], gslv0 = sv[m][6], gslv1 = sv[m][7];
  const float lo = sv[m][8], plo = sv[m][9];
  const float cm = sv[m][12], clv = sv[m][13];
  // (every per-image input was read at the top, before the first store:
  // stores through possibly-aliasing pointers would otherwise order each
  // later load behind them -- one memory round trip per load on this chain)
  const float tx = mog_tanhf(sl0), ty = mog_tanhf(sl1);
  const float cvar = mog_expf(clv);
  const float cl = cm + e_s * sqrtf(cvar);
  const float s = mog_sigmoidf(cl);
  float* tf = io.theta_fwd + (size_t)b * 6;
  tf[0] = s; tf[1] = 0.0f; tf[2] = tx; tf[3] = 0.0f; tf[4] = s; tf[5] = ty;
  float* tb = io.theta_back + (size_t)b * 6;
  tb[0] = 1.0f / s; tb[1] = 0.0f; tb[2] = -tx / s; tb[3] = 0.0f; tb[4] = 1.0f / s; tb[5] = -ty / s;
  io.ss[(size_t)b * 3] = sl0;
  io.ss[(size_t)b * 3 + 1] = sl1;
  io.ss[(size_t)b * 3 + 2] = cl;
  io.scale[b] = s;
  io.shift[2 * b] = tx;
  io.shift[2 * b + 1] = ty;
  // z_pres (:604-620)
  const float eps = 1e-9f;
  const float noise = mog_logf(uu + eps) - mog_logf((1.0f - uu) + eps);
  const float y = (lo + noise) / cfg.temperature;
  float z = mog_sigmoidf(y);
  if (!cfg.train) z = rintf(z);
  const float zprob = mog_sigmoidf(lo);
  io.zprob[b] = zprob;
  // entropy regulariser (:660-668), every executed step
  float prn = 0.0f;
  if (cfg.g_num > 1e-8f) {
    const float ent = zprob * mog_softplusf(-1.0f * lo) + (1.0f - zprob) * mog_softplusf(lo);
    prn = ent * cfg.g_num;
  }
  // z_pres KL with the OLD stopping sum (:688-703)
  const bool act_old = stop_old < cfg.thr;
  const float zkl = concrete_kl(y, plo, cfg.temperature, lo, cfg.temperature);
  const float stop_new = stop_old + (1.0f - z);
  io.stop[b] = stop_new;
  const bool act = stop_new < cfg.thr;
  if (act) {
    io.digits[b] = dig + 1;
    io.live[cfg.step + 1] = 1;
  }
  // scale / shift KLs with the NEW stopping sum (:728-765)
  const float dc = cm - cfg.gcm;
  const float skl = 0.5f * ((((cfg.gclv - clv) - 1.0f) + cvar / cfg.gcvar) + (dc * dc) / cfg.gcvar);
  float shs = 0.0f;
  {
    const float gsm[2] = {gsm0, gsm1}, gslv[2] = {gslv0, gslv1};
    const float sm[2] = {sm0, sm1}, slv[2] = {slv0, slv1};
    for (int d = 0; d < 2; ++d) {
      const float gv = mog_expf(gslv[d]);
      const float svar = mog_expf(slv[d]);
      const float dd = sm[d] - gsm[d];
      shs = shs + ((((gslv[d] - slv[d]) - 1.0f) + svar / gv) + (dd * dd) / gv);
    }
  }
  io.zmask[b] = act ? 1.0f : 0.0f;
  io.zval[b] = z;
  io.zc[b] = act ? z : 0.0f;
  float* rr = io.rec;
  const float rv[Q_N] = {sm0, sm1, slv0, slv1, sl0, sl1, cm, clv, cl, s, tx, ty,
                         gsm0, gsm1, gslv0, gslv1, plo, lo, y, z,
                         act_old ? 1.0f : 0.0f, act ? 1.0f : 0.0f, live ? 1.0f : 0.0f,
                         act_old ? zkl : 0.0f, act ? skl : 0.0f, act ? 0.5f * shs : 0.0f,
                         live ? prn : 0.0f, zprob};
#pragma unroll
  for (int k = 0; k < Q_N; ++k) rr[(size_t)k * B + b] = rv[k];
}

struct AsrLossCfg {
  int B, T, C, nc, cons[8];
  float g_num, g_margin, g_element, g_bbox, g_size, g_area, area_min, area_max;
  float grad_scale, inv_batch_global;
};

__device__ __forceinline__ float recv(const float* rec, int t, int k, int B, int b) {
  return rec[((size_t)t * Q_N + k) * B + b];
}

__device__ __forceinline__ int executed_steps(const int* live, int T) {
  int n = 0;
  for (int t = 0; t < T; ++t) n += live[t] != 0;
  return n;
}

__device__ __forceinline__ float sigmoid_ce(float z, float x) {
#pragma clang fp contract(off)
  const float ax = x < 0.0f ? -x : x;
  return ((x > 0.0f ? x : 0.0f) - x * z) + mog_log1pf(mog_expf(-ax));
}

__device__ __forceinline__ float logit8(float p) {
#pragma clang fp contract(off)
  return mog_logf(p + 1e-8f) - mog_logf((1.0f - p) + 1e-8f);
}

// per image: KL sums (runloss for the reconstruction kernel) and the
// structural regularisers over the executed steps (:917-935, :1017-1069)
__global__ __launch_bounds__(256) void asr_terms_kernel(AsrLossCfg c, const float* rec,
                                                        const float* vkl, const float* zmask,
                                                        const int* live, float* klsum,
                                                        float* pr, float* area_o, float* out_o,
                                                        float* size_o, float* over_o) {
#pragma clang fp contract(off)
  const int b = blockIdx.x * 256 + threadIdx.x;
  const int B = c.B;
  if (b >= B) return;
  const int Tx = executed_steps(live, c.T);
  float zs = 0.0f, ss = 0.0f, hs = 0.0f, vs = 0.0f, ps = 0.0f;
  for (int t = 0; t < Tx; ++t) {
    zs = zs + recv(rec, t, Q_ZKL, B, b);
    ss = ss + recv(rec, t, Q_SKL, B, b);
    hs = hs + recv(rec, t, Q_SHKL, B, b);
    const size_t tb = (size_t)t * B + b;
    vs = vs + (zmask[tb] != 0.0f ? vkl[tb] : 0.0f);
    ps = ps + recv(rec, t, Q_PRN, B, b);
  }
  klsum[b] = (((0.0f + zs) + ss) + hs) + vs;
  const float C = (float)c.C;
  float area = 0.0f, outl = 0.0f, size = 0.0f, over = 0.0f;
  for (int t = 0; t < Tx; ++t) {
    const float sc = recv(rec, t, Q_S, B, b) * C;
    area = area + (fmaxf(c.area_max - sc, 0.0f) + fmaxf(sc - c.area_min, 0.0f));
  }
  area = Tx > 0 ? area / (float)Tx : 0.0f;
  for (int i = 0; i < Tx; ++i) {
    const float cxi = ((recv(rec, i, Q_TX, B, b) + 1.0f) * C) / 2.0f;
    const float cyi = ((recv(rec, i, Q_TY, B, b) + 1.0f) * C) / 2.0f;
    const float sci = recv(rec, i, Q_S, B, b) * C;
    const float mnx = cxi - 0.5f * sci, mny = cyi - 0.5f * sci;
    const float mxx = cxi + 0.5f * sci, mxy = cyi + 0.5f * sci;
    outl = outl + (((fmaxf(-1.0f * mnx, 0.0f) + fmaxf(-1.0f * mny, 0.0f)) + fmaxf(mxx - C, 0.0f)) +
                   fmaxf(mxy - C, 0.0f));
    for (int j = 0; j < Tx; ++j) {
      const float scj = recv(rec, j, Q_S, B, b) * C;
      size = size + fmaxf(fabsf(sci - scj) - 3.0f, 0.0f);
      const float cxj = ((recv(rec, j, Q_TX, B, b) + 1.0f) * C) / 2.0f;
      const float cyj = ((recv(rec, j, Q_TY, B, b) + 1.0f) * C) / 2.0f;
      const float md = fmaxf(fabsf(cxi - cxj), fabsf(cyi - cyj));
      const float smean = (sci + scj) / 2.0f;
      over = over + fmaxf(smean - md, 0.0f) * (i == j ? 0.0f : 1.0f);
    }
  }
  float p = 0.0f + ps;
  p = p + c.g_area * area;
  p = p + over * c.g_bbox;
  p = p + outl * c.g_bbox;
  p = p + size * c.g_size;
  pr[b] = p;
  area_o[b] = area;
  out_o[b] = outl;
  size_o[b] = size;
  over_o[b] = over;
}

// zsum[t] = sum_b z_pres_prob[t][b] (one block per step; the margin loss
// needs the batch mean, all-reduced over data-parallel ranks by the host)
__global__ __launch_bounds__(256) void asr_zprob_sum_kernel(int B, const float* rec, float* zsum) {
  __shared__ float red[4];
  const int t = blockIdx.x;
  float s = 0.0f;
  for (int b = threadIdx.x; b < B; b += 256) s += recv(rec, t, Q_ZPROB, B, b);
  s = mog_block_sum256(s, red);
  if (threadIdx.x == 0) zsum[t] = s;
}

__device__ __forceinline__ float margin_objective(const AsrLossCfg& c, int t) {
#pragma clang fp contract(off)
  float cnt = 0.0f;
  for (int k = 0; k < c.nc; ++k) cnt = cnt + (t < c.cons[k] ? 1.0f : 0.0f);
  return cnt / (float)c.nc;
}

// loss_b = (elbo_b + pr_b) + element_b in place (elbo_b = klsum_b + BCE_b from
// the reconstruction kernel); margin[0] (:970-1015, :1078-1079)
__global__ __launch_bounds__(256) void asr_finalize_kernel(AsrLossCfg c, const float* rec,
                                                           const int* live, const float* zsum,
                                                           const float* pr, float* loss,
                                                           float* element, float* margin) {
#pragma clang fp contract(off)
  const int b = blockIdx.x * 256 + threadIdx.x;
  const int B = c.B;
  const int Tx = executed_steps(live, c.T);
  if (b == 0) {
    float mg = 0.0f;
    if (c.g_margin > 1e-8f)
      for (int t = 0; t < Tx; ++t) {
        const float pm = zsum[t] * c.inv_batch_global;
        mg = mg + sigmoid_ce(margin_objective(c, t), logit8(pm)) * c.g_margin;
      }
    margin[0] = mg;
  }
  if (b >= B) return;
  float elem = 0.0f;
  if (c.g_margin > 1e-8f) {
    float best = 0.0f;
    for (int k = 0; k < c.nc; ++k) {
      float sum = 0.0f;
      for (int t = 0; t < Tx; ++t)
        sum = sum + sigmoid_ce(t < c.cons[k] ? 1.0f : 0.0f, logit8(recv(rec, t, Q_ZPROB, B, b)));
      best = k == 0 ? sum : fminf(best, sum);
    }
    elem = best * c.g_element;
  }
  element[b] = elem;
  loss[b] = (loss[b] + pr[b]) + elem;
}

// d(loss)/d(s, tx, ty, lo) of every executed step from the regularisers:
// entropy, area, bbox out / size / overlap (x grad_scale), element-wise
// number loss (x grad_scale) and the margin loss (x 1 / global batch: it is
// added outside the batch mean).  dreg [T][4][B].
__global__ __launch_bounds__(256) void asr_terms_bwd_kernel(AsrLossCfg c, const float* rec,
                                                            const int* live, const float* zsum,
                                                            float* dreg) {
#pragma clang fp contract(off)
  const int b = blockIdx.x * 256 + threadIdx.x;
  const int B = c.B;
  if (b >= B) return;
  const int Tx = executed_steps(live, c.T);
  const float C = (float)c.C, gL = c.grad_scale;
  float ds[8] = {0}, dx[8] = {0}, dy[8] = {0}, dp[8] = {0}, dl[8] = {0};
  float sc[8], cx[8], cy[8];
  for (int t = 0; t < Tx; ++t) {
    sc[t] = recv(rec, t, Q_S, B, b) * C;
    cx[t] = ((recv(rec, t, Q_TX, B, b) + 1.0f) * C) / 2.0f;
    cy[t] = ((recv(rec, t, Q_TY, B, b) + 1.0f) * C) / 2.0f;
  }
  // dsc / dcx / dcy accumulate in canvas units, converted at the end
  float dsc[8] = {0}, dcx[8] = {0}, dcy[8] = {0};
  if (Tx > 0) {
    const float ga = gL * c.g_area / (float)Tx;
    for (int t = 0; t < Tx; ++t)
      dsc[t] += ga * ((c.area_max - sc[t] >= 0.0f ? -1.0f : 0.0f) +
                      (sc[t] - c.area_min >= 0.0f ? 1.0f : 0.0f));
  }
  const float gb = gL * c.g_bbox, gs = gL * c.g_size;
  for (int i = 0; i < Tx; ++i) {
    const float mnx = cx[i] - 0.5f * sc[i], mny = cy[i] - 0.5f * sc[i];
    const float mxx = cx[i] + 0.5f * sc[i], mxy = cy[i] + 0.5f * sc[i];
    const float dmnx = -1.0f * mnx >= 0.0f ? -gb : 0.0f;
    const float dmny = -1.0f * mny >= 0.0f ? -gb : 0.0f;
    const float dmxx = mxx - C >= 0.0f ? gb : 0.0f;
    const float dmxy = mxy - C >= 0.0f ? gb : 0.0f;
    dcx[i] += dmnx + dmxx;
    dcy[i] += dmny + dmxy;
    dsc[i] += 0.5f * (dmxx + dmxy) - 0.5f * (dmnx + dmny);
    for (int j = 0; j < Tx; ++j) {
      const float d = sc[i] - sc[j];
      if (fabsf(d) - 3.0f >= 0.0f) {
        const float sg = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
        dsc[i] += gs * sg;
        dsc[j] -= gs * sg;
      }
      if (i == j) continue;
      const float ddx = cx[i] - cx[j], ddy = cy[i] - cy[j];
      const float ax = fabsf(ddx), ay = fabsf(ddy);
      const float md = fmaxf(ax, ay);
      const float smean = (sc[i] + sc[j]) / 2.0f;
      if (smean - md >= 0.0f) {
        dsc[i] += 0.5f * gb;
        dsc[j] += 0.5f * gb;
        if (ax >= ay) {
          const float sg = ddx > 0.0f ? 1.0f : (ddx < 0.0f ? -1.0f : 0.0f);
          dcx[i] -= gb * sg;
          dcx[j] += gb * sg;
        } else {
          const float sg = ddy > 0.0f ? 1.0f : (ddy < 0.0f ? -1.0f : 0.0f);
          dcy[i] -= gb * sg;
          dcy[j] += gb * sg;
        }
      }
    }
  }
  for (int t = 0; t < Tx; ++t) {
    ds[t] = dsc[t] * C;
    dx[t] = dcx[t] * C / 2.0f;
    dy[t] = dcy[t] * C / 2.0f;
  }
  // number losses through z_pres_prob = sigmoid(lo)
  if (c.g_margin > 1e-8f) {
    float sums[8];
    float best = 0.0f;
    for (int k = 0; k < c.nc; ++k) {
      float sum = 0.0f;
      for (int t = 0; t < Tx; ++t)
        sum = sum + sigmoid_ce(t < c.cons[k] ? 1.0f : 0.0f, logit8(recv(rec, t, Q_ZPROB, B, b)));
      sums[k] = sum;
      best = k == 0 ? sum : fminf(best, sum);
    }
    int ties = 0;
    for (int k = 0; k < c.nc; ++k) ties += sums[k] == best;
    const float ge = gL * c.g_element / (float)ties;
    for (int t = 0; t < Tx; ++t) {
      const float p = recv(rec, t, Q_ZPROB, B, b);
      const float x = logit8(p);
      const float dxdp = 1.0f / (p + 1e-8f) + 1.0f / ((1.0f - p) + 1e-8f);
      float g = 0.0f;
      for (int k = 0; k < c.nc; ++k)
        if (sums[k] == best) g += (mog_sigmoidf(x) - (t < c.cons[k] ? 1.0f : 0.0f)) * ge;
      const float pm = zsum[t] * c.inv_batch_global;
      const float xm = logit8(pm);
      const float dm = (mog_sigmoidf(xm) - margin_objective(c, t)) * c.g_margin *
                       (1.0f / (pm + 1e-8f) + 1.0f / ((1.0f - pm) + 1e-8f));
      dp[t] = g * dxdp + dm * c.inv_batch_global;
    }
  }
  for (int t = 0; t < Tx; ++t) {
    const float lo = recv(rec, t, Q_LO, B, b);
    const float p = recv(rec, t, Q_ZPROB, B, b);
    float d = dp[t] * p * (1.0f - p);
    if (c.g_num > 1e-8f) {
      const float ge = gL * c.g_num;
      const float A = mog_softplusf(-1.0f * lo), Bv = mog_softplusf(lo);
      d += ge * ((A - Bv) * p * (1.0f - p) - p * mog_sigmoidf(-lo) + (1.0f - p) * mog_sigmoidf(lo));
    }
    dl[t] = d;
  }
  for (int t = 0; t < c.T; ++t) {
    const bool e = t < Tx;
    float* o = dreg + (size_t)t * 4 * B;
    o[b] = e ? ds[t] : 0.0f;
    o[B + b] = e ? dx[t] : 0.0f;
    o[2 * B + b] = e ? dy[t] : 0.0f;
    o[3 * B + b] = e ? dl[t] : 0.0f;
  }
}

struct AsrBwdIO {
  const float* rec;          // [Q_N, B]
  const float* eps_shift;    // [B,2]
  const float* eps_scale;    // [B]
  const float* dtheta_fwd;   // [B,6] STN-read backward
  const float* dtheta_back;  // [B,6] STN-write backward (already scaled by active * z)
  const float* dot;          // [B] sum_p dcanvas * w
  const float* dreg;         // [4, B] regulariser gradients of this step
  const float* dss;          // [B,3] carry from the next step's LSTM inputs (or null)
  float* douts;              // [B, D_N]
  float* dpre[8];            // [B,64] pre-activation gradients of the hidden layers
};

// One wave per image: backward of asr_step_fwd_kernel.
__global__ __launch_bounds__(256) void asr_step_bwd_kernel(AsrCfg cfg, AsrW W, AsrHid hp,
                                                           AsrBwdIO io) {
#pragma clang fp contract(off)
  __shared__ float sv[4][16];
  const int m = threadIdx.x >> 6, q = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + m;
  const int B = cfg.B;
  const bool ok = b < B;
  const int bc = ok ? b : 0;
  const float* r = io.rec;
  auto R = [&](int k) { return r[(size_t)k * B + bc]; };
  const float gL = cfg.grad_scale, T = cfg.temperature;
  if (q == 0) {
    const float s = R(Q_S), tx = R(Q_TX), ty = R(Q_TY), z = R(Q_Z), y = R(Q_Y);
    const float lo = R(Q_LO), plo = R(Q_PLO), cm = R(Q_CM), clv = R(Q_CLV);
    const bool act_old = R(Q_ACT_OLD) != 0.0f, act = R(Q_ACT) != 0.0f;
    const float* dr = io.dtheta_fwd + (size_t)bc * 6;
    const float* dw = io.dtheta_back + (size_t)bc * 6;
    const float s2 = s * s;
    const float da = dw[0] + dw[4];
    const float ds = ((dr[0] + dr[4] + da * (-1.0f / s2)) + dw[2] * (tx / s2) + dw[5] * (ty / s2)) +
                     io.dreg[bc];
    const float dtx = (dr[2] - dw[2] / s) + io.dreg[B + bc];
    const float dty = (dr[5] - dw[5] / s) + io.dreg[2 * B + bc];
    // z_pres: canvas term (train model) + concrete KL vs the (learned) prior
    const float dz = act ? io.dot[bc] : 0.0f;
    float dy = cfg.train ? dz * z * (1.0f - z) : 0.0f;
    const float sq = mog_sigmoidf(-y * T + lo), sp = mog_sigmoidf(-y * T + plo);
    const float wz = act_old ? gL : 0.0f;
    dy += wz * (2.0f * T * (sq - sp));
    float dlo = wz * (1.0f - 2.0f * sq) + dy / T + io.dreg[3 * B + bc];
    const float dplo = cfg.fix_steps >= 0 ? 0.0f : wz * (2.0f * sp - 1.0f);
    // scale latent (carry: the next step's LSTM inputs see cl)
    const float wn = act ? gL : 0.0f;
    const float cvar = mog_expf(clv);
    const float dcl = ds * s * (1.0f - s) + (io.dss ? io.dss[(size_t)bc * 3 + 2] : 0.0f);
    const float dcm = dcl + wn * (cm - cfg.gcm) / cfg.gcvar;
    const float dclv = dcl * io.eps_scale[bc] * 0.5f * sqrtf(cvar) +
                       wn * 0.5f * (-1.0f + cvar / cfg.gcvar);
    sv[m][0] = dtx; sv[m][1] = dty; sv[m][2] = dlo; sv[m][3] = dplo;
    sv[m][4] = dcm; sv[m][5] = dclv; sv[m][6] = wn;
  }
  __syncthreads();
  // scale hidden layers: dpre6/7 and their contribution to the shift latent
  const size_t rq = (size_t)bc * HS + q;
  const float dcm = sv[m][4], dclv = sv[m][5];
  // operands loaded unconditionally (a load under the relu test compiles to
  // a branch with a vmcnt(0) wait inside); same arithmetic where h > 0
  const float w6 = W.w[W_IC1][q], w7 = W.w[W_IC3][q];
  const float d6 = hp.h[6][rq] > 0.0f ? dcm * w6 : 0.0f;
  const float d7 = hp.h[7][rq] > 0.0f ? dclv * w7 : 0.0f;
  if (ok) {
    io.dpre[6][rq] = d6;
    io.dpre[7][rq] = d7;
  }
  float p0 = d6 * W.w[W_IC0][256 * HS + q] + d7 * W.w[W_IC2][256 * HS + q];
  float p1 = d6 * W.w[W_IC0][257 * HS + q] + d7 * W.w[W_IC2][257 * HS + q];
  p0 = mog_wave_sum(p0);
  p1 = mog_wave_sum(p1);
  if (q == 0) {
    const float tx = R(Q_TX), ty = R(Q_TY), wn = sv[m][6];
    const float carry0 = io.dss ? io.dss[(size_t)bc * 3] : 0.0f;
    const float carry1 = io.dss ? io.dss[(size_t)bc * 3 + 1] : 0.0f;
    const float dsl[2] = {
        sv[m][0] * (1.0f - tx * tx) + carry0 + dcm * W.w[W_IC1][HS] + dclv * W.w[W_IC3][HS] + p0,
        sv[m][1] * (1.0f - ty * ty) + carry1 + dcm * W.w[W_IC1][HS + 1] +
            dclv * W.w[W_IC3][HS + 1] + p1};
    float o[D_N];
    for (int d = 0; d < 2; ++d) {
      const float sm = R(Q_SM0 + d), slv = R(Q_SLV0 + d);
      const float gsm = R(Q_GSM0 + d), gslv = R(Q_GSLV0 + d);
      const float svar = mog_expf(slv), gv = mog_expf(gslv);
      const float dd = sm - gsm;
      o[D_SM0 + d] = dsl[d] + wn * dd / gv;
      o[D_SLV0 + d] = dsl[d] * io.eps_shift[(size_t)bc * 2 + d] * 0.5f * sqrtf(svar) +
                      wn * 0.5f * (-1.0f + svar / gv);
      o[D_GSM0 + d] = -wn * dd / gv;
      o[D_GSLV0 + d] = wn * 0.5f * ((1.0f - svar / gv) - (dd * dd) / gv);
    }
    o[D_LO] = sv[m][2];
    o[D_PLO] = sv[m][3];
    o[D_CM] = dcm;
    o[D_CLV] = dclv;
    for (int k = 0; k < D_N; ++k)
      if (ok) io.douts[(size_t)bc * D_N + k] = o[k];
    sv[m][0] = o[D_SM0]; sv[m][1] = o[D_SM1]; sv[m][2] = o[D_SLV0]; sv[m][3] = o[D_SLV1];
    sv[m][8] = o[D_LO]; sv[m][9] = o[D_GSM0]; sv[m][10] = o[D_GSM1];
    sv[m][11] = o[D_GSLV0]; sv[m][12] = o[D_GSLV1]; sv[m][13] = o[D_PLO];
  }
  __syncthreads();
  if (!ok) return;
  const float* v = sv[m];
  // every operand loaded before the first store (unconditionally, see above)
  float hv[6], wa[6], wb[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) hv[k] = hp.h[k][rq];
  hv[5] = hp.h[5] ? hp.h[5][rq] : 0.0f;
  wa[0] = W.w[W_IS1][2 * q]; wb[0] = W.w[W_IS1][2 * q + 1];
  wa[1] = W.w[W_IS3][2 * q]; wb[1] = W.w[W_IS3][2 * q + 1];
  wa[2] = W.w[W_ZL1][q];
  wa[3] = W.w[W_GS1][2 * q]; wb[3] = W.w[W_GS1][2 * q + 1];
  wa[4] = W.w[W_GS3][2 * q]; wb[4] = W.w[W_GS3][2 * q + 1];
  wa[5] = W.w[W_ZP1][q];
  io.dpre[0][rq] = hv[0] > 0.0f ? v[0] * wa[0] + v[1] * wb[0] : 0.0f;
  io.dpre[1][rq] = hv[1] > 0.0f ? v[2] * wa[1] + v[3] * wb[1] : 0.0f;
  io.dpre[2][rq] = hv[2] > 0.0f ? v[8] * wa[2] : 0.0f;
  io.dpre[3][rq] = hv[3] > 0.0f ? v[9] * wa[3] + v[10] * wb[3] : 0.0f;
  io.dpre[4][rq] = hv[4] > 0.0f ? v[11] * wa[4] + v[12] * wb[4] : 0.0f;
  if (io.dpre[5]) io.dpre[5][rq] = (hp.h[5] && hv[5] > 0.0f) ? v[13] * wa[5] : 0.0f;
}

}  // namespace

extern "C" int mog_asr_pack(int B, int Z, int H, int ld, const float* z, const float* ss,
                            const float* h, float* out, const float* h2, float* out2,
                            void* stream) {
  MOG_CHECK_ARG(B >= 0 && Z > 0 && H > 0 && ld >= Z + 3 + H && out);
  if (B == 0) return 0;
  const long n = (long)B * ld * (out2 ? 2 : 1);
  asr_pack_kernel<<<mog_cdiv(n, 256), 256, 0, mog_stream(stream)>>>(B, Z, H, ld, z, ss, h, out, h2,
                                                                   out2);
  MOG_LAUNCH_RET();
}

extern "C" int mog_asr_unpack(int B, int Z, int H, int ld, const float* dU, const float* dUg,
                              float* dz, float* dss, float* dh, float* dhg, int acc_dz,
                              void* stream) {
  MOG_CHECK_ARG(B >= 0 && Z > 0 && H > 0 && ld >= Z + 3 + H && dU && dUg && dz && dss && dh &&
                dhg);
  if (B == 0) return 0;
  asr_unpack_kernel<<<mog_cdiv((long)B * (Z + 3 + H), 256), 256, 0, mog_stream(stream)>>>(
      B, Z, H, ld, dU, dUg, dz, dss, dh, dhg, acc_dz, 1, 0);
  MOG_LAUNCH_RET();
}

extern "C" int mog_asr_unpack_parts(int B, int Z, int H, int ld, const float* dU,
                                    const float* dUg, int nparts, long part_stride, float* dz,
                                    float* dss, float* dh, float* dhg, int acc_dz,
                                    void* stream) {
  MOG_CHECK_ARG(B >= 0 && Z > 0 && H > 0 && ld >= Z + 3 + H && dU && dUg && dz && dss && dh &&
                dhg && nparts >= 1 && nparts <= 4 && (nparts == 1 || part_stride >= (long)B * ld));
  if (B == 0) return 0;
  asr_unpack_kernel<<<mog_cdiv((long)B * (Z + 3 + H), 256), 256, 0, mog_stream(stream)>>>(
      B, Z, H, ld, dU, dUg, dz, dss, dh, dhg, acc_dz, nparts, part_stride);
  MOG_LAUNCH_RET();
}

static int fill_w(AsrW& W, const float* const* w) {
  for (int i = 0; i < W_N; ++i) {
    if (!w[i]) return 0;
    W.w[i] = w[i];
  }
  return 1;
}

extern "C" int mog_asr_step_forward(int B, int step, int train, int fix_steps, float thr,
                                    float temperature, float scale_prior_mean,
                                    float scale_prior_var, float scale_prior_logvar,
                                    float gamma_num, const float* const* w, float* const* hid,
                                    const float* eps_shift, const float* eps_scale,
                                    const float* u, float* stop, int* digits, int* live,
                                    float* rec, float* theta_fwd, float* theta_back, float* ss,
                                    float* scale, float* shift, float* zprob, float* zmask,
                                    float* zval, float* zc, void* stream) {
  MOG_CHECK_ARG(B >= 0 && w && hid && eps_shift && eps_scale && u && stop && digits && live);
  MOG_CHECK_ARG(rec && theta_fwd && theta_back && ss && scale && shift && zprob && zmask && zval &&
                zc);
  if (B == 0) return 0;
  AsrCfg c{B, step, train, fix_steps, thr, temperature, scale_prior_mean, scale_prior_var,
           scale_prior_logvar, gamma_num, 0.0f};
  AsrW W;
  MOG_CHECK_ARG(fill_w(W, w));
  AsrHid hp;
  for (int i = 0; i < 8; ++i) {
    MOG_CHECK_ARG(hid[i] || (i == 5 && fix_steps >= 0));
    hp.h[i] = hid[i];
  }
  AsrFwdIO io{eps_shift, eps_scale, u,     stop,  digits, live, rec, theta_fwd, theta_back,
              ss,        scale,     shift, zprob, zmask, zval,   zc};
  asr_step_fwd_kernel<<<mog_cdiv(B, 4), 256, 0, mog_stream(stream)>>>(c, W, hp, io);
  MOG_LAUNCH_RET();
}

static int fill_loss_cfg(AsrLossCfg& c, int B, int T, int C, int nc, const int* cons,
                         const float* gammas, float grad_scale, float inv_batch_global) {
  if (nc < 1 || nc > 8 || !cons || !gammas || T > 8) return 0;
  c.B = B; c.T = T; c.C = C; c.nc = nc;
  for (int i = 0; i < 8; ++i) c.cons[i] = i < nc ? cons[i] : 0;
  c.g_num = gammas[0]; c.g_margin = gammas[1]; c.g_element = gammas[2]; c.g_bbox = gammas[3];
  c.g_size = gammas[4]; c.g_area = gammas[5]; c.area_min = gammas[6]; c.area_max = gammas[7];
  c.grad_scale = grad_scale; c.inv_batch_global = inv_batch_global;
  return 1;
}

extern "C" int mog_asr_terms(int B, int T, int C, int nc, const int* cons, const float* gammas,
                             const float* rec, const float* vkl, const float* zmask,
                             const int* live, float* klsum, float* pr, float* area, float* out,
                             float* size, float* overlap, float* zsum, void* stream) {
  MOG_CHECK_ARG(B >= 0 && T >= 1 && rec && vkl && zmask && live && klsum && pr && area && out &&
                size && overlap && zsum);
  AsrLossCfg c;
  MOG_CHECK_ARG(fill_loss_cfg(c, B, T, C, nc, cons, gammas, 0.0f, 0.0f));
  if (B == 0) return 0;
  asr_terms_kernel<<<mog_cdiv(B, 256), 256, 0, mog_stream(stream)>>>(c, rec, vkl, zmask, live,
                                                                     klsum, pr, area, out, size,
                                                                     overlap);
  asr_zprob_sum_kernel<<<T, 256, 0, mog_stream(stream)>>>(B, rec, zsum);
  MOG_LAUNCH_RET();
}

extern "C" int mog_asr_finalize(int B, int T, int C, int nc, const int* cons,
                                const float* gammas, float inv_batch_global, const float* rec,
                                const int* live, const float* zsum, const float* pr, float* loss,
                                float* element, float* margin, void* stream) {
  MOG_CHECK_ARG(B >= 0 && T >= 1 && rec && live && zsum && pr && loss && element && margin);
  AsrLossCfg c;
  MOG_CHECK_ARG(fill_loss_cfg(c, B, T, C, nc, cons, gammas, 0.0f, inv_batch_global));
  asr_finalize_kernel<<<mog_cdiv(B > 0 ? B : 1, 256), 256, 0, mog_stream(stream)>>>(
      c, rec, live, zsum, pr, loss, element, margin);
  MOG_LAUNCH_RET();
}

extern "C" int mog_asr_terms_backward(int B, int T, int C, int nc, const int* cons,
                                      const float* gammas, float grad_scale,
                                      float inv_batch_global, const float* rec, const int* live,
                                      const float* zsum, float* dreg, void* stream) {
  MOG_CHECK_ARG(B >= 0 && T >= 1 && rec && live && zsum && dreg);
  AsrLossCfg c;
  MOG_CHECK_ARG(fill_loss_cfg(c, B, T, C, nc, cons, gammas, grad_scale, inv_batch_global));
  if (B == 0) return 0;
  asr_terms_bwd_kernel<<<mog_cdiv(B, 256), 256, 0, mog_stream(stream)>>>(c, rec, live, zsum, dreg);
  MOG_LAUNCH_RET();
}

extern "C" int mog_asr_step_backward(int B, int train, int fix_steps, float temperature,
                                     float scale_prior_mean, float scale_prior_var,
                                     float grad_scale, const float* const* w,
                                     float* const* hid, const float* rec, const float* eps_shift,
                                     const float* eps_scale, const float* dtheta_fwd,
                                     const float* dtheta_back, const float* dot,
                                     const float* dreg, const float* dss, float* douts,
                                     float* const* dpre, void* stream) {
  MOG_CHECK_ARG(B >= 0 && w && hid && rec && eps_shift && eps_scale && dtheta_fwd && dtheta_back);
  MOG_CHECK_ARG(dot && dreg && douts && dpre);
  if (B == 0) return 0;
  AsrCfg c{B, 0, train, fix_steps, 0.0f, temperature, scale_prior_mean, scale_prior_var, 0.0f,
           0.0f, grad_scale};
  AsrW W;
  MOG_CHECK_ARG(fill_w(W, w));
  AsrHid hp;
  AsrBwdIO io;
  io.rec = rec; io.eps_shift = eps_shift; io.eps_scale = eps_scale; io.dtheta_fwd = dtheta_fwd;
  io.dtheta_back = dtheta_back; io.dot = dot; io.dreg = dreg; io.dss = dss; io.douts = douts;
  for (int i = 0; i < 8; ++i) {
    MOG_CHECK_ARG((hid[i] && dpre[i]) || (i == 5 && fix_steps >= 0));
    hp.h[i] = hid[i];
    io.dpre[i] = dpre[i];
  }
  asr_step_bwd_kernel<<<mog_cdiv(B, 4), 256, 0, mog_stream(stream)>>>(c, W, hp, io);
  MOG_LAUNCH_RET();
}
