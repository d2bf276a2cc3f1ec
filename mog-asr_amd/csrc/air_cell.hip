// Per-object-step cell kernels of the AIR loop (air/air_model.py:435-736) and
// the reconstruction loss (:866-900), forward and backward, for gfx950.
//
// The GEMM-shaped pieces (LSTM x/h projections, head hidden layers, VAE
// layers) run on the MFMA GEMM (gemm_f32.hip / vae_fused.hip); what remains
// per step is O(B) scalar logic and O(B*H) gate elementwise work, fused here:
//   lstm_gates_fwd/bwd   BasicLSTMCell gates (TF-1.12, i,j,f,o, forget_bias 1)
//   step_scalars_fwd     head output layers (k-ordered fma chains), Gaussian
//                        sampling of scale/shift (:458-498, _sample_from_mvn
//                        :186-192), theta / theta^-1 (:500-577), concrete
//                        z_pres sample (concrete.py:20-27) + KL (:30-64),
//                        stopping sum / digit count / live flag (:428-432,
//                        :644-663), scale & shift KLs (:677-705)
//   step_scalars_bwd     the matching hand-derived backward
//   vae_sample_fwd/bwd   z = mu + eps sqrt(exp(lv)) (vae.py:27-30) + VAE KL
//                        (air_model.py:718-736)
//   recon_loss           clip, BCE, MSE, per-image loss, dL/dcanvas (:866-900)
#include <algorithm>

#include "mog_common.h"

namespace {

// ------------------------------------------------------------------ LSTM ---
// G: [B, 4H] pre-activation (i, j, f, o); bias added here when `bias` != null
// (step 0, where the h-projection of the zero state is skipped).
struct LstmFwd {
  const float* G;
  const float* bias;
  const float* c_prev;
  float* c_out;
  float* h_out;
};

__device__ __forceinline__ void lstm_fwd_body(const LstmFwd& a, int B, int H, long idx) {
#pragma clang fp contract(off)
  if (idx >= (long)B * H) return;
  const int b = idx / H, u = idx - (long)b * H;
  const float* g = a.G + (size_t)b * 4 * H;
  float gi = g[u], gj = g[H + u], gf = g[2 * H + u], go = g[3 * H + u];
  if (a.bias) {
    const float* bias = a.bias;
    gi = gi + bias[u]; gj = gj + bias[H + u]; gf = gf + bias[2 * H + u]; go = go + bias[3 * H + u];
  }
  const float c0 = a.c_prev ? a.c_prev[idx] : 0.0f;
  const float nc = c0 * mog_sigmoidf(gf + 1.0f) + mog_sigmoidf(gi) * mog_tanhf(gj);
  a.c_out[idx] = nc;
  a.h_out[idx] = mog_tanhf(nc) * mog_sigmoidf(go);
}

__global__ __launch_bounds__(256) void lstm_fwd_kernel(const LstmFwd a, int B, int H) {
  lstm_fwd_body(a, B, H, (long)blockIdx.x * 256 + threadIdx.x);
}

// two independent cells of one batch (AIR-ASR's inference and generative
// LSTMCells), blockIdx.y picking the cell: one launch per step instead of two
__global__ __launch_bounds__(256) void lstm_fwd_pair_kernel(const LstmFwd a0, const LstmFwd a1,
                                                            int B, int H) {
  lstm_fwd_body(blockIdx.y ? a1 : a0, B, H, (long)blockIdx.x * 256 + threadIdx.x);
}

// dh, dc (incoming) -> dG [B,4H], dc_prev [B,H]; dGsum += dG (sum over steps
// for the hoisted x-projection gradient).
struct LstmBwd {
  const float* G;
  const float* bias;
  const float* c_prev;
  const float* c_cur;
  const float* dh;
  const float* dc;
  float* dG;
  float* dc_prev;
  float* dGsum;
  // dh += parts[0] + parts[1] + ... (nparts K-slices of the hidden-state
  // gradient GEMM, part_stride elements apart), added in part order
  const float* dh_parts = nullptr;
  int nparts = 0;
  long part_stride = 0;
};

__device__ __forceinline__ void lstm_bwd_body(const LstmBwd& a, int B, int H, long idx) {
  if (idx >= (long)B * H) return;
  const int b = idx / H, u = idx - (long)b * H;
  const float* g = a.G + (size_t)b * 4 * H;
  // every load up front and unconditional, the optional operands read
  // through a valid stand-in pointer and selected away (a load under `p ? ..`
  // compiles to a branch with a vmcnt(0) wait inside; the dGsum loads would
  // otherwise wait behind the dG stores, which the compiler must assume alias)
  const float* bp = a.bias ? a.bias : a.G;
  const float* cp = a.c_prev ? a.c_prev : a.c_cur;
  const float* dp = a.dc ? a.dc : a.dh;
  float* sp = a.dGsum ? a.dGsum + (size_t)b * 4 * H : a.dG + (size_t)b * 4 * H;
  float gi = g[u], gj = g[H + u], gf = g[2 * H + u], go = g[3 * H + u];
  const float bi = bp[u], bj = bp[H + u], bf = bp[2 * H + u], bo = bp[3 * H + u];
  const float cpv = cp[idx], ctv = a.c_cur[idx], dcv = dp[idx];
  float dhv = a.dh[idx];
  if (a.nparts > 0) {
    float pv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pv[j] = j < a.nparts ? a.dh_parts[j * a.part_stride + idx] : 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < a.nparts) dhv = dhv + pv[j];
  }
  const float s0 = sp[u], s1 = sp[H + u], s2 = sp[2 * H + u], s3 = sp[3 * H + u];
  if (a.bias) {
    gi = gi + bi; gj = gj + bj; gf = gf + bf; go = go + bo;
  }
  const float si = mog_sigmoidf(gi), tj = mog_tanhf(gj), sf = mog_sigmoidf(gf + 1.0f);
  const float so = mog_sigmoidf(go);
  const float c0 = a.c_prev ? cpv : 0.0f;
  const float tc = mog_tanhf(ctv);
  const float dct = (a.dc ? dcv : 0.0f) + dhv * so * (1.0f - tc * tc);
  const float dgo = dhv * tc * so * (1.0f - so);
  const float dgf = dct * c0 * sf * (1.0f - sf);
  const float dgi = dct * tj * si * (1.0f - si);
  const float dgj = dct * si * (1.0f - tj * tj);
  float* d = a.dG + (size_t)b * 4 * H;
  d[u] = dgi; d[H + u] = dgj; d[2 * H + u] = dgf; d[3 * H + u] = dgo;
  if (a.dGsum) {
    sp[u] = s0 + dgi; sp[H + u] = s1 + dgj; sp[2 * H + u] = s2 + dgf; sp[3 * H + u] = s3 + dgo;
  }
  if (a.dc_prev) a.dc_prev[idx] = dct * sf;
}

__global__ __launch_bounds__(256) void lstm_bwd_kernel(const LstmBwd a, int B, int H) {
  lstm_bwd_body(a, B, H, (long)blockIdx.x * 256 + threadIdx.x);
}

__global__ __launch_bounds__(256) void lstm_bwd_pair_kernel(const LstmBwd a0, const LstmBwd a1,
                                                            int B, int H) {
  lstm_bwd_body(blockIdx.y ? a1 : a0, B, H, (long)blockIdx.x * 256 + threadIdx.x);
}

// -------------------------------------------------------- step scalars ---
struct StepCfg {
  int B, H, HS, HZ, train, use_num_prior, step;
  float thr, temperature, prior_lo, prior_bias;
  float s_pm, s_pv, s_plv, h_pm, h_pv, h_plv;
  float grad_scale;  // dL/d(per-image loss) = 1/B_global
  // when set, the z_pres prior log-odds is read from device memory instead of
  // prior_lo (the annealed value of a captured step changes every replay)
  const float* prior_lo_dev;
};

__device__ __forceinline__ float prior_log_odds(const StepCfg& c) {
  return c.prior_lo_dev ? *c.prior_lo_dev : c.prior_lo;
}

// record slots [NREC][B] per step
enum {
  R_SM, R_SLV, R_HM0, R_HM1, R_HLV0, R_HLV1, R_LO, R_S, R_TX, R_TY, R_Y, R_Z,
  R_ACT_OLD, R_ACT, R_LIVE, R_ZC, R_ZTERM, R_NREC
};

struct HeadPtrs {
  const float* hid[5];  // post-relu hidden [B, HS] for sm, slv, hm, hlv, lo
  const float* w2[5];   // [HS, k]
  const float* b2[5];   // [k]
};

// sum_k a[k] w[k ldw] as ONE fma chain in k order (the oracle's dense()).
// The operands of 32 k-steps are loaded before their fmas: a rolled
// load-then-fma loop paid one memory round trip per k (16 us per launch at
// the reference's batch of 64, where the step kernel is one or two
// workgroups); same fma sequence, same bits.
__device__ __forceinline__ float chain_dot(const float* a, const float* w, int K, int ldw) {
#pragma clang fp contract(off)
  constexpr int KB = 32;
  float acc = 0.0f;
  int k = 0;
  for (; k + KB <= K; k += KB) {
    float av[KB], wv[KB];
#pragma unroll
    for (int i = 0; i < KB; ++i) {
      av[i] = a[k + i];
      wv[i] = w[(size_t)(k + i) * ldw];
    }
#pragma unroll
    for (int i = 0; i < KB; ++i) acc = fmaf(av[i], wv[i], acc);
  }
  for (; k < K; ++k) acc = fmaf(a[k], w[(size_t)k * ldw], acc);
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

__device__ __forceinline__ float gauss_kl_term(float plv, float lv, float var, float pv,
                                               float mean, float pm) {
#pragma clang fp contract(off)
  const float d = mean - pm;
  return (((plv - lv) - 1.0f) + var / pv) + (d * d) / pv;
}

struct StepFwdIO {
  const float* eps_scale;  // [B]
  const float* eps_shift;  // [B,2]
  const float* u;          // [B]
  float* stop;             // [B] state
  float* runloss;          // [B] state
  int* digits;             // [B] state
  int* live;               // [T+1] flags; live[step] read, live[step+1] set
  float* rec;              // [R_NREC, B] records for this step
  float* theta_fwd;        // [B,6]
  float* theta_back;       // [B,6]
  float* scale_out;        // [B]
  float* shift_out;        // [B,2]
  float* zprob_out;        // [B]
  float* zkl_out;          // [B]
  float* skl_out;          // [B]
  float* shkl_out;         // [B]
  float* zmask;            // [B] active (canvas mask)
  float* zval;             // [B] z_pres value (canvas coefficient)
  float* zc;               // [B] active ? z : 0 (STN-write backward scale; may be null)
};

// 8 lanes per image: lanes 0..6 each evaluate one head-output fma chain
// (scale-mean, scale-logvar, shift-mean x/y, shift-logvar x/y, z_pres
// log-odds), lane 0 then runs the scalar step logic.
__global__ __launch_bounds__(256) void step_fwd_kernel(StepCfg cfg, HeadPtrs hp, StepFwdIO io) {
#pragma clang fp contract(off)
  const int B = cfg.B;
  const int b = blockIdx.x * 32 + (threadIdx.x >> 3);
  const int j = threadIdx.x & 7;
  const int HS = cfg.HS, HZ = cfg.HZ;
  // lane -> (head, output column, width of that head's output)
  const int head = j == 0 ? 0 : j == 1 ? 1 : j <= 3 ? 2 : j <= 5 ? 3 : 4;
  const int col = (j == 3 || j == 5) ? 1 : 0;
  const int kw = (head == 2 || head == 3) ? 2 : 1;
  // every per-image input loaded up front, before the head dot chains (from
  // a clamped image index, by every lane): the outputs below are stores
  // through pointers the compiler must assume may alias them, so a load
  // issued after a store waits for it, and loads behind the dot chains and the
  // early return would add a memory round trip after them -- at small batches
  // (one or two workgroups) those round trips are the kernel's time
  const int bc = min(b, B - 1);
  const float e_s = io.eps_scale[bc], e_h0 = io.eps_shift[2 * bc], e_h1 = io.eps_shift[2 * bc + 1];
  const float uu = io.u[bc];
  const int live = io.live[cfg.step];
  const float stop_old = io.stop[bc];
  const float rl0 = io.runloss[bc];
  const int dig = io.digits[bc];
  float v = 0.0f;
  if (b < B && j < 7) {
    const int K = head == 4 ? HZ : HS;
    v = chain_dot(hp.hid[head] + (size_t)b * K, hp.w2[head] + col, K, kw) + hp.b2[head][col];
  }
  const float sm = __shfl(v, 0, 8), slv = __shfl(v, 1, 8);
  const float hm0 = __shfl(v, 2, 8), hm1 = __shfl(v, 3, 8);
  const float hv0 = __shfl(v, 4, 8), hv1 = __shfl(v, 5, 8);
  const float lo = __shfl(v, 6, 8);
  if (b >= B || j != 0) return;

  // scale / shift sampling (air_model.py:471-477, :492-498; :186-192)
  const float svar = mog_expf(slv);
  const float s = mog_sigmoidf(sm + e_s * sqrtf(svar));
  const float hvar0 = mog_expf(hv0), hvar1 = mog_expf(hv1);
  const float tx = mog_tanhf(hm0 + e_h0 * sqrtf(hvar0));
  const float ty = mog_tanhf(hm1 + e_h1 * sqrtf(hvar1));
  float* tf = io.theta_fwd + (size_t)b * 6;
  tf[0] = s; tf[1] = 0.0f; tf[2] = tx; tf[3] = 0.0f; tf[4] = s; tf[5] = ty;
  const float is = 1.0f / s;
  float* tb = io.theta_back + (size_t)b * 6;
  tb[0] = is; tb[1] = 0.0f; tb[2] = -tx / s; tb[3] = 0.0f; tb[4] = is; tb[5] = -ty / s;
  io.scale_out[b] = s;
  io.shift_out[2 * b] = tx;
  io.shift_out[2 * b + 1] = ty;

  // z_pres (air_model.py:590-620, concrete.py:20-27)
  const float eps = 1e-9f;
  const float noise = mog_logf(uu + eps) - mog_logf((1.0f - uu) + eps);
  const float y = (lo + noise) / cfg.temperature;
  float z = mog_sigmoidf(y);
  if (!cfg.train) z = rintf(z);
  io.zprob_out[b] = mog_sigmoidf(lo);

  // z_pres KL with the OLD stopping sum (:622-653)
  float kl_end = 0.0f;
  if (cfg.use_num_prior) kl_end = concrete_kl(y, -100.0f, cfg.temperature, lo, cfg.temperature);
  const float zkl = concrete_kl(y, prior_log_odds(cfg) + cfg.prior_bias, cfg.temperature, lo,
                                cfg.temperature);
  const bool act_old = stop_old < cfg.thr;
  float rl = rl0;
  // the z_pres term this step adds (recorded: mog_air_runloss replays the sum)
  const float zterm = live ? (act_old ? zkl : kl_end) : 0.0f;
  if (live) rl = rl + zterm;
  io.zkl_out[b] = zkl;

  // stopping sum, digit count, live flag for the next step (:428-432, :659-663)
  const float stop_new = stop_old + (1.0f - z);
  io.stop[b] = stop_new;
  const bool act = stop_new < cfg.thr;
  if (act) {
    io.digits[b] = dig + 1;
    io.live[cfg.step + 1] = 1;
  }

  // scale & shift KLs with the NEW stopping sum (:677-705)
  const float skl = 0.5f * gauss_kl_term(cfg.s_plv, slv, svar, cfg.s_pv, sm, cfg.s_pm);
  if (act) rl = rl + skl;
  const float shs = gauss_kl_term(cfg.h_plv, hv0, hvar0, cfg.h_pv, hm0, cfg.h_pm) +
                    gauss_kl_term(cfg.h_plv, hv1, hvar1, cfg.h_pv, hm1, cfg.h_pm);
  const float shkl = 0.5f * shs;
  if (act) rl = rl + shkl;
  io.runloss[b] = rl;
  io.skl_out[b] = skl;
  io.shkl_out[b] = shkl;
  io.zmask[b] = act ? 1.0f : 0.0f;
  io.zval[b] = z;

  float* r = io.rec;
  r[R_SM * B + b] = sm; r[R_SLV * B + b] = slv;
  r[R_HM0 * B + b] = hm0; r[R_HM1 * B + b] = hm1;
  r[R_HLV0 * B + b] = hv0; r[R_HLV1 * B + b] = hv1;
  r[R_LO * B + b] = lo; r[R_S * B + b] = s; r[R_TX * B + b] = tx; r[R_TY * B + b] = ty;
  r[R_Y * B + b] = y; r[R_Z * B + b] = z;
  r[R_ACT_OLD * B + b] = act_old ? 1.0f : 0.0f;
  r[R_ACT * B + b] = act ? 1.0f : 0.0f;
  r[R_LIVE * B + b] = live ? 1.0f : 0.0f;
  r[R_ZC * B + b] = act ? z : 0.0f;
  r[R_ZTERM * B + b] = zterm;
  if (io.zc) io.zc[b] = act ? z : 0.0f;
}

// Every loop step of the batch in ONE launch (AIR: the heads read h_t only --
// the step's VAE never feeds the recurrence -- so once the LSTM chain has run,
// every step's head outputs are available and only the per-image loop state
// is sequential).  Operands of step t at step-0 pointer + t * (B * width);
// the step values are the ones step_fwd_kernel computes, in the same order.
// What depends on the batch-wide loop predicate is NOT resolved here: live[t]
// is known only once every image of step t - 1 (and every rank, under data
// parallelism) has run, so rec[R_ZTERM] holds the z_pres term the step adds
// IF it is live (act_old ? zkl : kl_end), rec[R_LIVE] 1, and runloss is not
// touched: mog_air_runloss with `live` applies the predicate and replays the
// running loss (runloss_kernel), which gives the bits of T single-step
// launches.  Lanes: 8 per loop step (lanes 0..6 one head-output chain each),
// LPI = 8 * steps rounded to a power of two per image; every step's state-free
// values (sampling, theta, z_pres, KLs) in lane 0 of its group at once; lane 0
// of the image then walks the steps for the stopping sum, counts, masks.
constexpr int MAX_STEPS_FWD = 8;
struct StepsFwdIO {
  StepFwdIO s;       // step-0 pointers (runloss unused)
  long hid_step;     // elements between two steps' rows of one head's hidden layer
  int steps;
  float prior_bias[MAX_STEPS_FWD];
};

template <int LPI>
__global__ __launch_bounds__(256) void step_fwd_steps_kernel(StepCfg cfg, HeadPtrs hp,
                                                             StepsFwdIO q) {
#pragma clang fp contract(off)
  constexpr int IPB = 256 / LPI;  // images per block
  const int B = cfg.B, T = q.steps;
  const StepFwdIO& io = q.s;
  const int b = blockIdx.x * IPB + threadIdx.x / LPI;
  const int li = threadIdx.x % LPI;
  const int t = li >> 3, j = li & 7, g0 = li & ~7;
  const int head = j == 0 ? 0 : j == 1 ? 1 : j <= 3 ? 2 : j <= 5 ? 3 : 4;
  const int col = (j == 3 || j == 5) ? 1 : 0;
  const int kw = (head == 2 || head == 3) ? 2 : 1;
  const int bc = min(b, B - 1), tc = min(t, T - 1);
  const long rb = (long)tc * B + bc;  // row of (step tc, image bc)
  // every input up front (see step_fwd_kernel)
  const float e_s = io.eps_scale[rb], e_h0 = io.eps_shift[2 * rb], e_h1 = io.eps_shift[2 * rb + 1];
  const float uu = io.u[rb];
  const float stop0 = io.stop[bc];
  const int dig0 = io.digits[bc];
  const float pbias = q.prior_bias[tc];
  float v = 0.0f;
  if (b < B && t < T && j < 7) {
    const int K = head == 4 ? cfg.HZ : cfg.HS;
    v = chain_dot(hp.hid[head] + tc * q.hid_step + (size_t)bc * K, hp.w2[head] + col, K, kw) +
        hp.b2[head][col];
  }
  const float sm = __shfl(v, g0, LPI), slv = __shfl(v, g0 + 1, LPI);
  const float hm0 = __shfl(v, g0 + 2, LPI), hm1 = __shfl(v, g0 + 3, LPI);
  const float hv0 = __shfl(v, g0 + 4, LPI), hv1 = __shfl(v, g0 + 5, LPI);
  const float lo = __shfl(v, g0 + 6, LPI);

  // the step's state-free values, as step_fwd_kernel computes them
  const float svar = mog_expf(slv);
  const float s = mog_sigmoidf(sm + e_s * sqrtf(svar));
  const float hvar0 = mog_expf(hv0), hvar1 = mog_expf(hv1);
  const float tx = mog_tanhf(hm0 + e_h0 * sqrtf(hvar0));
  const float ty = mog_tanhf(hm1 + e_h1 * sqrtf(hvar1));
  const float eps = 1e-9f;
  const float noise = mog_logf(uu + eps) - mog_logf((1.0f - uu) + eps);
  const float y = (lo + noise) / cfg.temperature;
  float z = mog_sigmoidf(y);
  if (!cfg.train) z = rintf(z);
  float kl_end = 0.0f;
  if (cfg.use_num_prior) kl_end = concrete_kl(y, -100.0f, cfg.temperature, lo, cfg.temperature);
  const float zkl = concrete_kl(y, prior_log_odds(cfg) + pbias, cfg.temperature, lo,
                                cfg.temperature);
  const float skl = 0.5f * gauss_kl_term(cfg.s_plv, slv, svar, cfg.s_pv, sm, cfg.s_pm);
  const float shs = gauss_kl_term(cfg.h_plv, hv0, hvar0, cfg.h_pv, hm0, cfg.h_pm) +
                    gauss_kl_term(cfg.h_plv, hv1, hvar1, cfg.h_pv, hm1, cfg.h_pm);
  const float shkl = 0.5f * shs;
  if (b < B && t < T && j == 0) {
    float* tf = io.theta_fwd + rb * 6;
    tf[0] = s; tf[1] = 0.0f; tf[2] = tx; tf[3] = 0.0f; tf[4] = s; tf[5] = ty;
    const float is = 1.0f / s;
    float* tb = io.theta_back + rb * 6;
    tb[0] = is; tb[1] = 0.0f; tb[2] = -tx / s; tb[3] = 0.0f; tb[4] = is; tb[5] = -ty / s;
    io.scale_out[rb] = s;
    io.shift_out[2 * rb] = tx;
    io.shift_out[2 * rb + 1] = ty;
    io.zprob_out[rb] = mog_sigmoidf(lo);
    io.zkl_out[rb] = zkl;
    io.skl_out[rb] = skl;
    io.shkl_out[rb] = shkl;
    float* r = io.rec + (size_t)tc * R_NREC * B;
    r[R_SM * B + bc] = sm; r[R_SLV * B + bc] = slv;
    r[R_HM0 * B + bc] = hm0; r[R_HM1 * B + bc] = hm1;
    r[R_HLV0 * B + bc] = hv0; r[R_HLV1 * B + bc] = hv1;
    r[R_LO * B + bc] = lo; r[R_S * B + bc] = s; r[R_TX * B + bc] = tx; r[R_TY * B + bc] = ty;
    r[R_Y * B + bc] = y; r[R_Z * B + bc] = z;
  }
  // the loop state, step by step (lane 0 of the image; every lane shuffles)
  float zs[MAX_STEPS_FWD], zk[MAX_STEPS_FWD], ke[MAX_STEPS_FWD];
#pragma unroll
  for (int u = 0; u < MAX_STEPS_FWD; ++u) {
    if (8 * u < LPI) {
      zs[u] = __shfl(z, 8 * u, LPI);
      zk[u] = __shfl(zkl, 8 * u, LPI);
      ke[u] = __shfl(kl_end, 8 * u, LPI);
    }
  }
  if (b >= B || li != 0) return;
  float stop_old = stop0;
  int dig = dig0;
#pragma unroll
  for (int u = 0; u < MAX_STEPS_FWD; ++u) {
    if (8 * u >= LPI || u >= T) break;
    const long ru = (long)u * B + b;
    const bool act_old = stop_old < cfg.thr;
    const float zterm = act_old ? zk[u] : ke[u];  // (applied if live: mog_air_runloss)
    const float stop_new = stop_old + (1.0f - zs[u]);
    const bool act = stop_new < cfg.thr;
    if (act) {
      dig = dig + 1;
      io.live[u + 1] = 1;
    }
    io.zmask[ru] = act ? 1.0f : 0.0f;
    io.zval[ru] = zs[u];
    if (io.zc) io.zc[ru] = act ? zs[u] : 0.0f;
    float* r = io.rec + (size_t)u * R_NREC * B;
    r[R_ACT_OLD * B + b] = act_old ? 1.0f : 0.0f;
    r[R_ACT * B + b] = act ? 1.0f : 0.0f;
    r[R_LIVE * B + b] = 1.0f;
    r[R_ZC * B + b] = act ? zs[u] : 0.0f;
    r[R_ZTERM * B + b] = zterm;
    stop_old = stop_new;
  }
  io.stop[b] = stop_old;
  io.digits[b] = dig;
}

struct StepBwdIO {
  const float* rec;         // [R_NREC, B]
  const float* eps_scale;   // [B]
  const float* eps_shift;   // [B,2]
  const float* dtheta_fwd;  // [B,6] from STN-read backward
  const float* dtheta_back; // [B,6] from STN-write backward (already z*active scaled)
  const float* dot;         // [B] sum_p dcanvas*w  (canvas -> z_pres)
  const float* dloss;       // [B] per-image cotangent of the running loss (or null: grad_scale)
  float* dout;              // [5][B, 2] grads wrt head outputs, head stride dout_hs
  long dout_hs;
  int steps;                // loop steps in one launch: rows b = t * B + i, records of
                            // step t at rec + t * R_NREC * B, the rest [steps * B] rows
};

__global__ __launch_bounds__(256) void step_bwd_kernel(StepCfg cfg, StepBwdIO io) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  const int B = cfg.B;
  if (b >= B * io.steps) return;
  const int st = b / B, bi = b - st * B;  // loop step, image
  const float* r = io.rec + (size_t)st * R_NREC * B;  // step st's records
  const float sm = r[R_SM * B + bi], slv = r[R_SLV * B + bi];
  const float hm0 = r[R_HM0 * B + bi], hm1 = r[R_HM1 * B + bi];
  const float hv0 = r[R_HLV0 * B + bi], hv1 = r[R_HLV1 * B + bi];
  const float lo = r[R_LO * B + bi], s = r[R_S * B + bi], tx = r[R_TX * B + bi];
  const float ty = r[R_TY * B + bi], y = r[R_Y * B + bi], z = r[R_Z * B + bi];
  const bool act_old = r[R_ACT_OLD * B + bi] != 0.0f, act = r[R_ACT * B + bi] != 0.0f;
  const bool live = r[R_LIVE * B + bi] != 0.0f;
  const float gL = io.dloss ? io.dloss[bi] : cfg.grad_scale;
  const float T = cfg.temperature;

  // theta gradients -> (s, tx, ty)
  const float* dr = io.dtheta_fwd + (size_t)b * 6;
  const float* dw = io.dtheta_back + (size_t)b * 6;
  const float da = dw[0] + dw[4];
  const float s2 = s * s;
  float ds = dr[0] + dr[4] + da * (-1.0f / s2) + dw[2] * (tx / s2) + dw[5] * (ty / s2);
  float dtx = dr[2] - dw[2] / s;
  float dty = dr[5] - dw[5] / s;

  // z_pres: canvas term + concrete KL (train model only)
  float dz = act ? io.dot[b] : 0.0f;
  float dy = cfg.train ? dz * z * (1.0f - z) : 0.0f;
  const float aq = -y * T + lo;
  const float ap = -y * T + (prior_log_odds(cfg) + cfg.prior_bias);
  const float sq = mog_sigmoidf(aq), sp = mog_sigmoidf(ap);
  const float wz = (live && act_old) ? gL : 0.0f;
  float dlo = 0.0f;
  dy += wz * (2.0f * T * (sq - sp));
  dlo += wz * (1.0f - 2.0f * sq);
  if (cfg.use_num_prior) {
    const float we = (live && !act_old) ? gL : 0.0f;
    const float spe = mog_sigmoidf(-y * T + -100.0f);
    dy += we * (2.0f * T * (sq - spe));
    dlo += we * (1.0f - 2.0f * sq);
  }
  dlo += dy / T;

  // scale: s = sigmoid(sm + e*sqrt(exp(slv)))
  const float wn = act ? gL : 0.0f;
  const float dpre_s = ds * s * (1.0f - s);
  const float svar = mog_expf(slv);
  const float dsm = dpre_s + wn * (sm - cfg.s_pm) / cfg.s_pv;
  const float dslv = dpre_s * io.eps_scale[b] * 0.5f * sqrtf(svar) +
                     wn * 0.5f * (-1.0f + svar / cfg.s_pv);
  // shift: t = tanh(hm + e*sqrt(exp(hlv)))
  const float dpx = dtx * (1.0f - tx * tx), dpy = dty * (1.0f - ty * ty);
  const float hvar0 = mog_expf(hv0), hvar1 = mog_expf(hv1);
  const float dhm0 = dpx + wn * (hm0 - cfg.h_pm) / cfg.h_pv;
  const float dhm1 = dpy + wn * (hm1 - cfg.h_pm) / cfg.h_pv;
  const float dhv0 = dpx * io.eps_shift[2 * b] * 0.5f * sqrtf(hvar0) +
                     wn * 0.5f * (-1.0f + hvar0 / cfg.h_pv);
  const float dhv1 = dpy * io.eps_shift[2 * b + 1] * 0.5f * sqrtf(hvar1) +
                     wn * 0.5f * (-1.0f + hvar1 / cfg.h_pv);
  float* o = io.dout + 2 * b;
  const long hs = io.dout_hs;
  o[0] = dsm; o[1] = 0.0f;
  o[hs] = dslv; o[hs + 1] = 0.0f;
  o[2 * hs] = dhm0; o[2 * hs + 1] = dhm1;
  o[3 * hs] = dhv0; o[3 * hs + 1] = dhv1;
  o[4 * hs] = dlo; o[4 * hs + 1] = 0.0f;
}

// dHh_z[b][l] = relu'(Hh) * sum_c dout_z[b][c] W2_z[l][c]
// dhid layout: head z at dhid + z * dhid_hs, rows HS apart -- or, when
// dhid_hs == HS (heads side by side), rows 5 * HS apart: [B][5][HS], so that
// dh = [dhid_0 .. dhid_4] [W1_0 .. W1_4]^T is one plain GEMM over K = 5 HS
__global__ __launch_bounds__(256) void heads_hidden_bwd_kernel(HeadPtrs hp, const float* dout,
                                                               long dout_hs, float* dhid,
                                                               long dhid_hs, int B, int HS) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= 5L * B * HS) return;
  const int zh = idx / ((long)B * HS);
  const long rem = idx - (long)zh * B * HS;
  const int b = rem / HS, l = rem - (long)b * HS;
  const long rs = dhid_hs == HS ? 5L * HS : HS;
  const int k = (zh == 2 || zh == 3) ? 2 : 1;
  const float h = hp.hid[zh][(size_t)b * HS + l];
  float v = 0.0f;
  if (h > 0.0f) {
    v = dout[zh * dout_hs + b * 2] * hp.w2[zh][l * k];
    if (k == 2) v += dout[zh * dout_hs + b * 2 + 1] * hp.w2[zh][l * k + 1];
  }
  dhid[zh * dhid_hs + (long)b * rs + l] = v;
}

// The same, four hidden units per thread (HS % 4 == 0, 16-byte aligned rows):
// one head per grid row (blockIdx.y), 32-bit index math, 16-byte loads of the
// hidden activations and stores of dhid
__global__ __launch_bounds__(256) void heads_hidden_bwd4_kernel(HeadPtrs hp, const float* dout,
                                                                long dout_hs, float* dhid,
                                                                long dhid_hs, int B, int HS) {
  const int zh = blockIdx.y;
  const int hq = HS >> 2;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= B * hq) return;
  const int b = q / hq, l0 = (q - b * hq) * 4;
  const int k = (zh == 2 || zh == 3) ? 2 : 1;
  const float4 h = *reinterpret_cast<const float4*>(hp.hid[zh] + (size_t)b * HS + l0);
  const float* dz = dout + zh * dout_hs + (size_t)b * 2;
  const float d0 = dz[0], d1 = k == 2 ? dz[1] : 0.0f;
  const float* w = hp.w2[zh];
  const float hv[4] = {h.x, h.y, h.z, h.w};
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int l = l0 + e;
    // weights loaded unconditionally (a load under the relu test compiles to
    // a branch with a vmcnt(0) wait inside); same arithmetic where h > 0
    const float w0 = w[l * k], w1 = w[l * k + (k == 2 ? 1 : 0)];
    float a = d0 * w0;
    if (k == 2) a += d1 * w1;
    v[e] = hv[e] > 0.0f ? a : 0.0f;
  }
  const long rs = dhid_hs == HS ? 5L * HS : HS;
  *reinterpret_cast<float4*>(dhid + zh * dhid_hs + (size_t)b * rs + l0) =
      make_float4(v[0], v[1], v[2], v[3]);
}

// Weight / bias gradients of the heads' output layers (air_model.py:462-499:
// dW2_z = hid_z^T dout_z, db2_z = colsum dout_z over the R = T*B rows; HS x 1
// or HS x 2 each), deterministic: row chunk s of head z sums its CH rows in
// row order into work[z][s][.] (thread t < 2 HS: weight (t % HS, t / HS);
// 2 HS, 2 HS + 1: the bias columns), then heads_out_reduce_kernel adds the
// chunks in chunk order into the gradients.  (At the batch sizes that split K
// the 1- / 2-column products wasted most of a 64- or 128-wide MFMA tile;
// this reads the hidden activations once.)
constexpr int HO_CH = 128, HO_MAXH = 5;
struct HeadsOut {
  const float* hid[HO_MAXH];  // [R][HS]
  const float* dout[HO_MAXH]; // [R][2]
  float* gw[HO_MAXH];         // [HS][k]
  float* gb[HO_MAXH];         // [k]
  int k[HO_MAXH];
  int R, HS, S;
  float* work;                // [nheads][S][2 HS + 2]
};

__global__ __launch_bounds__(256) void heads_out_partial_kernel(HeadsOut a) {
  const int z = blockIdx.y, sc = blockIdx.x, t = threadIdx.x;
  const int HS = a.HS, W = 2 * HS + 2;
  if (t >= W) return;
  const int r0 = sc * HO_CH, r1 = min(a.R, r0 + HO_CH);
  const float* hid = a.hid[z];
  const float* dout = a.dout[z];
  const bool bias = t >= 2 * HS;
  const int l = bias ? 0 : t % HS, c = bias ? t - 2 * HS : t / HS;
  float acc = 0.0f;
  int b = r0;
  // 32 rows' operands in flight per round trip (the loads of a chunk would
  // otherwise be one latency each)
  for (; b + 32 <= r1; b += 32) {
    float h[32], d[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      h[i] = bias ? 1.0f : hid[(size_t)(b + i) * HS + l];
      d[i] = dout[(size_t)(b + i) * 2 + c];
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) acc = fmaf(h[i], d[i], acc);
  }
  for (; b < r1; ++b) acc = fmaf(bias ? 1.0f : hid[(size_t)b * HS + l], dout[(size_t)b * 2 + c], acc);
  a.work[((size_t)z * a.S + sc) * W + t] = acc;
}

__global__ __launch_bounds__(256) void heads_out_reduce_kernel(HeadsOut a) {
  const int z = blockIdx.x, t = threadIdx.x;
  const int HS = a.HS, W = 2 * HS + 2;
  if (t >= W) return;
  const bool bias = t >= 2 * HS;
  const int l = bias ? 0 : t % HS, c = bias ? t - 2 * HS : t / HS;
  if (c >= a.k[z]) return;
  const float* w = a.work + (size_t)z * a.S * W + t;
  float sum = 0.0f;
  // in chunk order; 32 partials loaded per round trip
  for (int s0 = 0; s0 < a.S; s0 += 32) {
    float v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = s0 + i < a.S ? w[(size_t)(s0 + i) * W] : 0.0f;
#pragma unroll
    for (int i = 0; i < 32; ++i)
      if (s0 + i < a.S) sum = sum + v[i];
  }
  float* dst = bias ? a.gb[z] + c : a.gw[z] + l * a.k[z] + c;
  if (bias && a.gb[z] == nullptr) return;
  *dst = *dst + sum;
}

// --------------------------------------------------------- VAE sample ---
struct VaeCfg {
  int B, Z;
  float v_pm, v_pv, v_plv, grad_scale;
};

// z = mu + eps*sqrt(exp(lv)); vkl = 0.5*sum_k term_k (sequential in k);
// runloss += act ? vkl : 0.  One wave per image: lane k owns latent k, lane 0
// then sums the KL terms in k order (Z <= 64).
__global__ __launch_bounds__(256) void vae_sample_fwd_kernel(VaeCfg c, const float* mu,
                                                             const float* lv, const float* eps,
                                                             float* z, __bf16* zb, int ldzb,
                                                             const float* act, float* runloss,
                                                             float* vkl_out) {
#pragma clang fp contract(off)
  __shared__ float terms[4][64];
  const int w = threadIdx.x >> 6, k = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + w;
  if (b < c.B && k < c.Z) {
    const size_t i = (size_t)b * c.Z + k;
    const float l = lv[i];
    const float var = mog_expf(l);
    const float zv = mu[i] + eps[i] * sqrtf(var);
    z[i] = zv;
    if (zb) zb[(size_t)b * ldzb + k] = (__bf16)zv;
    terms[w][k] = gauss_kl_term(c.v_plv, l, var, c.v_pv, mu[i], c.v_pm);
  }
  __syncthreads();
  if (b >= c.B || k != 0) return;
  float sum = 0.0f;
  for (int q = 0; q < c.Z; ++q) sum = sum + terms[w][q];
  const float vkl = 0.5f * sum;
  vkl_out[b] = vkl;
  if (runloss && act[b] != 0.0f) runloss[b] = runloss[b] + vkl;
}

// Per-image running loss of all T steps replayed from the step records in the
// order the step kernels accumulate it (step_fwd_kernel, then the VAE KL):
// for the VAE of every step run after the loop (AIR, all T*B rows at once).
// With `live` (the records of step_fwd_steps_kernel): the loop predicate is
// applied first -- the z_pres term of a step that is not live is 0 and its
// records say so (rec[R_ZTERM], rec[R_LIVE] rewritten).
__global__ __launch_bounds__(256) void runloss_kernel(int T, int B, float* __restrict__ rec,
                                                      long rstride, const float* __restrict__ skl,
                                                      const float* __restrict__ shkl,
                                                      const float* __restrict__ vkl,
                                                      float* runloss, const int* live) {
#pragma clang fp contract(off)
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  float rl = 0.0f;
  for (int t = 0; t < T; ++t) {
    float* r = rec + t * rstride;
    if (live) {
      const bool lv = live[t] != 0;
      const float zt = lv ? r[R_ZTERM * B + b] : 0.0f;
      r[R_ZTERM * B + b] = zt;
      r[R_LIVE * B + b] = lv ? 1.0f : 0.0f;
    }
    rl = rl + r[R_ZTERM * B + b];
    if (r[R_ACT * B + b] != 0.0f) {
      const size_t i = (size_t)t * B + b;
      rl = rl + skl[i];
      rl = rl + shkl[i];
      rl = rl + vkl[i];
    }
  }
  runloss[b] = rl;
}

__global__ __launch_bounds__(256) void vae_sample_bwd_kernel(VaeCfg c, const float* mu,
                                                             const float* lv, const float* eps,
                                                             const float* dz, const float* act,
                                                             float* dmu, float* dlv,
                                                             __bf16* dmub, __bf16* dlvb,
                                                             int ldb) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)c.B * c.Z) return;
  const int b = i / c.Z, k = i - (long)b * c.Z;
  const float wn = act[b] != 0.0f ? c.grad_scale : 0.0f;
  const float var = mog_expf(lv[i]);
  const float g = dz[i];
  const float vm = g + wn * (mu[i] - c.v_pm) / c.v_pv;
  const float vl = g * eps[i] * 0.5f * sqrtf(var) + wn * 0.5f * (-1.0f + var / c.v_pv);
  if (dmu) dmu[i] = vm;
  if (dlv) dlv[i] = vl;
  if (dmub) dmub[(size_t)b * ldb + k] = (__bf16)vm;
  if (dlvb) dlvb[(size_t)b * ldb + k] = (__bf16)vl;
}

// dm = dr * r * (1 - r)   (TF SigmoidGrad); fp32 or bf16 output
template <bool BF16>
__global__ __launch_bounds__(256) void sigmoid_bwd_kernel(const float* r, const float* dr,
                                                          void* dm, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float v = r[i];
  const float d = dr[i] * v * (1.0f - v);
  if (BF16) reinterpret_cast<__bf16*>(dm)[i] = (__bf16)d;
  else reinterpret_cast<float*>(dm)[i] = d;
}

// ---------------------------------------------------------------- loss ---
// One block per image: clip, BCE, MSE, per-image loss, dL/dcanvas.
__device__ __forceinline__ void recon_pixel(float c, float xv, float grad_scale, float& bce,
                                            float& mse, float& r_out, float& g_out) {
#pragma clang fp contract(off)
  const float r = fmaxf(fminf(c, 1.0f), 0.0f);
  // the BCE is a 2500-term reduction compared within 1e-5 relative, so the
  // hardware log (v_log_f32, ~1 ulp) is used here, not the bit-exact spec
  const float lr = __logf(r + 1e-10f);
  const float l1r = __logf((1.0f - r) + 1e-10f);
  bce = bce + (xv * lr + (1.0f - xv) * l1r);
  const float d = xv - r;
  mse = mse + d * d;
  r_out = r;
  const bool pass = (c >= 0.0f) && (c <= 1.0f);  // TF Min/Max grads pass at equality
  const float g = -(xv * (1.0f / (r + 1e-10f)) - (1.0f - xv) * (1.0f / ((1.0f - r) + 1e-10f)));
  g_out = pass ? g * grad_scale : 0.0f;
}

// One block per image, four pixels per thread-iteration (16-byte accesses).
// With nparts > 0 the canvas is the step-ordered sum of the per-step
// contributions ((p0 + p1) + p2 ..., the accumulation order of
// air_model.py:665-675) and is written to canvas_out when given.  With
// part_rows, part t of image b holds only rows [lo, hi) (part_rows[t*B + b] =
// lo | hi << 16, row ranges aligned so that no 4-pixel group straddles them)
// and is +0 elsewhere: those pixels are never read and +0 is added instead,
// which leaves the sum bit-identical.
template <bool VEC>
__global__ __launch_bounds__(256) void recon_loss_kernel(
    const float* __restrict__ x, const float* __restrict__ canvas_in,
    const float* __restrict__ parts, int nparts, long part_stride,
    const int* __restrict__ part_rows, int B, int C, float* canvas_out,
    const float* __restrict__ runloss, const int* __restrict__ digits,
    const int* __restrict__ targets, int C2, float grad_scale, float* recon, float* bce_out,
    float* mse_out, float* loss_out, float* acc_out, float* dcanvas) {
#pragma clang fp contract(off)
  __shared__ float red[4];
  const int b = blockIdx.x;
  const size_t base = (size_t)b * C2;
  float bce = 0.0f, mse = 0.0f;
  constexpr int V = VEC ? 4 : 1;
  typedef float vec __attribute__((ext_vector_type(V)));
  auto part = [&](int t, int p) -> vec {  // part t's pixels p..p+V-1 (+0 where not stored)
    vec v = 0.0f;
    const int pr = part_rows ? part_rows[(size_t)t * B + b] : 0;
    if (!part_rows || (p >= (pr & 0xffff) * C && p < (pr >> 16) * C))
      v = *reinterpret_cast<const vec*>(parts + t * part_stride + base + p);
    return v;
  };
  for (int p = threadIdx.x * V; p < C2; p += 256 * V) {
    vec c;
    if (nparts > 0) {
      c = part(0, p);
      for (int t = 1; t < nparts; ++t) c = c + part(t, p);
      if (canvas_out) *reinterpret_cast<vec*>(canvas_out + base + p) = c;
    } else {
      c = *reinterpret_cast<const vec*>(canvas_in + base + p);
    }
    const vec xv = *reinterpret_cast<const vec*>(x + base + p);
    vec r, g;
#pragma unroll
    for (int u = 0; u < V; ++u) {
      float ru, gu;
      recon_pixel(c[u], xv[u], grad_scale, bce, mse, ru, gu);
      r[u] = ru;
      g[u] = gu;
    }
    if (recon) *reinterpret_cast<vec*>(recon + base + p) = r;
    if (dcanvas) *reinterpret_cast<vec*>(dcanvas + base + p) = g;
  }
  bce = mog_block_sum256(bce, red);
  __syncthreads();
  mse = mog_block_sum256(mse, red);
  if (threadIdx.x == 0) {
    bce_out[b] = -bce;
    mse_out[b] = mse;
    loss_out[b] = runloss[b] + (-bce);
    if (acc_out) acc_out[b] = (targets && targets[b] == digits[b]) ? 1.0f : 0.0f;
  }
}

// mean over B of up to 4 per-image vectors -> out[4] (single block, fixed order)
// One 1024-thread block; each array is read with all its loads in flight at
// once (four independent partial sums per thread, 16-byte loads when the
// array allows), then reduced over the block.  (The former 256-thread
// single-accumulator loop was one dependent load chain per thread: 26 us at
// B = 8192.)
__global__ __launch_bounds__(1024) void batch_mean_kernel(const float* a0, const float* a1,
                                                          const float* a2, const float* a3,
                                                          int B, float inv, float* out) {
  __shared__ float red[4][16];
  const float* v[4] = {a0, a1, a2, a3};
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float s = 0.0f;
    if (v[k]) {
      float p[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if ((B & 3) == 0 && (reinterpret_cast<size_t>(v[k]) & 15) == 0) {
        const float4* q = reinterpret_cast<const float4*>(v[k]);
        for (int i = t; i < B / 4; i += 1024) {
          const float4 x = q[i];
          p[0] += x.x; p[1] += x.y; p[2] += x.z; p[3] += x.w;
        }
      } else {
        for (int i = t; i < B; i += 1024) p[0] += v[k][i];
      }
      s = (p[0] + p[1]) + (p[2] + p[3]);
    }
    s = mog_wave_sum(s);
    if (l == 0) red[k][w] = s;
  }
  __syncthreads();
  if (t < 4 && v[t]) {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red[t][i];
    out[t] = s * inv;
  }
}

// column sums of X [R, N] (row stride ld) -> atomically added into out[N]
__global__ __launch_bounds__(256) void colsum_kernel(const float* X, int R, int N, int ld,
                                                     int rows_per_block, float* out) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= N) return;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(R, r0 + rows_per_block);
  float s = 0.0f;
  for (int r = r0; r < r1; ++r) s += X[(size_t)r * ld + col];
  atomicAdd(out + col, s);
}

// Up to 8 buffers filled with a 32-bit pattern in one launch (the step's
// loop-state resets: stopping sum, running loss, counts, live flags; the
// gradient buffer): grid row j covers buffer j.
constexpr int FILL_MAX = 8;
struct FillBatch {
  unsigned* dst[FILL_MAX];
  long n[FILL_MAX];
  unsigned v[FILL_MAX];
};
__global__ __launch_bounds__(256) void fill32_batch_kernel(FillBatch f) {
  const int j = blockIdx.y;
  const long n = f.n[j], stride = (long)gridDim.x * 256 * 4;
  const unsigned v = f.v[j];
  unsigned* d = f.dst[j];
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 4 <= n && (reinterpret_cast<size_t>(d + i) & 15) == 0) {
      *reinterpret_cast<uint4*>(d + i) = make_uint4(v, v, v, v);
    } else {
      for (long k = i; k < n && k < i + 4; ++k) d[k] = v;
    }
  }
}

// Up to FILL_MAX copies of 32-bit words in one launch (grid row j: copy j):
// a captured step's inputs into the graph's static buffers
struct CopyBatch {
  unsigned* dst[FILL_MAX];
  const unsigned* src[FILL_MAX];
  long n[FILL_MAX];
};
__global__ __launch_bounds__(256) void copy32_batch_kernel(CopyBatch f) {
  const int j = blockIdx.y;
  const long n = f.n[j], stride = (long)gridDim.x * 256 * 4;
  unsigned* d = f.dst[j];
  const unsigned* a = f.src[j];
  const bool vec = ((reinterpret_cast<size_t>(d) | reinterpret_cast<size_t>(a)) & 15) == 0;
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
    if (vec && i + 4 <= n) {
      *reinterpret_cast<uint4*>(d + i) = *reinterpret_cast<const uint4*>(a + i);
    } else {
      for (long k = i; k < n && k < i + 4; ++k) d[k] = a[k];
    }
  }
}

// Up to FILL_MAX matrix transposes in one launch (grid row j: matrix j,
// dst[c][r] = src[r][c], rows x cols): the small-batch forward's transposed
// copies of the VAE layers whose N or K (the latent 50) misses the LDS-DMA
// alignment, refreshed inside the captured step
struct TransBatch {
  float* dst[FILL_MAX];
  const float* src[FILL_MAX];
  int rows[FILL_MAX], cols[FILL_MAX];
};
__global__ __launch_bounds__(256) void transpose32_batch_kernel(TransBatch f) {
  const int j = blockIdx.y;
  const long n = (long)f.rows[j] * f.cols[j], stride = (long)gridDim.x * 256;
  const int cols = f.cols[j], rows = f.rows[j];
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const int c = (int)(i / rows), r = (int)(i - (long)c * rows);  // dst order: coalesced stores
    f.dst[j][i] = f.src[j][(size_t)r * cols + c];
  }
}

// out[i] = a[i] + b[i]
__global__ __launch_bounds__(256) void add_kernel(const float* a, const float* b, float* out,
                                                  long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}

// Generation prior draws (air_model.py:1013-1035 via _sample_from_mvn
// :186-192; vae.py:63-66): per image the glimpse scale / shift and the
// backward transform, per latent element z = prior mean + eps sqrt(exp(lv)).
__global__ __launch_bounds__(256) void gen_prior_kernel(int G, int Z, float s_pm, float s_plv,
                                                        float h_pm, float h_plv, float v_pm,
                                                        float v_plv, const float* eps_scale,
                                                        const float* eps_shift,
                                                        const float* eps_z, float* theta_back,
                                                        float* scale, float* shift, float* z) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < G * Z) z[i] = v_pm + eps_z[i] * sqrtf(mog_expf(v_plv));
  if (i >= G) return;
  const float s = mog_sigmoidf(s_pm + eps_scale[i] * sqrtf(mog_expf(s_plv)));
  const float hv = sqrtf(mog_expf(h_plv));
  const float tx = mog_tanhf(h_pm + eps_shift[2 * i] * hv);
  const float ty = mog_tanhf(h_pm + eps_shift[2 * i + 1] * hv);
  float* tb = theta_back + (size_t)i * 6;
  tb[0] = 1.0f / s; tb[1] = 0.0f; tb[2] = -tx / s;
  tb[3] = 0.0f; tb[4] = 1.0f / s; tb[5] = -ty / s;
  scale[i] = s;
  shift[2 * i] = tx;
  shift[2 * i + 1] = ty;
}

}  // namespace

// ============================================================== C ABI ======
extern "C" int mog_lstm_cell_forward(const float* G, const float* bias, const float* c_prev,
                                     float* c_out, float* h_out, int B, int H, void* stream) {
  MOG_CHECK_ARG(G && c_out && h_out && B >= 0 && H > 0);
  if (B == 0) return 0;
  lstm_fwd_kernel<<<mog_cdiv((long)B * H, 256), 256, 0, mog_stream(stream)>>>(
      LstmFwd{G, bias, c_prev, c_out, h_out}, B, H);
  MOG_LAUNCH_RET();
}

extern "C" int mog_lstm_cell_backward(const float* G, const float* bias, const float* c_prev,
                                      const float* c_cur, const float* dh, const float* dc,
                                      float* dG, float* dc_prev, float* dGsum, int B, int H,
                                      void* stream) {
  MOG_CHECK_ARG(G && c_cur && dh && dG && B >= 0 && H > 0);
  if (B == 0) return 0;
  lstm_bwd_kernel<<<mog_cdiv((long)B * H, 256), 256, 0, mog_stream(stream)>>>(
      LstmBwd{G, bias, c_prev, c_cur, dh, dc, dG, dc_prev, dGsum}, B, H);
  MOG_LAUNCH_RET();
}

extern "C" int mog_lstm_cell_backward_parts(const float* G, const float* bias,
                                            const float* c_prev, const float* c_cur,
                                            const float* dh, const float* dh_parts, int nparts,
                                            long part_stride, const float* dc, float* dG,
                                            float* dc_prev, float* dGsum, int B, int H,
                                            void* stream) {
  MOG_CHECK_ARG(G && c_cur && dh && dG && B >= 0 && H > 0 && nparts >= 0 && nparts <= 4);
  MOG_CHECK_ARG(nparts == 0 || (dh_parts && part_stride >= (long)B * H));
  if (B == 0) return 0;
  LstmBwd a{G, bias, c_prev, c_cur, dh, dc, dG, dc_prev, dGsum};
  a.dh_parts = dh_parts;
  a.nparts = nparts;
  a.part_stride = part_stride;
  lstm_bwd_kernel<<<mog_cdiv((long)B * H, 256), 256, 0, mog_stream(stream)>>>(a, B, H);
  MOG_LAUNCH_RET();
}

extern "C" int mog_lstm_cell_forward_pair(const float* const* cells, int B, int H, void* stream) {
  MOG_CHECK_ARG(cells && B >= 0 && H > 0);
  const float* const* a = cells;
  const float* const* b = cells + 5;
  MOG_CHECK_ARG(a[0] && a[3] && a[4] && b[0] && b[3] && b[4]);
  if (B == 0) return 0;
  lstm_fwd_pair_kernel<<<dim3(mog_cdiv((long)B * H, 256), 2), 256, 0, mog_stream(stream)>>>(
      LstmFwd{a[0], a[1], a[2], const_cast<float*>(a[3]), const_cast<float*>(a[4])},
      LstmFwd{b[0], b[1], b[2], const_cast<float*>(b[3]), const_cast<float*>(b[4])}, B, H);
  MOG_LAUNCH_RET();
}

extern "C" int mog_lstm_cell_backward_pair(const float* const* cells, int B, int H,
                                           void* stream) {
  MOG_CHECK_ARG(cells && B >= 0 && H > 0);
  LstmBwd c[2];
  for (int k = 0; k < 2; ++k) {
    const float* const* a = cells + 9 * k;
    MOG_CHECK_ARG(a[0] && a[3] && a[4] && a[6]);
    c[k] = LstmBwd{a[0], a[1], a[2], a[3], a[4], a[5], const_cast<float*>(a[6]),
                   const_cast<float*>(a[7]), const_cast<float*>(a[8])};
  }
  if (B == 0) return 0;
  lstm_bwd_pair_kernel<<<dim3(mog_cdiv((long)B * H, 256), 2), 256, 0, mog_stream(stream)>>>(
      c[0], c[1], B, H);
  MOG_LAUNCH_RET();
}

extern "C" int mog_air_step_forward(
    int B, int HS, int HZ, int step, int train, int use_num_prior, float thr, float temperature,
    float prior_lo, float prior_bias, float s_pm, float s_pv, float s_plv, float h_pm, float h_pv,
    float h_plv, const float* const* hid, const float* const* w2, const float* const* b2,
    const float* eps_scale, const float* eps_shift, const float* u, float* stop, float* runloss,
    int* digits, int* live, float* rec, float* theta_fwd, float* theta_back, float* scale_out,
    float* shift_out, float* zprob_out, float* zkl_out, float* skl_out, float* shkl_out,
    float* zmask, float* zval, float* zc, const float* prior_lo_dev, void* stream) {
  MOG_CHECK_ARG(B >= 0 && hid && w2 && b2 && eps_scale && eps_shift && u && stop && runloss);
  MOG_CHECK_ARG(digits && live && rec && theta_fwd && theta_back && scale_out && shift_out);
  MOG_CHECK_ARG(zprob_out && zkl_out && skl_out && shkl_out && zmask && zval);
  if (B == 0) return 0;
  StepCfg c;
  c.B = B; c.H = 0; c.HS = HS; c.HZ = HZ; c.train = train; c.use_num_prior = use_num_prior;
  c.step = step; c.thr = thr; c.temperature = temperature; c.prior_lo = prior_lo;
  c.prior_bias = prior_bias; c.s_pm = s_pm; c.s_pv = s_pv; c.s_plv = s_plv; c.h_pm = h_pm;
  c.h_pv = h_pv; c.h_plv = h_plv; c.grad_scale = 0.0f; c.prior_lo_dev = prior_lo_dev;
  HeadPtrs hp;
  for (int i = 0; i < 5; ++i) {
    MOG_CHECK_ARG(hid[i] && w2[i] && b2[i]);
    hp.hid[i] = hid[i]; hp.w2[i] = w2[i]; hp.b2[i] = b2[i];
  }
  StepFwdIO io{eps_scale, eps_shift, u,       stop,     runloss,  digits,    live,
               rec,       theta_fwd, theta_back, scale_out, shift_out, zprob_out, zkl_out,
               skl_out,   shkl_out,  zmask,   zval,     zc};
  step_fwd_kernel<<<mog_cdiv(B, 32), 256, 0, mog_stream(stream)>>>(c, hp, io);
  MOG_LAUNCH_RET();
}

extern "C" int mog_air_step_forward_steps(
    int steps, int B, int HS, int HZ, int train, int use_num_prior, float thr, float temperature,
    float prior_lo, const float* prior_bias, float s_pm, float s_pv, float s_plv, float h_pm,
    float h_pv, float h_plv, const float* const* hid, long hid_step, const float* const* w2,
    const float* const* b2, const float* eps_scale, const float* eps_shift, const float* u,
    float* stop, int* digits, int* live, float* rec, float* theta_fwd, float* theta_back,
    float* scale_out, float* shift_out, float* zprob_out, float* zkl_out, float* skl_out,
    float* shkl_out, float* zmask, float* zval, float* zc, const float* prior_lo_dev,
    void* stream) {
  MOG_CHECK_ARG(steps >= 1 && steps <= MAX_STEPS_FWD && B >= 0 && prior_bias);
  MOG_CHECK_ARG(hid && w2 && b2 && eps_scale && eps_shift && u && stop);
  MOG_CHECK_ARG(digits && live && rec && theta_fwd && theta_back && scale_out && shift_out);
  MOG_CHECK_ARG(zprob_out && zkl_out && skl_out && shkl_out && zmask && zval);
  MOG_CHECK_ARG(hid_step >= (long)B * (HS > HZ ? HS : HZ));
  if (B == 0) return 0;
  StepCfg c;
  c.B = B; c.H = 0; c.HS = HS; c.HZ = HZ; c.train = train; c.use_num_prior = use_num_prior;
  c.step = 0; c.thr = thr; c.temperature = temperature; c.prior_lo = prior_lo;
  c.prior_bias = 0.0f; c.s_pm = s_pm; c.s_pv = s_pv; c.s_plv = s_plv; c.h_pm = h_pm;
  c.h_pv = h_pv; c.h_plv = h_plv; c.grad_scale = 0.0f; c.prior_lo_dev = prior_lo_dev;
  HeadPtrs hp;
  for (int i = 0; i < 5; ++i) {
    MOG_CHECK_ARG(hid[i] && w2[i] && b2[i]);
    hp.hid[i] = hid[i]; hp.w2[i] = w2[i]; hp.b2[i] = b2[i];
  }
  StepsFwdIO q;
  q.s = StepFwdIO{eps_scale, eps_shift, u,         stop,      nullptr,  digits,  live,
                  rec,       theta_fwd, theta_back, scale_out, shift_out, zprob_out, zkl_out,
                  skl_out,   shkl_out,  zmask,     zval,      zc};
  q.hid_step = hid_step;
  q.steps = steps;
  for (int t = 0; t < MAX_STEPS_FWD; ++t) q.prior_bias[t] = t < steps ? prior_bias[t] : 0.0f;
  hipStream_t s = mog_stream(stream);
  const int lpi = steps == 1 ? 8 : steps == 2 ? 16 : steps <= 4 ? 32 : 64;
  const int grid = mog_cdiv((long)B * lpi, 256);
  switch (lpi) {
    case 8: step_fwd_steps_kernel<8><<<grid, 256, 0, s>>>(c, hp, q); break;
    case 16: step_fwd_steps_kernel<16><<<grid, 256, 0, s>>>(c, hp, q); break;
    case 32: step_fwd_steps_kernel<32><<<grid, 256, 0, s>>>(c, hp, q); break;
    default: step_fwd_steps_kernel<64><<<grid, 256, 0, s>>>(c, hp, q); break;
  }
  MOG_LAUNCH_RET();
}

extern "C" int mog_air_step_backward_steps(
    int steps, int B, int HS, int train, int use_num_prior, float temperature, float prior_lo,
    float prior_bias, float s_pm, float s_pv, float h_pm, float h_pv, float grad_scale,
    const float* dloss, const float* rec, const float* eps_scale, const float* eps_shift,
    const float* dtheta_fwd, const float* dtheta_back, const float* dot, const float* const* hid,
    const float* const* w2, float* dout, long dout_hs, float* dhid, long dhid_hs,
    const float* prior_lo_dev, void* stream);

extern "C" int mog_air_step_backward(int B, int HS, int train, int use_num_prior,
                                     float temperature, float prior_lo, float prior_bias,
                                     float s_pm, float s_pv, float h_pm, float h_pv,
                                     float grad_scale, const float* dloss, const float* rec,
                                     const float* eps_scale, const float* eps_shift,
                                     const float* dtheta_fwd,
                                     const float* dtheta_back, const float* dot,
                                     const float* const* hid, const float* const* w2,
                                     float* dout, long dout_hs, float* dhid, long dhid_hs,
                                     const float* prior_lo_dev, void* stream) {
  return mog_air_step_backward_steps(1, B, HS, train, use_num_prior, temperature, prior_lo,
                                     prior_bias, s_pm, s_pv, h_pm, h_pv, grad_scale, dloss, rec,
                                     eps_scale, eps_shift, dtheta_fwd, dtheta_back, dot, hid, w2,
                                     dout, dout_hs, dhid, dhid_hs, prior_lo_dev, stream);
}

extern "C" int mog_air_step_backward_steps(
    int steps, int B, int HS, int train, int use_num_prior, float temperature, float prior_lo,
    float prior_bias, float s_pm, float s_pv, float h_pm, float h_pv, float grad_scale,
    const float* dloss, const float* rec, const float* eps_scale, const float* eps_shift,
    const float* dtheta_fwd, const float* dtheta_back, const float* dot, const float* const* hid,
    const float* const* w2, float* dout, long dout_hs, float* dhid, long dhid_hs,
    const float* prior_lo_dev, void* stream) {
  MOG_CHECK_ARG(steps >= 1 && B >= 0 && rec && eps_scale && eps_shift && dtheta_fwd &&
                dtheta_back && dot);
  MOG_CHECK_ARG(hid && w2 && dout && dhid);
  if (B == 0) return 0;
  const int rows = steps * B;  // the head-hidden kernels see the steps as one batch
  StepCfg c;
  c.B = B; c.H = 0; c.HS = HS; c.HZ = HS; c.train = train; c.use_num_prior = use_num_prior;
  c.step = 0; c.thr = 0.0f; c.temperature = temperature; c.prior_lo = prior_lo;
  c.prior_bias = prior_bias; c.s_pm = s_pm; c.s_pv = s_pv; c.s_plv = 0.0f; c.h_pm = h_pm;
  c.h_pv = h_pv; c.h_plv = 0.0f; c.grad_scale = grad_scale; c.prior_lo_dev = prior_lo_dev;
  StepBwdIO io{rec, eps_scale, eps_shift, dtheta_fwd, dtheta_back, dot, dloss, dout, dout_hs,
               steps};
  hipStream_t s = mog_stream(stream);
  step_bwd_kernel<<<mog_cdiv(rows, 256), 256, 0, s>>>(c, io);
  HeadPtrs hp;
  for (int i = 0; i < 5; ++i) {
    MOG_CHECK_ARG(hid[i] && w2[i]);
    hp.hid[i] = hid[i]; hp.w2[i] = w2[i]; hp.b2[i] = nullptr;
  }
  bool vec = HS % 4 == 0 && (dhid_hs % 4) == 0 && (reinterpret_cast<uintptr_t>(dhid) & 15) == 0;
  for (int i = 0; i < 5; ++i) vec = vec && (reinterpret_cast<uintptr_t>(hid[i]) & 15) == 0;
  if (vec)
    heads_hidden_bwd4_kernel<<<dim3(mog_cdiv((long)rows * (HS / 4), 256), 5), 256, 0, s>>>(
        hp, dout, dout_hs, dhid, dhid_hs, rows, HS);
  else
    heads_hidden_bwd_kernel<<<mog_cdiv(5L * rows * HS, 256), 256, 0, s>>>(hp, dout, dout_hs, dhid,
                                                                           dhid_hs, rows, HS);
  MOG_LAUNCH_RET();
}

extern "C" int mog_vae_sample_forward(int B, int Z, float v_pm, float v_pv, float v_plv,
                                      const float* mu, const float* lv, const float* eps,
                                      float* z, void* z_bf16, int ld_zb, const float* act,
                                      float* runloss, float* vkl, void* stream) {
  MOG_CHECK_ARG(B >= 0 && Z > 0 && Z <= 64 && mu && lv && eps && z && act && vkl);
  MOG_CHECK_ARG(!z_bf16 || ld_zb >= Z);
  if (B == 0) return 0;
  VaeCfg c{B, Z, v_pm, v_pv, v_plv, 0.0f};
  vae_sample_fwd_kernel<<<mog_cdiv(B, 4), 256, 0, mog_stream(stream)>>>(
      c, mu, lv, eps, z, reinterpret_cast<__bf16*>(z_bf16), ld_zb, act, runloss, vkl);
  MOG_LAUNCH_RET();
}

extern "C" int mog_air_runloss(int T, int B, float* rec, long rec_step_stride,
                               const float* skl, const float* shkl, const float* vkl,
                               float* runloss, const int* live, void* stream) {
  MOG_CHECK_ARG(T >= 1 && B >= 0 && rec && skl && shkl && vkl && runloss);
  MOG_CHECK_ARG(rec_step_stride >= (long)R_NREC * B);
  if (B == 0) return 0;
  runloss_kernel<<<mog_cdiv(B, 256), 256, 0, mog_stream(stream)>>>(
      T, B, rec, rec_step_stride, skl, shkl, vkl, runloss, live);
  MOG_LAUNCH_RET();
}

extern "C" int mog_vae_sample_backward(int B, int Z, float v_pm, float v_pv, float grad_scale,
                                       const float* mu, const float* lv, const float* eps,
                                       const float* dz, const float* act, float* dmu,
                                       float* dlv, void* dmu_bf16, void* dlv_bf16, int ld_b,
                                       void* stream) {
  MOG_CHECK_ARG(B >= 0 && Z > 0 && mu && lv && eps && dz && act);
  MOG_CHECK_ARG((dmu && dlv) || (dmu_bf16 && dlv_bf16 && ld_b >= Z));
  if (B == 0) return 0;
  VaeCfg c{B, Z, v_pm, v_pv, 0.0f, grad_scale};
  vae_sample_bwd_kernel<<<mog_cdiv((long)B * Z, 256), 256, 0, mog_stream(stream)>>>(
      c, mu, lv, eps, dz, act, dmu, dlv, reinterpret_cast<__bf16*>(dmu_bf16),
      reinterpret_cast<__bf16*>(dlv_bf16), ld_b);
  MOG_LAUNCH_RET();
}

extern "C" int mog_sigmoid_backward(const float* r, const float* dr, void* dm, long n,
                                    int out_bf16, void* stream) {
  MOG_CHECK_ARG(r && dr && dm && n >= 0);
  if (n == 0) return 0;
  if (out_bf16)
    sigmoid_bwd_kernel<true><<<mog_cdiv(n, 256), 256, 0, mog_stream(stream)>>>(r, dr, dm, n);
  else
    sigmoid_bwd_kernel<false><<<mog_cdiv(n, 256), 256, 0, mog_stream(stream)>>>(r, dr, dm, n);
  MOG_LAUNCH_RET();
}

extern "C" int mog_recon_loss(const float* x, float* canvas, const float* parts, int nparts,
                              long part_stride, const int* part_rows, int C,
                              const float* runloss, const int* digits,
                              const int* targets, int B, int C2, float grad_scale, float* recon,
                              float* bce, float* mse, float* loss, float* acc, float* dcanvas,
                              void* stream) {
  MOG_CHECK_ARG(x && runloss && digits && bce && mse && loss && B >= 0 && C2 > 0);
  MOG_CHECK_ARG(nparts >= 0 &&
                (nparts > 0 ? parts != nullptr && part_stride >= (long)B * C2
                            : canvas != nullptr));
  MOG_CHECK_ARG(!part_rows || (nparts > 0 && C > 0 && C * C == C2 && (C2 % 4 != 0 || C % 2 == 0)));
  if (B == 0) return 0;
  if (C2 % 4 == 0)
    recon_loss_kernel<true><<<B, 256, 0, mog_stream(stream)>>>(
        x, canvas, parts, nparts, part_stride, part_rows, B, C, canvas, runloss, digits, targets, C2, grad_scale,
        recon, bce, mse, loss, acc, dcanvas);
  else
    recon_loss_kernel<false><<<B, 256, 0, mog_stream(stream)>>>(
        x, canvas, parts, nparts, part_stride, part_rows, B, C, canvas, runloss, digits, targets, C2, grad_scale,
        recon, bce, mse, loss, acc, dcanvas);
  MOG_LAUNCH_RET();
}

extern "C" int mog_batch_mean(const float* a0, const float* a1, const float* a2, const float* a3,
                              int B, float* out, void* stream) {
  MOG_CHECK_ARG(out && B > 0);
  batch_mean_kernel<<<1, 1024, 0, mog_stream(stream)>>>(a0, a1, a2, a3, B, 1.0f / (float)B, out);
  MOG_LAUNCH_RET();
}

extern "C" long mog_heads_output_wgrad_work_elems(int nheads, int R, int HS) {
  if (nheads < 1 || nheads > HO_MAXH || R < 0 || HS < 1 || HS > 127) return -1;
  return (long)nheads * mog_cdiv(R > 0 ? R : 1, HO_CH) * (2 * HS + 2);
}

extern "C" int mog_heads_output_wgrad(int nheads, const float* const* hid,
                                      const float* const* dout, float* const* gw,
                                      float* const* gb, const int* k, int R, int HS, float* work,
                                      long work_elems, void* stream) {
  MOG_CHECK_ARG(nheads >= 1 && nheads <= HO_MAXH && hid && dout && gw && k && work);
  MOG_CHECK_ARG(R >= 0 && HS >= 1 && HS <= 127);
  MOG_CHECK_ARG(work_elems >= mog_heads_output_wgrad_work_elems(nheads, R, HS));
  if (R == 0) return 0;
  HeadsOut a{};
  for (int z = 0; z < nheads; ++z) {
    MOG_CHECK_ARG(hid[z] && dout[z] && gw[z] && (k[z] == 1 || k[z] == 2));
    a.hid[z] = hid[z]; a.dout[z] = dout[z]; a.gw[z] = gw[z]; a.gb[z] = gb ? gb[z] : nullptr;
    a.k[z] = k[z];
  }
  a.R = R; a.HS = HS; a.S = (int)mog_cdiv(R, HO_CH); a.work = work;
  hipStream_t s = mog_stream(stream);
  heads_out_partial_kernel<<<dim3(a.S, nheads), 256, 0, s>>>(a);
  heads_out_reduce_kernel<<<nheads, 256, 0, s>>>(a);
  MOG_LAUNCH_RET();
}

extern "C" int mog_colsum_add(const float* X, int R, int N, int ld, float* out, void* stream) {
  MOG_CHECK_ARG(X && out && R >= 0 && N >= 0);
  if (R == 0 || N == 0) return 0;
  const int rpb = 256;
  dim3 g(mog_cdiv(N, 256), mog_cdiv(R, rpb));
  colsum_kernel<<<g, 256, 0, mog_stream(stream)>>>(X, R, N, ld, rpb, out);
  MOG_LAUNCH_RET();
}

extern "C" int mog_fill32_batch(int nbuf, void* const* dst, const long* n, const unsigned* value,
                                void* stream) {
  MOG_CHECK_ARG(nbuf >= 0 && nbuf <= FILL_MAX && (nbuf == 0 || (dst && n && value)));
  FillBatch f;
  long mx = 0;
  for (int j = 0; j < FILL_MAX; ++j) {
    const bool on = j < nbuf;
    f.dst[j] = on ? reinterpret_cast<unsigned*>(dst[j]) : nullptr;
    f.n[j] = on ? n[j] : 0;
    f.v[j] = on ? value[j] : 0u;
    if (on) {
      MOG_CHECK_ARG(dst[j] != nullptr && n[j] >= 0 && (reinterpret_cast<size_t>(dst[j]) & 3) == 0);
      mx = n[j] > mx ? n[j] : mx;
    }
  }
  if (nbuf == 0 || mx == 0) return 0;
  const long blocks = std::min<long>((long)mog_cdiv((mx + 3) / 4, 256), 2048);
  fill32_batch_kernel<<<dim3((unsigned)blocks, nbuf), 256, 0, mog_stream(stream)>>>(f);
  MOG_LAUNCH_RET();
}

extern "C" int mog_copy32_batch(int nbuf, void* const* dst, const void* const* src,
                                const long* n, void* stream) {
  MOG_CHECK_ARG(nbuf >= 0 && nbuf <= FILL_MAX && (nbuf == 0 || (dst && src && n)));
  CopyBatch f;
  long mx = 0;
  for (int j = 0; j < FILL_MAX; ++j) {
    const bool on = j < nbuf;
    f.dst[j] = on ? reinterpret_cast<unsigned*>(dst[j]) : nullptr;
    f.src[j] = on ? reinterpret_cast<const unsigned*>(src[j]) : nullptr;
    f.n[j] = on ? n[j] : 0;
    if (on) {
      MOG_CHECK_ARG(dst[j] && src[j] && n[j] >= 0 &&
                    ((reinterpret_cast<size_t>(dst[j]) | reinterpret_cast<size_t>(src[j])) & 3) == 0);
      mx = n[j] > mx ? n[j] : mx;
    }
  }
  if (nbuf == 0 || mx == 0) return 0;
  const long blocks = std::min<long>((long)mog_cdiv((mx + 3) / 4, 256), 2048);
  copy32_batch_kernel<<<dim3((unsigned)blocks, nbuf), 256, 0, mog_stream(stream)>>>(f);
  MOG_LAUNCH_RET();
}

extern "C" int mog_transpose32_batch(int nbuf, float* const* dst, const float* const* src,
                                     const int* rows, const int* cols, void* stream) {
  MOG_CHECK_ARG(nbuf >= 0 && nbuf <= FILL_MAX && (nbuf == 0 || (dst && src && rows && cols)));
  TransBatch f{};
  long mx = 0;
  for (int j = 0; j < nbuf; ++j) {
    MOG_CHECK_ARG(dst[j] && src[j] && rows[j] >= 0 && cols[j] >= 0);
    f.dst[j] = dst[j]; f.src[j] = src[j]; f.rows[j] = rows[j]; f.cols[j] = cols[j];
    mx = std::max<long>(mx, (long)rows[j] * cols[j]);
  }
  if (nbuf == 0 || mx == 0) return 0;
  const long blocks = std::min<long>((long)mog_cdiv(mx, 256), 1024);
  transpose32_batch_kernel<<<dim3((unsigned)blocks, nbuf), 256, 0, mog_stream(stream)>>>(f);
  MOG_LAUNCH_RET();
}

extern "C" int mog_add(const float* a, const float* b, float* out, long n, void* stream) {
  MOG_CHECK_ARG(a && b && out && n >= 0);
  if (n == 0) return 0;
  add_kernel<<<mog_cdiv(n, 256), 256, 0, mog_stream(stream)>>>(a, b, out, n);
  MOG_LAUNCH_RET();
}

extern "C" int mog_generation_prior(int G, int Z, float s_pm, float s_plv, float h_pm,
                                    float h_plv, float v_pm, float v_plv, const float* eps_scale,
                                    const float* eps_shift, const float* eps_z, float* theta_back,
                                    float* scale, float* shift, float* z, void* stream) {
  MOG_CHECK_ARG(G >= 0 && Z > 0 && eps_scale && eps_shift && eps_z && theta_back && scale &&
                shift && z);
  if (G == 0) return 0;
  gen_prior_kernel<<<mog_cdiv((long)G * Z, 256), 256, 0, mog_stream(stream)>>>(
      G, Z, s_pm, s_plv, h_pm, h_plv, v_pm, v_plv, eps_scale, eps_shift, eps_z, theta_back, scale,
      shift, z);
  MOG_LAUNCH_RET();
}
