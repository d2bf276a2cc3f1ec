/*
 * oracle/air_ref.c — TEST INFRASTRUCTURE ONLY.  CPU restatement (plain C,
 * fp32) of the reference AIR forward loop, used by tests/, smoke() and the
 * bench's cpu checks as the parity oracle.  The product path never links or
 * calls this file.
 *
 * Follows (reference = /root/reference, TF-1.12 semantics per SURVEY.md App. A):
 *   air/air_model.py:426-851   while-loop body (LSTM, heads, STN, VAE, z_pres,
 *                               masks, canvas, KLs) and loop condition :428-432
 *   air/air_model.py:866-900   clip, BCE, MSE, per-image loss, accuracy
 *   air/transformer.py:48-171  STN (_meshgrid, _transform, _interpolate)
 *   air/vae.py:5-48            glimpse VAE
 *   air/concrete.py:20-64      relaxed-Bernoulli sample and its MC KL
 *   TF-1.12 BasicLSTMCell      gate order i,j,f,o, forget_bias 1.0
 *
 * Arithmetic conventions (the parity contract):
 *   - every dense layer is matmul then bias_add: the dot product is ONE fp32
 *     fma chain in natural k order starting from +0, then "+ bias" rounded
 *     separately (what a k-ordered fp32 MFMA chain produces on gfx950);
 *   - the LSTM input is concat([x, h]) so the chain runs over x then h;
 *   - elementwise transcendentals come from include/mog_math.h;
 *   - every other op is one IEEE op per TF op, in the reference's order,
 *     compiled with -ffp-contract=off;
 *   - reductions (KL over latent dims, BCE/MSE over pixels) are sequential.
 * Parity against TF-1.12 itself is UNPINNED (TF absent, reference has no
 * tests or golden files).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mog_math.h"

typedef struct {
  int B, C, W, max_steps, H, Z, R1, R2, G1, G2, HS, HZ;
  int train;          /* 1: relaxed z_pres (train model); 0: rounded (test) */
  int use_num_prior;  /* -ap: marginal_objective bias + z_pres_kl_end */
  float lik_std, thr, temperature;
  float scale_prior_mean, scale_prior_var, scale_prior_logvar;
  float shift_prior_mean, shift_prior_var, shift_prior_logvar;
  float vae_prior_mean, vae_prior_var, vae_prior_logvar;
  float z_pres_prior_log_odds;
  const float* marginal_objective; /* [max_steps], used iff use_num_prior */
} AirCfg;

/* parameter slots, TF layout [in, out] row-major */
enum {
  P_LSTM_K, P_LSTM_B,
  P_SM_W1, P_SM_B1, P_SM_W2, P_SM_B2,
  P_SV_W1, P_SV_B1, P_SV_W2, P_SV_B2,
  P_HM_W1, P_HM_B1, P_HM_W2, P_HM_B2,
  P_HV_W1, P_HV_B1, P_HV_W2, P_HV_B2,
  P_R1_W, P_R1_B, P_R2_W, P_R2_B,
  P_MU_W, P_MU_B, P_LV_W, P_LV_B,
  P_G1_W, P_G1_B, P_G2_W, P_G2_B, P_GO_W, P_GO_B,
  P_Z_W1, P_Z_B1, P_Z_W2, P_Z_B2,
  P_COUNT
};

typedef struct {
  const float* eps_scale; /* [T,B]   */
  const float* eps_shift; /* [T,B,2] */
  const float* eps_z;     /* [T,B,Z] */
  const float* eps_x;     /* [T,B,W*W] */
  const float* u;         /* [T,B]   */
} AirNoise;

typedef struct {
  float *scale, *shift, *st_back, *window, *latent, *z_pres_prob;
  float *z_pres_kl, *scale_kl, *shift_kl, *vae_kl;
  float *glimpse, *z_pres, *mu, *logvar, *h;            /* debug/backward */
  float *canvas, *recon, *bce, *mse, *running_loss, *loss;
  int* digits;
} AirOut;

/* dense layer: out[b][n] = chain_k(in[b][k] w[k][n]) + bias[n] */
static void dense(const float* in, int B, int K, const float* w, const float* bias,
                  int N, float* out) {
  for (int b = 0; b < B; ++b)
    for (int n = 0; n < N; ++n) {
      float acc = 0.0f;
      const float* a = in + (size_t)b * K;
      for (int k = 0; k < K; ++k) acc = fmaf(a[k], w[(size_t)k * N + n], acc);
      out[(size_t)b * N + n] = acc + bias[n];
    }
}

static float relu(float x) { return x > 0.0f ? x : 0.0f; }

/* TF LinSpace: start + step*i, last element = stop (transformer.py:119-136) */
static float linspace_at(int i, int n) {
  if (n == 1) return -1.0f;
  if (i == n - 1) return 1.0f;
  const float step = 2.0f / (float)(n - 1);
  return -1.0f + step * (float)i;
}

/* STN for one image: U [Hin, Win] -> out [Hout, Wout] (transformer.py:48-171) */
void oracle_stn(const float* U, int Hin, int Win, const float th[6], int Hout, int Wout,
                float* out) {
  const float wm = (float)Win - 1.001f;
  const float hm = (float)Hin - 1.001f;
  for (int i = 0; i < Hout; ++i) {
    const float yt = linspace_at(i, Hout);
    for (int j = 0; j < Wout; ++j) {
      const float xt = linspace_at(j, Wout);
      /* T_g = theta @ [x_t, y_t, 1]  (:152-163) */
      const float xs = (th[0] * xt + th[1] * yt) + th[2] * 1.0f;
      const float ys = (th[3] * xt + th[4] * yt) + th[5] * 1.0f;
      /* (:75-76) */
      const float x = ((xs + 1.0f) * wm) / 2.0f;
      const float y = ((ys + 1.0f) * hm) / 2.0f;
      /* (:79-87) floor, +1, clip */
      float fx = floorf(x), fy = floorf(y);
      if (fx < -1073741824.0f) fx = -1073741824.0f;
      if (fx > 1073741824.0f) fx = 1073741824.0f;
      if (fy < -1073741824.0f) fy = -1073741824.0f;
      if (fy > 1073741824.0f) fy = 1073741824.0f;
      int x0 = (int)fx, y0 = (int)fy;
      int x1 = x0 + 1, y1 = y0 + 1;
      x0 = x0 < 0 ? 0 : (x0 > Win - 1 ? Win - 1 : x0);
      x1 = x1 < 0 ? 0 : (x1 > Win - 1 ? Win - 1 : x1);
      y0 = y0 < 0 ? 0 : (y0 > Hin - 1 ? Hin - 1 : y0);
      y1 = y1 < 0 ? 0 : (y1 > Hin - 1 ? Hin - 1 : y1);
      const float Ia = U[y0 * Win + x0], Ib = U[y1 * Win + x0];
      const float Ic = U[y0 * Win + x1], Id = U[y1 * Win + x1];
      const float x0f = (float)x0, x1f = (float)x1, y0f = (float)y0, y1f = (float)y1;
      /* (:108-116) */
      const float wa = (x1f - x) * (y1f - y);
      const float wb = (x1f - x) * (y - y0f);
      const float wc = (x - x0f) * (y1f - y);
      const float wd = (x - x0f) * (y - y0f);
      out[i * Wout + j] = ((wa * Ia + wb * Ib) + wc * Ic) + wd * Id;
    }
  }
}

/* reduce_logsumexp([0, a]) per TF-1.12 math_ops.reduce_logsumexp */
static float lse0(float a) {
  float m = a > 0.0f ? a : 0.0f;
  if (!(m - m == 0.0f)) m = 0.0f; /* non-finite max -> 0 */
  return mog_logf(mog_expf(0.0f - m) + mog_expf(a - m)) + m;
}

/* concrete.py:30-64 */
float oracle_concrete_kl(float y, float plo, float pT, float qlo, float qT) {
  const float eps = 1e-9f; /* 10e-10 */
  const float lse_p = lse0(-y * pT + plo);
  const float log_prior = ((mog_logf(pT + eps) - y * (pT + 1.0f)) + plo) - 2.0f * lse_p;
  const float lse_q = lse0(-y * qT + qlo);
  const float log_post = ((mog_logf(qT + eps) - y * (qT + 1.0f)) + qlo) - 2.0f * lse_q;
  return log_post - log_prior;
}

static float gauss_kl_term(float plv, float lv, float var, float pv, float mean, float pm) {
  const float d = mean - pm;
  return (((plv - lv) - 1.0f) + var / pv) + (d * d) / pv;
}

/* Runs the reference forward; returns the number of executed loop steps. */
int oracle_air_forward(const AirCfg* cfg, const float* const* P, const AirNoise* nz,
                       const float* images, const int* targets, AirOut* o,
                       float* accuracy_out) {
  const int B = cfg->B, C = cfg->C, W = cfg->W, T = cfg->max_steps, H = cfg->H;
  const int Z = cfg->Z, C2 = C * C, W2 = W * W, G4 = 4 * H;
  const float eps = 1e-9f;

  float* hbuf = (float*)calloc((size_t)B * H, 4);
  float* cbuf = (float*)calloc((size_t)B * H, 4);
  float* gates = (float*)malloc((size_t)B * G4 * 4);
  float* stop = (float*)calloc(B, 4);
  float* runloss = (float*)calloc(B, 4);
  int* digits = (int*)calloc(B, 4);
  float* canvas = (float*)calloc((size_t)B * C2, 4);
  float* hid = (float*)malloc((size_t)B * 64 * 4 * 8);
  float* tmp2 = (float*)malloc((size_t)B * 8 * 4);
  float* a1 = (float*)malloc((size_t)B * cfg->R1 * 4);
  float* a2 = (float*)malloc((size_t)B * cfg->R2 * 4);
  float* mu = (float*)malloc((size_t)B * Z * 4);
  float* lv = (float*)malloc((size_t)B * Z * 4);
  float* z = (float*)malloc((size_t)B * Z * 4);
  float* d1 = (float*)malloc((size_t)B * cfg->G1 * 4);
  float* d2 = (float*)malloc((size_t)B * cfg->G2 * 4);
  float* m = (float*)malloc((size_t)B * W2 * 4);
  float* g = (float*)malloc((size_t)B * W2 * 4);
  float* r = (float*)malloc((size_t)B * W2 * 4);
  float* wr = (float*)malloc((size_t)C2 * 4);
  float* sm = (float*)malloc(B * 4), *sv = (float*)malloc(B * 4);
  float* hm = (float*)malloc(B * 8), *hv = (float*)malloc(B * 8);
  float* lo = (float*)malloc(B * 4);

  int step = 0;
  for (;;) {
    /* cond (:428-432) */
    int any = 0;
    for (int b = 0; b < B; ++b) any |= stop[b] < cfg->thr;
    if (!(step < T && any)) break;

    /* LSTM (:454-456): gates = concat([x,h]) K + b; chain over x then h */
    const float* K = P[P_LSTM_K];
    for (int b = 0; b < B; ++b)
      for (int n = 0; n < G4; ++n) {
        float acc = 0.0f;
        for (int k = 0; k < C2; ++k)
          acc = fmaf(images[(size_t)b * C2 + k], K[(size_t)k * G4 + n], acc);
        for (int k = 0; k < H; ++k)
          acc = fmaf(hbuf[(size_t)b * H + k], K[(size_t)(C2 + k) * G4 + n], acc);
        gates[(size_t)b * G4 + n] = acc + P[P_LSTM_B][n];
      }
    for (int b = 0; b < B; ++b)
      for (int u = 0; u < H; ++u) {
        const float* gr = gates + (size_t)b * G4;
        const float gi = gr[u], gj = gr[H + u], gf = gr[2 * H + u], go = gr[3 * H + u];
        const float c0 = cbuf[(size_t)b * H + u];
        const float nc = c0 * mog_sigmoidf(gf + 1.0f) + mog_sigmoidf(gi) * mog_tanhf(gj);
        cbuf[(size_t)b * H + u] = nc;
        hbuf[(size_t)b * H + u] = mog_tanhf(nc) * mog_sigmoidf(go);
      }
    if (o->h) memcpy(o->h + (size_t)step * B * H, hbuf, (size_t)B * H * 4);

    /* heads (:458-498) : fc(relu) 64 -> fc */
    const int HS = cfg->HS, HZ = cfg->HZ;
    dense(hbuf, B, H, P[P_SM_W1], P[P_SM_B1], HS, hid);
    for (int i = 0; i < B * HS; ++i) hid[i] = relu(hid[i]);
    dense(hid, B, HS, P[P_SM_W2], P[P_SM_B2], 1, sm);
    dense(hbuf, B, H, P[P_SV_W1], P[P_SV_B1], HS, hid);
    for (int i = 0; i < B * HS; ++i) hid[i] = relu(hid[i]);
    dense(hid, B, HS, P[P_SV_W2], P[P_SV_B2], 1, sv);
    dense(hbuf, B, H, P[P_HM_W1], P[P_HM_B1], HS, hid);
    for (int i = 0; i < B * HS; ++i) hid[i] = relu(hid[i]);
    dense(hid, B, HS, P[P_HM_W2], P[P_HM_B2], 2, hm);
    dense(hbuf, B, H, P[P_HV_W1], P[P_HV_B1], HS, hid);
    for (int i = 0; i < B * HS; ++i) hid[i] = relu(hid[i]);
    dense(hid, B, HS, P[P_HV_W2], P[P_HV_B2], 2, hv);
    dense(hbuf, B, H, P[P_Z_W1], P[P_Z_B1], HZ, hid);
    for (int i = 0; i < B * HZ; ++i) hid[i] = relu(hid[i]);
    dense(hid, B, HZ, P[P_Z_W2], P[P_Z_B2], 1, lo);

    for (int b = 0; b < B; ++b) {
      const size_t tb = (size_t)step * B + b;
      /* scale (:471-477), _sample_from_mvn (:186-192) */
      const float svar = mog_expf(sv[b]);
      const float s = mog_sigmoidf(sm[b] + nz->eps_scale[tb] * sqrtf(svar));
      /* shift (:492-498) */
      float sh[2], shvar[2];
      for (int d = 0; d < 2; ++d) {
        shvar[d] = mog_expf(hv[b * 2 + d]);
        sh[d] = mog_tanhf(hm[b * 2 + d] + nz->eps_shift[tb * 2 + d] * sqrtf(shvar[d]));
      }
      const float tx = sh[0], ty = sh[1];
      o->scale[tb] = s;
      o->shift[tb * 2] = tx;
      o->shift[tb * 2 + 1] = ty;
      /* READ (:500-531) */
      const float th[6] = {s, 0.0f, tx, 0.0f, s, ty};
      oracle_stn(images + (size_t)b * C2, C, C, th, W, W, g + (size_t)b * W2);
      /* theta_recon (:552-572) */
      const float is = 1.0f / s;
      float* stb = o->st_back + tb * 6;
      stb[0] = is; stb[1] = 0.0f; stb[2] = -tx / s;
      stb[3] = 0.0f; stb[4] = is; stb[5] = -ty / s;
      (void)svar;
    }

    /* VAE (vae.py:5-48) */
    dense(g, B, W2, P[P_R1_W], P[P_R1_B], cfg->R1, a1);
    for (int i = 0; i < B * cfg->R1; ++i) a1[i] = mog_softplusf(a1[i]);
    dense(a1, B, cfg->R1, P[P_R2_W], P[P_R2_B], cfg->R2, a2);
    for (int i = 0; i < B * cfg->R2; ++i) a2[i] = mog_softplusf(a2[i]);
    dense(a2, B, cfg->R2, P[P_MU_W], P[P_MU_B], Z, mu);
    dense(a2, B, cfg->R2, P[P_LV_W], P[P_LV_B], Z, lv);
    for (int i = 0; i < B * Z; ++i)
      z[i] = mu[i] + nz->eps_z[(size_t)step * B * Z + i] * sqrtf(mog_expf(lv[i]));
    dense(z, B, Z, P[P_G1_W], P[P_G1_B], cfg->G1, d1);
    for (int i = 0; i < B * cfg->G1; ++i) d1[i] = mog_softplusf(d1[i]);
    dense(d1, B, cfg->G1, P[P_G2_W], P[P_G2_B], cfg->G2, d2);
    for (int i = 0; i < B * cfg->G2; ++i) d2[i] = mog_softplusf(d2[i]);
    dense(d2, B, cfg->G2, P[P_GO_W], P[P_GO_B], W2, m);
    for (int i = 0; i < B * W2; ++i)
      r[i] = mog_sigmoidf(m[i] + nz->eps_x[(size_t)step * B * W2 + i] * cfg->lik_std);

    for (int b = 0; b < B; ++b) {
      const size_t tb = (size_t)step * B + b;
      memcpy(o->window + tb * W2, r + (size_t)b * W2, W2 * 4);
      memcpy(o->latent + tb * Z, z + (size_t)b * Z, Z * 4);
      if (o->glimpse) memcpy(o->glimpse + tb * W2, g + (size_t)b * W2, W2 * 4);
      if (o->mu) memcpy(o->mu + tb * Z, mu + (size_t)b * Z, Z * 4);
      if (o->logvar) memcpy(o->logvar + tb * Z, lv + (size_t)b * Z, Z * 4);

      /* WRITE (:580-588) */
      oracle_stn(r + (size_t)b * W2, W, W, o->st_back + tb * 6, C, C, wr);

      /* z_pres (:590-620) */
      const float noise = mog_logf(nz->u[tb] + eps) - mog_logf((1.0f - nz->u[tb]) + eps);
      const float y = (lo[b] + noise) / cfg->temperature;
      float zp = mog_sigmoidf(y);
      if (!cfg->train) zp = rintf(zp);
      o->z_pres_prob[tb] = mog_sigmoidf(lo[b]);
      if (o->z_pres) o->z_pres[tb] = zp;

      /* z_pres KL with OLD stopping sum (:622-653) */
      float bias = 0.0f, kl_end = 0.0f;
      if (cfg->use_num_prior) {
        bias = cfg->marginal_objective[step];
        kl_end = oracle_concrete_kl(y, -100.0f, cfg->temperature, lo[b], cfg->temperature);
      }
      const float zkl = oracle_concrete_kl(y, cfg->z_pres_prior_log_odds + bias,
                                           cfg->temperature, lo[b], cfg->temperature);
      runloss[b] = runloss[b] + (stop[b] < cfg->thr ? zkl : kl_end);
      o->z_pres_kl[tb] = zkl;

      /* stop / digits / canvas (:659-675) */
      stop[b] = stop[b] + (1.0f - zp);
      const int active = stop[b] < cfg->thr;
      digits[b] += active;
      float* cv = canvas + (size_t)b * C2;
      if (active)
        for (int p = 0; p < C2; ++p) cv[p] = cv[p] + zp * wr[p];

      /* KLs with NEW stopping sum (:677-736) */
      const float slv = sv[b];
      const float skl = 0.5f * gauss_kl_term(cfg->scale_prior_logvar, slv, mog_expf(slv),
                                             cfg->scale_prior_var, sm[b], cfg->scale_prior_mean);
      if (active) runloss[b] = runloss[b] + skl;
      o->scale_kl[tb] = skl;
      float shs = 0.0f;
      for (int d = 0; d < 2; ++d) {
        const float hlv = hv[b * 2 + d];
        shs = shs + gauss_kl_term(cfg->shift_prior_logvar, hlv, mog_expf(hlv),
                                  cfg->shift_prior_var, hm[b * 2 + d], cfg->shift_prior_mean);
      }
      const float shkl = 0.5f * shs;
      if (active) runloss[b] = runloss[b] + shkl;
      o->shift_kl[tb] = shkl;
      float vs = 0.0f;
      for (int d = 0; d < Z; ++d) {
        const float l = lv[(size_t)b * Z + d];
        vs = vs + gauss_kl_term(cfg->vae_prior_logvar, l, mog_expf(l), cfg->vae_prior_var,
                                mu[(size_t)b * Z + d], cfg->vae_prior_mean);
      }
      const float vkl = 0.5f * vs;
      if (active) runloss[b] = runloss[b] + vkl;
      o->vae_kl[tb] = vkl;
    }
    ++step;
  }

  /* loss (:866-900) */
  double accsum = 0.0;
  for (int b = 0; b < B; ++b) {
    float bce = 0.0f, mse = 0.0f;
    for (int p = 0; p < C2; ++p) {
      const float c = canvas[(size_t)b * C2 + p];
      const float rc = fmaxf(fminf(c, 1.0f), 0.0f);
      const float x = images[(size_t)b * C2 + p];
      const float t = x * mog_logf(rc + 1e-10f) + (1.0f - x) * mog_logf((1.0f - rc) + 1e-10f);
      bce = bce + t;
      const float dx = x - rc;
      mse = mse + dx * dx;
      o->canvas[(size_t)b * C2 + p] = c;
      o->recon[(size_t)b * C2 + p] = rc;
    }
    o->bce[b] = -bce;
    o->mse[b] = mse;
    o->running_loss[b] = runloss[b];
    o->loss[b] = runloss[b] + (-bce);
    o->digits[b] = digits[b];
    accsum += (targets && targets[b] == digits[b]) ? 1.0 : 0.0;
  }
  if (accuracy_out) *accuracy_out = (float)(accsum / B);

  free(hbuf); free(cbuf); free(gates); free(stop); free(runloss); free(digits);
  free(canvas); free(hid); free(tmp2); free(a1); free(a2); free(mu); free(lv); free(z);
  free(d1); free(d2); free(m); free(g); free(r); free(wr); free(sm); free(sv); free(hm);
  free(hv); free(lo);
  return step;
}

/* vectorised wrappers so tests can pin mog_math.h against libm */
/* Generation loop (air_model.py:1001-1146, vae.py:51-86), test model: for
 * n_steps steps, scale ~ sigmoid(N(scale prior)), shift ~ tanh(N(shift
 * prior)) (_sample_from_mvn, :186-192), z ~ N(vae prior), r = sigmoid(decoder
 * + std eps_x), and the canvas adds every step's STN-written window
 * unweighted (the stopping sum stays 0 < thr, :1085-1097).  Noise slots
 * eps_scale [T,G], eps_shift [T,G,2], eps_z [T,G,Z], eps_x [T,G,W*W]. */
int oracle_air_generate(const AirCfg* cfg, const float* const* P, const AirNoise* nz, int G,
                        int n_steps, float* canvas, float* st_back) {
  const int C = cfg->C, W = cfg->W, C2 = C * C, W2 = W * W, Z = cfg->Z;
  float* z = (float*)calloc((size_t)G * Z, 4);
  float* d1 = (float*)calloc((size_t)G * cfg->G1, 4);
  float* d2 = (float*)calloc((size_t)G * cfg->G2, 4);
  float* m = (float*)calloc((size_t)G * W2, 4);
  float* wr = (float*)calloc((size_t)C2, 4);
  memset(canvas, 0, (size_t)G * C2 * 4);
  for (int step = 0; step < n_steps; ++step) {
    const float svar = mog_expf(cfg->scale_prior_logvar);
    const float hvar = mog_expf(cfg->shift_prior_logvar);
    const float zvar = mog_expf(cfg->vae_prior_logvar);
    for (int i = 0; i < G * Z; ++i)
      z[i] = cfg->vae_prior_mean + nz->eps_z[(size_t)step * G * Z + i] * sqrtf(zvar);
    dense(z, G, Z, P[P_G1_W], P[P_G1_B], cfg->G1, d1);
    for (int i = 0; i < G * cfg->G1; ++i) d1[i] = mog_softplusf(d1[i]);
    dense(d1, G, cfg->G1, P[P_G2_W], P[P_G2_B], cfg->G2, d2);
    for (int i = 0; i < G * cfg->G2; ++i) d2[i] = mog_softplusf(d2[i]);
    dense(d2, G, cfg->G2, P[P_GO_W], P[P_GO_B], W2, m);
    for (int i = 0; i < G * W2; ++i)
      m[i] = mog_sigmoidf(m[i] + nz->eps_x[(size_t)step * G * W2 + i] * cfg->lik_std);
    for (int b = 0; b < G; ++b) {
      const size_t tb = (size_t)step * G + b;
      const float s = mog_sigmoidf(cfg->scale_prior_mean + nz->eps_scale[tb] * sqrtf(svar));
      const float tx = mog_tanhf(cfg->shift_prior_mean + nz->eps_shift[tb * 2] * sqrtf(hvar));
      const float ty = mog_tanhf(cfg->shift_prior_mean + nz->eps_shift[tb * 2 + 1] * sqrtf(hvar));
      float* stb = st_back + tb * 6;
      stb[0] = 1.0f / s; stb[1] = 0.0f; stb[2] = -tx / s;
      stb[3] = 0.0f; stb[4] = 1.0f / s; stb[5] = -ty / s;
      oracle_stn(m + (size_t)b * W2, W, W, stb, C, C, wr);
      float* cv = canvas + (size_t)b * C2;
      for (int p = 0; p < C2; ++p) cv[p] = cv[p] + wr[p];
    }
  }
  free(z); free(d1); free(d2); free(m); free(wr);
  return n_steps;
}

void oracle_math_vec(int fn, const float* x, float* y, int n) {
  for (int i = 0; i < n; ++i) {
    switch (fn) {
      case 0: y[i] = mog_expf(x[i]); break;
      case 1: y[i] = mog_logf(x[i]); break;
      case 2: y[i] = mog_expm1f(x[i]); break;
      case 3: y[i] = mog_tanhf(x[i]); break;
      case 4: y[i] = mog_sigmoidf(x[i]); break;
      case 6: y[i] = mog_log1pf(x[i]); break;
      default: y[i] = mog_softplusf(x[i]); break;
    }
  }
}

/* exported k-ordered dense layer (parity check of the MFMA GEMM) */
void oracle_dense(const float* in, int B, int K, const float* w, const float* bias, int N,
                  float* out) {
  static const float zero = 0.0f;
  (void)zero;
  if (bias) {
    dense(in, B, K, w, bias, N, out);
  } else {
    for (int b = 0; b < B; ++b)
      for (int n = 0; n < N; ++n) {
        float acc = 0.0f;
        for (int k = 0; k < K; ++k) acc = fmaf(in[(size_t)b * K + k], w[(size_t)k * N + n], acc);
        out[(size_t)b * N + n] = acc;
      }
  }
}
