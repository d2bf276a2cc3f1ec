/*
 * oracle/asr_ref.c — TEST INFRASTRUCTURE ONLY.  CPU restatement (plain C,
 * fp32, -ffp-contract=off) of the AIR-ASR forward pass with its structural
 * regularisers, the parity oracle of the HIP ASR path (mog_air/asr_model.py).
 *
 * Follows air/air_number_bbox_location.py (reference = /root/reference):
 *   :384-777   while-loop body: inference LSTMCell on [x, z_prev, ss_prev],
 *              shift heads, scale heads on [h, shift_latent], generative
 *              LSTMCell on [z_prev, ss_prev] with learned shift prior and
 *              fixed scale prior, STN read / VAE / STN write, learned (or
 *              fix_steps) z_pres prior from the previous generative output,
 *              entropy regulariser, masks, KLs; loop predicate :386-390
 *   :917-1079  per-type KL sums, reconstruction, margin / element number
 *              losses on the (batch-mean) z_pres probabilities, area, bbox
 *              out / size / overlap losses, total loss
 * Same arithmetic conventions as air_ref.c (k-ordered fma chains for dense
 * layers, mog_math.h transcendentals, one IEEE op per TF op, sequential
 * reductions; TF's reduce_sum over the <= max_steps step records is taken
 * in step order).  Parity against TF-1.12 itself is UNPINNED.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mog_math.h"

void oracle_stn(const float* U, int Hin, int Win, const float th[6], int Hout, int Wout,
                float* out);
float oracle_concrete_kl(float y, float plo, float pT, float qlo, float qT);

typedef struct {
  int B, C, W, max_steps, H, Z, R1, R2, G1, G2, HS, HZ;
  int train, fix_steps; /* fix_steps < 0: learned z_pres prior */
  int n_constrains;
  int constrains[8];
  float lik_std, thr, temperature;
  float scale_prior_mean, scale_prior_var, scale_prior_logvar;
  float vae_prior_mean, vae_prior_var, vae_prior_logvar;
  float g_num, g_margin, g_element, g_bbox, g_size, g_area, area_min, area_max;
} AsrCfg;

/* parameter slots, TF layout [in, out] */
enum {
  A_INF_K, A_INF_B, A_GEN_K, A_GEN_B,
  A_IS_W0, A_IS_B0, A_IS_W1, A_IS_B1, A_IS_W2, A_IS_B2, A_IS_W3, A_IS_B3, /* inf_shift */
  A_IC_W0, A_IC_B0, A_IC_W1, A_IC_B1, A_IC_W2, A_IC_B2, A_IC_W3, A_IC_B3, /* inf_scale */
  A_GS_W0, A_GS_B0, A_GS_W1, A_GS_B1, A_GS_W2, A_GS_B2, A_GS_W3, A_GS_B3, /* gen_shift */
  A_ZP_W0, A_ZP_B0, A_ZP_W1, A_ZP_B1,                                     /* z_pres prior */
  A_ZL_W0, A_ZL_B0, A_ZL_W1, A_ZL_B1,                                     /* z_pres log-odds */
  A_R1_W, A_R1_B, A_R2_W, A_R2_B, A_MU_W, A_MU_B, A_LV_W, A_LV_B,
  A_G1_W, A_G1_B, A_G2_W, A_G2_B, A_GO_W, A_GO_B,
  A_COUNT
};

typedef struct {
  const float *eps_shift, *eps_scale, *eps_z, *eps_x, *u; /* [T,B,2] [T,B] [T,B,Z] [T,B,W2] [T,B] */
} AsrNoise;

typedef struct {
  float *scale, *shift, *st_back, *window, *latent, *z_pres_prob, *z_pres;   /* [T,B,.] */
  float *z_pres_kl, *scale_kl, *shift_kl, *vae_kl, *pr_num;                  /* [T,B] masked */
  float *canvas, *bce, *mse, *elbo, *pr_loss, *element, *loss;               /* [B,...] */
  float *area, *out, *size, *overlap;                                        /* [B] */
  float* margin;                                                             /* [1] */
  int* digits;
} AsrOut;

/* out[n] = chain_k(x[k] w[k][n]) over the concatenation of up to 4 input
 * segments (TF dense / LSTMCell on tf.concat), then + bias[n] */
static void dense_cat(const float* const* seg, const int* len, int nseg, const float* w, const float* bias,
                      int N, float* out) {
  for (int n = 0; n < N; ++n) {
    float acc = 0.0f;
    int k = 0;
    for (int s = 0; s < nseg; ++s)
      for (int i = 0; i < len[s]; ++i, ++k) acc = fmaf(seg[s][i], w[(size_t)k * N + n], acc);
    out[n] = bias ? acc + bias[n] : acc;
  }
}

static float relu(float x) { return x > 0.0f ? x : 0.0f; }

static void lstm(const float* gates, float* c, float* h, int H) {
  for (int u = 0; u < H; ++u) {
    const float gi = gates[u], gj = gates[H + u], gf = gates[2 * H + u], go = gates[3 * H + u];
    const float nc = c[u] * mog_sigmoidf(gf + 1.0f) + mog_sigmoidf(gi) * mog_tanhf(gj);
    c[u] = nc;
    h[u] = mog_tanhf(nc) * mog_sigmoidf(go);
  }
}

/* tf.nn.sigmoid_cross_entropy_with_logits: max(x,0) - x z + log(1 + exp(-|x|)) */
static float sigmoid_ce(float z, float x) {
  const float ax = x < 0.0f ? -x : x;
  return ((x > 0.0f ? x : 0.0f) - x * z) + mog_log1pf(mog_expf(-ax));
}

static float logit8(float p) { return mog_logf(p + 1e-8f) - mog_logf((1.0f - p) + 1e-8f); }

int oracle_asr_forward(const AsrCfg* cfg, const float* const* P, const AsrNoise* nz,
                       const float* images, const int* targets, AsrOut* o, float* acc_out) {
  const int B = cfg->B, C = cfg->C, W = cfg->W, T = cfg->max_steps, H = cfg->H, Z = cfg->Z;
  const int C2 = C * C, W2 = W * W, HS = cfg->HS, HZ = cfg->HZ;
  const float eps = 1e-9f;
  float* h = calloc((size_t)B * H, 4);
  float* c = calloc((size_t)B * H, 4);
  float* hg = calloc((size_t)B * H, 4);
  float* cg = calloc((size_t)B * H, 4);
  float* hg_prev = calloc((size_t)B * H, 4);  /* gen_prev_output */
  float* zprev = calloc((size_t)B * Z, 4);
  float* ssprev = calloc((size_t)B * 3, 4);
  float* znew = calloc((size_t)B * Z, 4);
  float* ssnew = calloc((size_t)B * 3, 4);
  float* stop = calloc(B, 4);
  float* canvas = calloc((size_t)B * C2, 4);
  float* gates = calloc(4 * H, 4);
  float* hid = calloc(HS > HZ ? HS : HZ, 4);
  float* hid2 = calloc(HS > HZ ? HS : HZ, 4);
  float* g = calloc(W2, 4);
  float* a1 = calloc(cfg->R1, 4);
  float* a2 = calloc(cfg->R2, 4);
  float* mu = calloc(Z, 4);
  float* lv = calloc(Z, 4);
  float* d1 = calloc(cfg->G1, 4);
  float* d2 = calloc(cfg->G2, 4);
  float* r = calloc(W2, 4);
  float* wr = calloc(C2, 4);
  memset(o->digits, 0, (size_t)B * 4);
  const float gclv = cfg->scale_prior_logvar, gcvar = cfg->scale_prior_var;
  const float gcm = cfg->scale_prior_mean;
  int step = 0;
  for (; step < T; ++step) {
    int any = 0;
    for (int b = 0; b < B; ++b) any |= stop[b] < cfg->thr;
    if (!any) break;
    for (int b = 0; b < B; ++b) {
      const size_t tb = (size_t)step * B + b;
      float* hb = h + (size_t)b * H;
      float* hgb = hg + (size_t)b * H;
      const float* zp = zprev + (size_t)b * Z;
      const float* sp = ssprev + (size_t)b * 3;
      /* inference LSTMCell on concat([x, z_prev, ss_prev]) (:403-412) */
      {
        const float* seg[4] = {images + (size_t)b * C2, zp, sp, hb};
        const int len[4] = {C2, Z, 3, H};
        dense_cat(seg, len, 4, P[A_INF_K], P[A_INF_B], 4 * H, gates);
        lstm(gates, c + (size_t)b * H, hb, H);
      }
      /* inf_shift (:414-427) */
      float sm[2], slv[2], svar[2], sl[2];
      {
        const float* seg[1] = {hb};
        const int len[1] = {H};
        dense_cat(seg, len, 1, P[A_IS_W0], P[A_IS_B0], HS, hid);
        for (int i = 0; i < HS; ++i) hid[i] = relu(hid[i]);
        const float* s2[1] = {hid};
        const int l2[1] = {HS};
        dense_cat(s2, l2, 1, P[A_IS_W1], P[A_IS_B1], 2, sm);
        dense_cat(seg, len, 1, P[A_IS_W2], P[A_IS_B2], HS, hid);
        for (int i = 0; i < HS; ++i) hid[i] = relu(hid[i]);
        dense_cat(s2, l2, 1, P[A_IS_W3], P[A_IS_B3], 2, slv);
        for (int d = 0; d < 2; ++d) {
          svar[d] = mog_expf(slv[d]);
          sl[d] = sm[d] + nz->eps_shift[tb * 2 + d] * sqrtf(svar[d]);
        }
      }
      const float tx = mog_tanhf(sl[0]), ty = mog_tanhf(sl[1]);
      /* inf_scale on concat([h, shift_latent]) (:429-452) */
      float cm, clv, cvar, cl;
      {
        const float* seg[2] = {hb, sl};
        const int len[2] = {H, 2};
        dense_cat(seg, len, 2, P[A_IC_W0], P[A_IC_B0], HS, hid);
        for (int i = 0; i < HS; ++i) hid[i] = relu(hid[i]);
        const float* s2[2] = {hid, sl};
        const int l2[2] = {HS, 2};
        dense_cat(s2, l2, 2, P[A_IC_W1], P[A_IC_B1], 1, &cm);
        dense_cat(seg, len, 2, P[A_IC_W2], P[A_IC_B2], HS, hid);
        for (int i = 0; i < HS; ++i) hid[i] = relu(hid[i]);
        dense_cat(s2, l2, 2, P[A_IC_W3], P[A_IC_B3], 1, &clv);
        cvar = mog_expf(clv);
        cl = cm + nz->eps_scale[tb] * sqrtf(cvar);
      }
      const float s = mog_sigmoidf(cl);
      ssnew[b * 3] = sl[0];
      ssnew[b * 3 + 1] = sl[1];
      ssnew[b * 3 + 2] = cl;
      /* generative LSTMCell on concat([z_prev, ss_prev]) (:457-463) */
      {
        const float* seg[3] = {zp, sp, hgb};
        const int len[3] = {Z, 3, H};
        dense_cat(seg, len, 3, P[A_GEN_K], P[A_GEN_B], 4 * H, gates);
        lstm(gates, cg + (size_t)b * H, hgb, H);
      }
      /* gen_shift (:465-474); fixed scale prior (:502-505) */
      float gsm[2], gslv[2];
      {
        const float* seg[1] = {hgb};
        const int len[1] = {H};
        dense_cat(seg, len, 1, P[A_GS_W0], P[A_GS_B0], HS, hid);
        for (int i = 0; i < HS; ++i) hid[i] = relu(hid[i]);
        const float* s2[1] = {hid};
        const int l2[1] = {HS};
        dense_cat(s2, l2, 1, P[A_GS_W1], P[A_GS_B1], 2, gsm);
        dense_cat(seg, len, 1, P[A_GS_W2], P[A_GS_B2], HS, hid);
        for (int i = 0; i < HS; ++i) hid[i] = relu(hid[i]);
        dense_cat(s2, l2, 1, P[A_GS_W3], P[A_GS_B3], 2, gslv);
      }
      o->scale[tb] = s;
      o->shift[tb * 2] = tx;
      o->shift[tb * 2 + 1] = ty;
      /* STN read, VAE (vae.py:5-48), STN write (:507-588) */
      const float th[6] = {s, 0.0f, tx, 0.0f, s, ty};
      oracle_stn(images + (size_t)b * C2, C, C, th, W, W, g);
      {
        const float* sg[1] = {g};
        int ln[1] = {W2};
        dense_cat(sg, ln, 1, P[A_R1_W], P[A_R1_B], cfg->R1, a1);
        for (int i = 0; i < cfg->R1; ++i) a1[i] = mog_softplusf(a1[i]);
        sg[0] = a1; ln[0] = cfg->R1;
        dense_cat(sg, ln, 1, P[A_R2_W], P[A_R2_B], cfg->R2, a2);
        for (int i = 0; i < cfg->R2; ++i) a2[i] = mog_softplusf(a2[i]);
        sg[0] = a2; ln[0] = cfg->R2;
        dense_cat(sg, ln, 1, P[A_MU_W], P[A_MU_B], Z, mu);
        dense_cat(sg, ln, 1, P[A_LV_W], P[A_LV_B], Z, lv);
        float* zb = znew + (size_t)b * Z;
        for (int i = 0; i < Z; ++i) zb[i] = mu[i] + nz->eps_z[tb * Z + i] * sqrtf(mog_expf(lv[i]));
        sg[0] = zb; ln[0] = Z;
        dense_cat(sg, ln, 1, P[A_G1_W], P[A_G1_B], cfg->G1, d1);
        for (int i = 0; i < cfg->G1; ++i) d1[i] = mog_softplusf(d1[i]);
        sg[0] = d1; ln[0] = cfg->G1;
        dense_cat(sg, ln, 1, P[A_G2_W], P[A_G2_B], cfg->G2, d2);
        for (int i = 0; i < cfg->G2; ++i) d2[i] = mog_softplusf(d2[i]);
        sg[0] = d2; ln[0] = cfg->G2;
        dense_cat(sg, ln, 1, P[A_GO_W], P[A_GO_B], W2, r);
        for (int i = 0; i < W2; ++i)
          r[i] = mog_sigmoidf(r[i] + nz->eps_x[tb * W2 + i] * cfg->lik_std);
        memcpy(o->window + tb * W2, r, W2 * 4);
        memcpy(o->latent + tb * Z, zb, Z * 4);
      }
      float* stb = o->st_back + tb * 6;
      stb[0] = 1.0f / s; stb[1] = 0.0f; stb[2] = -tx / s;
      stb[3] = 0.0f; stb[4] = 1.0f / s; stb[5] = -ty / s;
      oracle_stn(r, W, W, stb, C, C, wr);
      /* z_pres prior (:590-602) and log-odds (:604-609) */
      float plo, lo;
      if (cfg->fix_steps >= 0) {
        plo = step < cfg->fix_steps ? 100.0f : -100.0f;
      } else {
        const float* seg[1] = {hg_prev + (size_t)b * H};
        const int len[1] = {H};
        dense_cat(seg, len, 1, P[A_ZP_W0], P[A_ZP_B0], HZ, hid2);
        for (int i = 0; i < HZ; ++i) hid2[i] = relu(hid2[i]);
        const float* s2[1] = {hid2};
        const int l2[1] = {HZ};
        dense_cat(s2, l2, 1, P[A_ZP_W1], P[A_ZP_B1], 1, &plo);
      }
      {
        const float* seg[1] = {hb};
        const int len[1] = {H};
        dense_cat(seg, len, 1, P[A_ZL_W0], P[A_ZL_B0], HZ, hid2);
        for (int i = 0; i < HZ; ++i) hid2[i] = relu(hid2[i]);
        const float* s2[1] = {hid2};
        const int l2[1] = {HZ};
        dense_cat(s2, l2, 1, P[A_ZL_W1], P[A_ZL_B1], 1, &lo);
      }
      const float noise = mog_logf(nz->u[tb] + eps) - mog_logf((1.0f - nz->u[tb]) + eps);
      const float y = (lo + noise) / cfg->temperature;
      float zp_ = mog_sigmoidf(y);
      if (!cfg->train) zp_ = rintf(zp_);
      const float zprob = mog_sigmoidf(lo);
      o->z_pres_prob[tb] = zprob;
      o->z_pres[tb] = zp_;
      /* entropy regulariser (:660-668), every executed step */
      float prn = 0.0f;
      if (cfg->g_num > 1e-8f) {
        const float ent = zprob * mog_softplusf(-1.0f * lo) + (1.0f - zprob) * mog_softplusf(lo);
        prn = ent * cfg->g_num;
      }
      o->pr_num[tb] = prn;
      /* z_pres KL with the OLD stopping sum (:688-703) */
      const float zkl = oracle_concrete_kl(y, plo, cfg->temperature, lo, cfg->temperature);
      o->z_pres_kl[tb] = stop[b] < cfg->thr ? zkl : 0.0f;
      /* stop / digits / canvas (:709-726) */
      stop[b] = stop[b] + (1.0f - zp_);
      const int act = stop[b] < cfg->thr;
      o->digits[b] += act;
      float* cv = canvas + (size_t)b * C2;
      if (act)
        for (int p = 0; p < C2; ++p) cv[p] = cv[p] + zp_ * wr[p];
      /* scale / shift / VAE KLs with the NEW stopping sum (:728-772) */
      const float dc = cm - gcm;
      const float skl = 0.5f * ((((gclv - clv) - 1.0f) + cvar / gcvar) + (dc * dc) / gcvar);
      o->scale_kl[tb] = act ? skl : 0.0f;
      float shs = 0.0f;
      for (int d = 0; d < 2; ++d) {
        const float gv = mog_expf(gslv[d]);
        const float dd = sm[d] - gsm[d];
        shs = shs + ((((gslv[d] - slv[d]) - 1.0f) + svar[d] / gv) + (dd * dd) / gv);
      }
      o->shift_kl[tb] = act ? 0.5f * shs : 0.0f;
      float vs = 0.0f;
      for (int k = 0; k < Z; ++k) {
        const float dm = mu[k] - cfg->vae_prior_mean;
        vs = vs + ((((cfg->vae_prior_logvar - lv[k]) - 1.0f) + mog_expf(lv[k]) / cfg->vae_prior_var) +
                   (dm * dm) / cfg->vae_prior_var);
      }
      o->vae_kl[tb] = act ? 0.5f * vs : 0.0f;
    }
    /* carry to the next step */
    memcpy(zprev, znew, (size_t)B * Z * 4);
    memcpy(ssprev, ssnew, (size_t)B * 3 * 4);
    memcpy(hg_prev, hg, (size_t)B * H * 4);
  }
  const int Tx = step;
  /* batch-mean z_pres probability per step and the margin loss (:970-998) */
  float margin = 0.0f;
  float mo[16];
  const int NC = cfg->n_constrains;
  if (cfg->g_margin > 1e-8f) {
    for (int t = 0; t < Tx; ++t) {
      float cnt = 0.0f;
      for (int k = 0; k < NC; ++k) cnt = cnt + (t < cfg->constrains[k] ? 1.0f : 0.0f);
      mo[t] = cnt / (float)NC;
      float pm = 0.0f;
      for (int b = 0; b < B; ++b) pm = pm + o->z_pres_prob[(size_t)t * B + b];
      pm = pm / (float)B;
      margin = margin + sigmoid_ce(mo[t], logit8(pm)) * cfg->g_margin;
    }
  }
  *o->margin = margin;
  float acc = 0.0f;
  for (int b = 0; b < B; ++b) {
    const float* x = images + (size_t)b * C2;
    const float* cv = canvas + (size_t)b * C2;
    float bce = 0.0f, mse = 0.0f;
    for (int p = 0; p < C2; ++p) {
      const float rc = fmaxf(fminf(cv[p], 1.0f), 0.0f);
      o->canvas[(size_t)b * C2 + p] = cv[p];
      bce = bce + (x[p] * mog_logf(rc + 1e-10f) + (1.0f - x[p]) * mog_logf((1.0f - rc) + 1e-10f));
      const float d = x[p] - rc;
      mse = mse + d * d;
    }
    o->bce[b] = -bce;
    o->mse[b] = mse;
    /* elbo = sum_t z_pres_kl + sum_t scale_kl + sum_t shift_kl + sum_t vae_kl + recon */
    float zs = 0.0f, ss = 0.0f, hs = 0.0f, vsum = 0.0f, ps = 0.0f;
    for (int t = 0; t < Tx; ++t) {
      const size_t tb = (size_t)t * B + b;
      zs = zs + o->z_pres_kl[tb];
      ss = ss + o->scale_kl[tb];
      hs = hs + o->shift_kl[tb];
      vsum = vsum + o->vae_kl[tb];
      ps = ps + o->pr_num[tb];
    }
    const float elbo = ((((0.0f + zs) + ss) + hs) + vsum) + o->bce[b];
    o->elbo[b] = elbo;
    /* area (:1017-1027): mean over steps of max(amax - sC, 0) + max(sC - amin, 0) */
    float area = 0.0f, outl = 0.0f, size = 0.0f, over = 0.0f;
    for (int t = 0; t < Tx; ++t) {
      const float sc = o->scale[(size_t)t * B + b] * (float)C;
      area = area + (fmaxf(cfg->area_max - sc, 0.0f) + fmaxf(sc - cfg->area_min, 0.0f));
    }
    area = Tx > 0 ? area / (float)Tx : 0.0f;
    /* bbox out / size / overlap (:1029-1069) over all executed steps */
    for (int i = 0; i < Tx; ++i) {
      const size_t ti = (size_t)i * B + b;
      const float cxi = ((o->shift[ti * 2] + 1.0f) * (float)C) / 2.0f;
      const float cyi = ((o->shift[ti * 2 + 1] + 1.0f) * (float)C) / 2.0f;
      const float sci = o->scale[ti] * (float)C;
      const float mnx = cxi - 0.5f * sci, mny = cyi - 0.5f * sci;
      const float mxx = cxi + 0.5f * sci, mxy = cyi + 0.5f * sci;
      outl = outl + (((fmaxf(-1.0f * mnx, 0.0f) + fmaxf(-1.0f * mny, 0.0f)) +
                      fmaxf(mxx - (float)C, 0.0f)) + fmaxf(mxy - (float)C, 0.0f));
      for (int j = 0; j < Tx; ++j) {
        const size_t tj = (size_t)j * B + b;
        const float scj = o->scale[tj] * (float)C;
        size = size + fmaxf(fabsf(sci - scj) - 3.0f, 0.0f);
        const float cxj = ((o->shift[tj * 2] + 1.0f) * (float)C) / 2.0f;
        const float cyj = ((o->shift[tj * 2 + 1] + 1.0f) * (float)C) / 2.0f;
        const float md = fmaxf(fabsf(cxi - cxj), fabsf(cyi - cyj));
        const float smean = (sci + scj) / 2.0f;
        over = over + fmaxf(smean - md, 0.0f) * (i == j ? 0.0f : 1.0f);
      }
    }
    o->area[b] = area;
    o->out[b] = outl;
    o->size[b] = size;
    o->overlap[b] = over;
    float pr = 0.0f + ps;
    pr = pr + cfg->g_area * area;
    pr = pr + over * cfg->g_bbox;
    pr = pr + outl * cfg->g_bbox;
    pr = pr + size * cfg->g_size;
    o->pr_loss[b] = pr;
    /* element-wise number loss (:1000-1015): min over the allowed counts */
    float elem = 0.0f;
    if (cfg->g_margin > 1e-8f) {
      float best = 0.0f;
      for (int k = 0; k < NC; ++k) {
        float sum = 0.0f;
        for (int t = 0; t < Tx; ++t)
          sum = sum + sigmoid_ce(t < cfg->constrains[k] ? 1.0f : 0.0f,
                                 logit8(o->z_pres_prob[(size_t)t * B + b]));
        best = k == 0 ? sum : fminf(best, sum);
      }
      elem = best * cfg->g_element;
    }
    o->element[b] = elem;
    o->loss[b] = (elbo + pr) + elem;
    if (targets) acc = acc + (targets[b] == o->digits[b] ? 1.0f : 0.0f);
  }
  *acc_out = acc / (float)B;
  free(h); free(c); free(hg); free(cg); free(hg_prev); free(zprev); free(ssprev);
  free(znew); free(ssnew); free(stop); free(canvas); free(gates); free(hid); free(hid2);
  free(g); free(a1); free(a2); free(mu); free(lv); free(d1); free(d2); free(r); free(wr);
  return Tx;
}
