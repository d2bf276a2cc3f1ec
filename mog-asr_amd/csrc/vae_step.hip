// Fused per-object step: STN read -> glimpse VAE -> latent sample + KL ->
// STN write, one launch per loop step (air_model.py:500-588 + :718-736,
// vae.py:5-48, transformer.py:18-175).  This is the kernel SURVEY.md §8 D.3
// prices at 30,024 algorithmic HBM bytes per image-step.
//
// One workgroup = 16 waves = M = 16*MT images per CU (MT = 8: 128 images;
// MT = 4 / 2 for batches too small to give every CU 128).  Sixteen waves
// (four per SIMD) keep enough weight loads, gathers and stores in flight.  The bf16 weights
// (W^T in MFMA B-fragment order: one 1-KiB contiguous wave load per fragment)
// stream from L2 straight into the MFMA B operand, so the L2 -> CU weight
// traffic per image is 2.2 MB / M: the tile height M is what keeps the dense
// layers off the L2 bandwidth roof.  A workgroup never holds its whole glimpse
// (M x 800 bf16 would not fit): the STN read is pipelined k-step by k-step into
// the recognition layer -- the gathers of k-step ks+2 are in flight while the
// MFMAs of k-step ks run, samples for k-step ks+1 land in a two-slab LDS ring,
// and each slab is flushed to HBM as the saved glimpse.  The other layers keep
// their activations in one LDS arena (bf16, rows padded against bank
// conflicts; a layer whose output lands on its own input waits for the whole
// workgroup after its k loop).  Activations the backward needs (glimpse,
// softplus outputs, mu/logvar/z, r) are flushed with 16-byte stores.  The
// output layer's accumulator quads are transposed across lanes (DPP) so a lane
// owns four consecutive pixels -- one Philox quad of eps_x, one 16-byte store
// of r; the STN write stages r back M/4 images at a time and stores, per image,
// only the band-aligned rows of this step's canvas contribution z * w that can
// be nonzero (part_rows records them); mog_recon_loss sums the parts in step
// order, so the canvas is bit-identical to the running accumulation of
// air_model.py:665-675 and this kernel never waits on a canvas read.
//
// Precision: bf16 MFMA operands, fp32 accumulation and epilogues with
// hardware transcendentals (the bf16 configuration, BASELINE configs[1]).
#include "vae_tile.h"

namespace {


template <int MT, int NW, int OCC, int LA = 3>
__global__ __launch_bounds__(NW * 64, OCC) void stn_vae_step_kernel(StepArgs p) {
#pragma clang fp contract(off)
  using Ly = Lay<MT, NW>;
  constexpr int M = Ly::M;
  constexpr int NTHR = NW * 64;
  constexpr int TW = 64 / NW;  // recognition column tiles per MFMA wave
  static_assert(MT <= NW && (NW == 8 || NW == 16), "shape");
  __shared__ __attribute__((aligned(16))) unsigned char arena[Ly::ARENA];
  __shared__ float sth[M][12];
  __shared__ float szv[M];
  __shared__ int smask[M];
  __shared__ int ssep[M];  // bit 0: theta_f axis-aligned, bit 1: theta_b (and tables fit)
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int b0 = blockIdx.x * M;
  const int nb = min(M, p.B - b0);
  const int C = p.C;
  STAMP(11);

  // Prologue: every global load issued up front from clamped indices and
  // selected afterwards -- thetas, mask, z value, eps_z -- so the tile pays
  // one memory latency here, not a chain of them (a load under `if (m < nb)`
  // compiles to a branch with a vmcnt(0) wait inside; the z value waited for
  // the mask)
  constexpr int TH_IT = (M * 12 + NTHR - 1) / NTHR;
  constexpr int EZ_IT = (M * 50 / 4 + NTHR - 1) / NTHR;
  float thv[TH_IT];
#pragma unroll
  for (int j = 0; j < TH_IT; ++j) {
    const int i = tid + j * NTHR, m = min(i / 12, nb - 1), k = i % 12;
    thv[j] = k < 6 ? p.theta_f[(size_t)(b0 + m) * 6 + k] : p.theta_b[(size_t)(b0 + m) * 6 + k - 6];
  }
  const int tc = min(tid, nb - 1);
  const float mk = p.mask[b0 + tc], zv = p.zval[b0 + tc];
  const bool ez_al = ((reinterpret_cast<size_t>(p.eps_z) & 15) == 0);
  const int nez4 = ez_al ? nb * 50 / 4 : 0;
  float4 ezv[EZ_IT];
  if (ez_al) {  // (uniform)
    const float4* src = reinterpret_cast<const float4*>(p.eps_z + (size_t)b0 * 50);
#pragma unroll
    for (int j = 0; j < EZ_IT; ++j) ezv[j] = src[min(tid + j * NTHR, nez4 - 1)];
  }
#pragma unroll
  for (int j = 0; j < TH_IT; ++j) {
    const int i = tid + j * NTHR;
    if (i < M * 12) sth[i / 12][i % 12] = i / 12 < nb ? thv[j] : 0.0f;
  }
  if (tid < M) {
    const bool act = tid < nb && mk != 0.0f;
    smask[tid] = act;
    szv[tid] = act ? zv : 0.0f;
  }
  {  // eps_z of the tile -> LDS (contiguous [nb][50] rows), used in the sample phase
    float* sEz = reinterpret_cast<float*>(arena + Ly::OFF_EZ);
#pragma unroll
    for (int j = 0; j < EZ_IT; ++j)
      if (tid + j * NTHR < nez4) reinterpret_cast<float4*>(sEz)[tid + j * NTHR] = ezv[j];
    for (int i = nez4 * 4 + tid; i < nb * 50; i += NTHR) sEz[i] = p.eps_z[(size_t)b0 * 50 + i];
  }
  lds_barrier();
  bool sep_f = true;
  if (tid < M) {
    sep_f = stn_separable(&sth[tid][0]);
    ssep[tid] = (sep_f ? 1 : 0) | (stn_separable(&sth[tid][6]) && C <= CTAB_MAX ? 2 : 0);
  }
  {  // read tables: column entries in pair form, row entries {lo, hi byte offsets, hi - c, c - lo}
    float4* tabR = reinterpret_cast<float4*>(arena);
    for (int i = tid; i < M * TABR; i += NTHR) {
      const int m = i / TABR, n = i - (i / TABR) * TABR;
      const float* th = sth[m];
      tabR[i] = n < 28 ? col_pair4(axis_col(th, C, C, 28, 28, n), C)
                       : axis4(axis_row(th, C, C, 28, 28, n - 28), 4 * C);
    }
  }
  const bool all_sep = __syncthreads_and(sep_f) != 0;  // (no global stores issued yet)
  STAMP(0);

  // ---- 1+2. STN read (transformer.py:18-175) -> a1 = softplus(g W1 + b1) --
  {
    floatx4 acc[MT][TW];
    int ct[TW];
    floatx4 b1q[TW];
    if (all_sep) read_recognition<MT, NW, true, LA>(p, arena, sth, b0, nb, acc, ct, b1q);
    else read_recognition<MT, NW, false, 3>(p, arena, sth, b0, nb, acc, ct, b1q);
    STAMP(1);
    __bf16* sA1 = reinterpret_cast<__bf16*>(arena);
    const int li = lane & 15, g = lane >> 4;
    if (wv < NW / 2) {  // the MFMA waves hold the layer
#pragma unroll
      for (int c = 0; c < TW; ++c) {
        const int n0 = ct[c] * 16 + (li & ~3);
#pragma unroll
        for (int rt = 0; rt < MT; ++rt)
          store_softplus4(sA1 + (rt * 16 + g * 4 + (li & 3)) * S512 + n0, quad_transpose(acc[rt][c]),
                          b1q[c]);
      }
    }
  }
  lds_barrier();
  STAMP(2);
  __bf16* sA1 = reinterpret_cast<__bf16*>(arena);
  __bf16* sA2 = sA1;
  // ---- 3. a2 = softplus(a1 W2 + b2)  [M x 256], in place ------------------
  // (a1's saved copy is flushed inside the k loop, finished before the
  // in-place epilogue)
  {
    RowFlush<__bf16, 512, NTHR> fl(sA1, S512, p.a1b + (size_t)b0 * 512, 512, nb,
                                   (p.phases & 16) != 0, tid);
    if (p.phases & 2) {
      dense_tiles<MT, 512, 256, 16 / NW, 4, true>(sA1, S512, p.wt[1], p.bias[1], 0, 0, NW,
                                       [&](int m, int n0, const floatx4& v, const floatx4& b) {
                                         store_softplus4(sA2 + m * S256 + n0, v, b);
                                       },
                                       LdsBarrier{}, fl);
    } else {
      fl();
    }
  }
  lds_barrier();
  STAMP(3);
  // ---- 4. mu | lv = a2 W + b  [M x 50] fp32 (waves 0-3 | 4-7; the others --
  // flush a2's saved copy meanwhile)
  float* sMu = reinterpret_cast<float*>(arena + Ly::OFF_MU);
  float* sLv = reinterpret_cast<float*>(arena + Ly::OFF_LV);
  if (p.phases & 2) {
    auto epi_f32 = [&](float* dst) {
      return [dst](int m, int n0, const floatx4& v, const floatx4& b) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (n0 + k < 50) dst[m * 50 + n0 + k] = v[k] + b[k];
      };
    };
    if (wv < 8) {
      dense_tiles<MT, 256, 50, 1, 4, false>(sA2, S256, p.wt[2], p.bias[2], 0, 0, 4, epi_f32(sMu));
      dense_tiles<MT, 256, 50, 1, 4, false>(sA2, S256, p.wt[3], p.bias[3], 0, 4, 4, epi_f32(sLv));
    }
  }
  if (p.phases & 16) {
    if (NW == 16 && (p.phases & 2)) {
      if (wv >= 8) flush_rows<NTHR / 2>(sA2, S256, p.a2b + (size_t)b0 * 256, 256, 256, nb, tid - NTHR / 2);
    } else {
      flush_rows<NTHR>(sA2, S256, p.a2b + (size_t)b0 * 256, 256, 256, nb);
    }
  }
  lds_barrier();
  STAMP(4);
  // ---- 5. z = mu + eps sqrt(exp(lv)); VAE KL -> runloss (vae.py:27-30) ---
  float* sKl = reinterpret_cast<float*>(arena + Ly::OFF_KL);
  __bf16* sZ = reinterpret_cast<__bf16*>(arena + Ly::OFF_Z);
  {
    constexpr int NS = M * 64 / NTHR;
    const float* sEz = reinterpret_cast<const float*>(arena + Ly::OFF_EZ);
    float ez[NS];
#pragma unroll
    for (int it = 0; it < NS; ++it) {
      const int i = tid + it * NTHR, m = i >> 6, k = i & 63;
      ez[it] = (k < 50 && m < nb) ? sEz[m * 50 + k] : 0.0f;
    }
#pragma unroll
    for (int it = 0; it < NS; ++it) {
      const int i = tid + it * NTHR, m = i >> 6, k = i & 63;
      float zv = 0.0f;
      if (k < 50 && m < nb) {
        const size_t o = (size_t)(b0 + m) * 50 + k;
        const float l = sLv[m * 50 + k];
        const float mv = sMu[m * 50 + k];
        const float var = mog_expf(l);
        zv = mv + ez[it] * sqrtf(var);
        if (p.z) st_stream(p.z + o, zv);  // the latents (also a reported output)
        if (p.phases & 16) {   // saved for the backward
          st_stream(p.mu + o, mv);
          st_stream(p.lv + o, l);
          p.zb[(size_t)(b0 + m) * 56 + k] = (__bf16)zv;
        }
        const float d = mv - p.v_pm;
        sKl[m * 50 + k] = (((p.v_plv - l) - 1.0f) + var / p.v_pv) + (d * d) / p.v_pv;
      }
      sZ[m * SZ + k] = (__bf16)zv;
    }
  }
  lds_barrier();
  if (tid < nb) {  // sequential KL sum per image (k order, as vae_sample_fwd_kernel)
    const int m = tid;
    // (the running loss read before the sum: its latency under the adds)
    const float rl = p.runloss ? p.runloss[b0 + m] : 0.0f;
    float t[50];
#pragma unroll
    for (int k = 0; k < 50; ++k) t[k] = sKl[m * 50 + k];
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < 50; ++k) sum = sum + t[k];
    const float vkl = 0.5f * sum;
    p.vkl[b0 + m] = vkl;
    if (p.runloss && smask[m]) p.runloss[b0 + m] = rl + vkl;
  }
  STAMP(5);
  // ---- 6. d1 = softplus(z Wg1 + b)  [M x 256] (over mu | lv) ---------------
  __bf16* sD1 = reinterpret_cast<__bf16*>(arena + Ly::OFF_D1);
  if (p.phases & 2) {
    dense_tiles<MT, 64, 256, 16 / NW, 2, false>(sZ, SZ, p.wt[4], p.bias[4], 0, 0, NW,
                                     [&](int m, int n0, const floatx4& v, const floatx4& b) {
                                       store_softplus4(sD1 + m * S256 + n0, v, b);
                                     });
  }
  lds_barrier();
  STAMP(6);
  // ---- 7. d2 = softplus(d1 Wg2 + b)  [M x 512] at 0 (in place over d1; d1's
  // saved copy flushed inside the k loop) ---------------------------------------
  __bf16* sD2 = reinterpret_cast<__bf16*>(arena);
  {
    RowFlush<__bf16, 256, NTHR> fl(sD1, S256, p.d1b + (size_t)b0 * 256, 256, nb,
                                   (p.phases & 16) != 0, tid);
    if (p.phases & 2) {
      dense_tiles<MT, 256, 512, 32 / NW, NW / 4, true>(sD1, S256, p.wt[5], p.bias[5], 0, 0, NW,
                                       [&](int m, int n0, const floatx4& v, const floatx4& b) {
                                         store_softplus4(sD2 + m * S512 + n0, v, b);
                                       },
                                       LdsBarrier{}, fl);
    } else {
      fl();
    }
  }
  lds_barrier();
  STAMP(7);
  // ---- 8. r = sigmoid(d2 Wgo + b + std eps)  [M x 784] fp32 -> HBM ----------
  // (d2's saved copy flushed inside the first pass's k loop)
  // The 4 x 4 accumulator quads are transposed across lanes (two DPP quad
  // exchanges) so that a lane owns four consecutive pixels of one row: one
  // Philox quad of eps_x (generated in-kernel exactly as mog_rng_fill would,
  // or loaded), one 16-byte store of r.  49 column tiles: 32 (2 per wave) + 16
  // (1 per wave) + 1 split over the row tiles.
  if (p.phases & 2) {
    const float sd = p.lik_std;
    auto epi = [&](int m, int n, const floatx4& v, const floatx4& b) {
      if (m < nb) {
        float ev[4];
        const size_t q = (size_t)(b0 + m) * (W2 / 4) + (n >> 2);
        if (p.eps_gen) {
          mog_philox_quad(p.eps_seed, p.eps_offset + q, true, ev);
        } else {
          const float4 e4 = reinterpret_cast<const float4*>(p.eps_x)[q];
          ev[0] = e4.x; ev[1] = e4.y; ev[2] = e4.z; ev[3] = e4.w;
        }
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float y = __builtin_fmaf(ev[k], sd, v[k] + b[k]);
          o[k] = mog_sigmoid_hw(y);
        }
        reinterpret_cast<float4*>(p.r)[q] = make_float4(o[0], o[1], o[2], o[3]);
      }
    };
    RowFlush<__bf16, 512, NTHR> fl(sD2, S512, p.d2b + (size_t)b0 * 512, 512, nb,
                                   (p.phases & 16) != 0, tid);
    if constexpr (MT == 4) {
      dense_out<MT, 32 / NW, 4>(sD2, S512, p, 0, 0, NW, b0, nb, tid, fl);
      STAMP(8);
    } else {  // (the 32-image forms: the hook would not fit their registers)
      fl();
      dense_out<MT, 32 / NW, 4>(sD2, S512, p, 0, 0, NW, b0, nb, tid);
    }
    dense_out<MT, 16 / NW, 4>(sD2, S512, p, 32, 0, NW, b0, nb, tid);
    dense_rowsplit<MT, 512, W2>(sD2, S512, p.wt[6], p.bias[6], 48, epi);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // r stores done before other waves read it
  lds_barrier();
  STAMP(9);
  // ---- 9. STN write (stn_write_tile) --------------------------------------
  if (p.phases & 8)
    stn_write_tile<NW>(p.r, p.part, p.part_rows, C, arena, Ly::WSLOT, sth, smask, ssep, szv, b0, nb,
                       wv, lane);
  if (p.tstamp) {
    lds_barrier();
    STAMP(10);
  }
}


// ===========================================================================
// fp32 step kernel: the reference-precision form of the same fused step
// (air_model.py:523-588, vae.py:5-48, transformer.py:18-175 at fp32),
// bit-identical to the unfused fp32 sequence -- stn_forward, the seven
// mog_gemm_f32 chains with their exact epilogues and pre-activations,
// vae_sample_forward, mog_gemm_f32_sigmoid_philox, mog_stn_write_parts.
// Dense layers on v_mfma_f32_16x16x4_f32 fed in natural k order (MFMA kk of
// k-step ks takes k = 16 ks + 4 kk + g from lane group g), so every output is
// the one k-ordered fma chain of gemm_f32.hip, then + bias, then the
// epilogue.  A tile is 32 images x 16 waves (fp32 activations are twice the
// bf16 bytes); the layers are MFMA-bound (141 MFLOP per 64 images), so the
// phases need no overlap beyond the read / recognition split:
//   * LDS activations are rows of k PERMUTED inside each 16-group (k = 16 s +
//     4 j + g at 16 s + 4 g + j), so lane (row, g) reads its four k-slots of a
//     k-step with one ds_read_b128;
//   * weights are fp32 B-fragment packs (mog_pack_frag_f32): fragment (ks, ct)
//     is 1 KiB, lane (li, g) holds W[16 ks + 4 kk + g][16 ct + li], kk < 4;
//   * epilogues write pre- and post-activation rows to HBM (16-byte stores
//     after the quad transpose) and the post-activation into the next layer's
//     permuted LDS rows.
constexpr int FM = 32;             // images per tile
constexpr int FKS1 = 49;           // recognition k-steps (784 = 49 x 16: no padding)
constexpr int FKG = 7;             // k-steps per glimpse slab
constexpr int FSK = 16 * FKG + 4;  // slab row stride (floats)
constexpr int FS512 = 512 + 4, FS256 = 256 + 4, FSZ = 64 + 4, FS50 = 52;
static_assert(FKS1 % FKG == 0, "slabs");

// LDS arena (bytes): tables + two glimpse slabs during the read; R1 = a1 ->
// mu | lv | kl | z -> d2; R2 = a2 -> d1; write slots (r of one image per wave)
struct LayF {
  static constexpr int TAB = FM * TABR * 16;
  static constexpr int KB = FM * FSK * 4;
  static constexpr int R1 = FM * FS512 * 4;
  static constexpr int OFF_R2 = R1, R2 = FM * FS256 * 4;
  static constexpr int OFF_MU = 0, OFF_LV = FM * FS50 * 4, OFF_KL = 2 * FM * FS50 * 4,
                       OFF_Z = 3 * FM * FS50 * 4;
  static constexpr int WSLOT = W2 * 4;
  static constexpr int ARENA0 = cmax(OFF_R2 + R2, cmax(TAB + 2 * KB, 16 * WSLOT));
  static constexpr int OFF_EZ = ARENA0;
  static constexpr int ARENA = ARENA0 + FM * 50 * 4;
  static_assert(OFF_Z + FM * FSZ * 4 <= R1, "mu / lv / kl / z inside R1");
};

struct StepArgsF {
  const float* x;
  const float* theta_f;
  const float* theta_b;
  const float* mask;
  const float* zval;
  const float* eps_z;
  const float* eps_x;
  unsigned long long eps_seed, eps_offset;
  int eps_gen;
  const float* wt[7];  // fp32 B-fragment packs: r1, r2, mu, lv, g1, g2, go
  const float* bias[7];
  float* part;
  int* part_rows;
  float* runloss;
  float* vkl;
  float* g;                  // [B, 784]  saved for the backward (may be null: forward only)
  float *a1pre, *a1;         // [B, 512]
  float *a2pre, *a2;         // [B, 256]
  float *mu, *lv, *z;        // [B, 50]   (z always written)
  float *d1pre, *d1;         // [B, 256]
  float *d2pre, *d2;         // [B, 512]
  float* r;                  // [B, 784]  (always written)
  int B, C;
  int x_period;
  float lik_std, v_pm, v_pv, v_plv;
  int phases;                // (always all: the profiling masks are the bf16 kernel's)
  long long* tstamp;
};

// position of k inside a permuted row
__device__ __forceinline__ int kperm(int k) { return (k & ~15) | ((k & 3) << 2) | ((k >> 2) & 3); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t frag_rsrc_f32(const float* W) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(W), 0, 0x7ffffff0, 0x00020000);
}
template <int NCT>
__device__ __forceinline__ floatx4 load_frag_f32(__amdgpu_buffer_rsrc_t r, int voff, int ks) {
  return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, ks * NCT * 1024, 0));
}

// One fp32 dense layer over row tiles [0, MT) (rows from A + row0 * lda) and
// the column tiles of waves wbase .. wbase + nw - 1: wave w owns column tiles
// tile_base + (w + nw c + rot) % (nw TPW), c < TPW.  No barrier inside.
// epi(m, n0, v, b): row m, columns n0 .. n0+3 (quad-transposed), biases b.
template <int MT, int KS, int NCT, int TPW, int D, class Epi>
__device__ __forceinline__ void dense_f32(const float* A, int lda, const float* W,
                                          const float* __restrict__ bias, int N, int tile_base,
                                          int wbase, int nw, Epi epi, int tid) {
  const int rot = (int)(blockIdx.x >> 3);
  const int lane = tid & 63, w = (tid >> 6) - wbase;
  if (w < 0 || w >= nw) return;
  const int li = lane & 15, g = lane >> 4;
  int ct[TPW], wo[TPW];
  const __amdgpu_buffer_rsrc_t wr = frag_rsrc_f32(W);
  floatx4 bq[TPW];
#pragma unroll
  for (int c = 0; c < TPW; ++c) {
    ct[c] = tile_base + (w + nw * c + rot) % (nw * TPW);
    wo[c] = frag_voff(ct[c], lane);
    bq[c] = load_bias4(bias, ct[c] * 16 + (li & ~3), N);
  }
  floatx4 acc[MT][TPW];
#pragma unroll
  for (int rt = 0; rt < MT; ++rt)
#pragma unroll
    for (int c = 0; c < TPW; ++c) acc[rt][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  floatx4 q[D][TPW];
  auto loadB = [&](int ks, floatx4* b) {
#pragma unroll
    for (int c = 0; c < TPW; ++c) b[c] = load_frag_f32<NCT>(wr, wo[c], ks);
  };
#pragma unroll
  for (int d = 0; d < D && d < KS; ++d) loadB(d, q[d]);
  static_for<0, KS>([&](auto kc) {
    constexpr int ks = decltype(kc)::value;
    floatx4 a[MT];
#pragma unroll
    for (int rt = 0; rt < MT; ++rt)
      a[rt] = *reinterpret_cast<const floatx4*>(&A[(rt * 16 + li) * lda + 16 * ks + 4 * g]);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int rt = 0; rt < MT; ++rt)
#pragma unroll
        for (int c = 0; c < TPW; ++c)
          acc[rt][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rt][kk], q[ks % D][c][kk], acc[rt][c],
                                                            0, 0, 0);
    if constexpr (ks + D < KS) loadB(ks + D, q[ks % D]);
  });
#pragma unroll
  for (int c = 0; c < TPW; ++c)
#pragma unroll
    for (int rt = 0; rt < MT; ++rt)
      epi(rt * 16 + g * 4 + (li & 3), ct[c] * 16 + (li & ~3), quad_transpose(acc[rt][c], tid), bq[c]);
}

__global__ __launch_bounds__(1024, 1) void stn_vae_step_f32_kernel(StepArgsF p) {
#pragma clang fp contract(off)
  constexpr int M = FM, NW = 16, NTHR = 1024;
  __shared__ __attribute__((aligned(16))) unsigned char arena[LayF::ARENA];
  __shared__ float sth[M][12];
  __shared__ float szv[M];
  __shared__ int smask[M];
  __shared__ int ssep[M];
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, li = lane & 15, g = lane >> 4;
  const int b0 = blockIdx.x * M;
  const int nb = min(M, p.B - b0);
  const int C = p.C, C2 = C * C;
  STAMP(11);
  // ---- prologue: the bf16 kernel's (thetas, masks, read tables, eps_z) -----
  // every global load issued up front from clamped indices (one latency)
  constexpr int TH_IT = (M * 12 + NTHR - 1) / NTHR;
  constexpr int EZ_IT = (M * 50 + NTHR - 1) / NTHR;
  float thv[TH_IT], ezv[EZ_IT];
#pragma unroll
  for (int j = 0; j < TH_IT; ++j) {
    const int i = tid + j * NTHR, m = min(i / 12, nb - 1), k = i % 12;
    thv[j] = k < 6 ? p.theta_f[(size_t)(b0 + m) * 6 + k] : p.theta_b[(size_t)(b0 + m) * 6 + k - 6];
  }
  const int tc = min(tid, nb - 1);
  const float mk = p.mask[b0 + tc], zv = p.zval[b0 + tc];
#pragma unroll
  for (int j = 0; j < EZ_IT; ++j) ezv[j] = p.eps_z[(size_t)b0 * 50 + min(tid + j * NTHR, nb * 50 - 1)];
#pragma unroll
  for (int j = 0; j < TH_IT; ++j) {
    const int i = tid + j * NTHR;
    if (i < M * 12) sth[i / 12][i % 12] = i / 12 < nb ? thv[j] : 0.0f;
  }
  if (tid < M) {
    const bool act = tid < nb && mk != 0.0f;
    smask[tid] = act;
    szv[tid] = act ? zv : 0.0f;
  }
  {
    float* sEz = reinterpret_cast<float*>(arena + LayF::OFF_EZ);
#pragma unroll
    for (int j = 0; j < EZ_IT; ++j)
      if (tid + j * NTHR < nb * 50) sEz[tid + j * NTHR] = ezv[j];
  }
  lds_barrier();
  bool sep_f = true;
  if (tid < M) {
    sep_f = stn_separable(&sth[tid][0]);
    ssep[tid] = (sep_f ? 1 : 0) | (stn_separable(&sth[tid][6]) && C <= CTAB_MAX ? 2 : 0);
  }
  {
    float4* tabR = reinterpret_cast<float4*>(arena);
    for (int i = tid; i < M * TABR; i += NTHR) {
      const int m = i / TABR, n = i - (i / TABR) * TABR;
      const float* th = sth[m];
      tabR[i] = n < 28 ? col_pair4(axis_col(th, C, C, 28, 28, n), C)
                       : axis4(axis_row(th, C, C, 28, 28, n - 28), 4 * C);
    }
  }
  const bool all_sep = __syncthreads_and(sep_f) != 0;
  STAMP(0);
  const bool save = p.a1 != nullptr;

  // ---- 1+2. STN read (transformer.py:18-175) -> a1 = softplus(g W1 + b1) --
  // Waves 8-15 sample (lane: image (wv - 8) * 4 + (lane >> 4), pixel 16 ks +
  // (lane & 15) of k-step ks) into two LDS slabs of FKG k-steps and store g;
  // waves 0-7 run the MFMAs (four of the 32 column tiles each) on the other
  // slab; one barrier per slab.
  {
    const float4* tabR = reinterpret_cast<const float4*>(arena);
    floatx4 acc[2][4];
    int ct[4];
    if (wv >= 8) {
      constexpr int LA = 4;
      const int m = (wv - 8) * 4 + (lane >> 4), kk = lane & 15;
      const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(p.x) + (size_t)(b0 % p.x_period) * C2, 0, nb * C2 * 4, 0x00020000);
      const int xo = m * C2 * 4;
      float I[LA][4];
      auto geom = [&](int ks, float4& ex, float4& ey) {
        const int k = 16 * ks + kk;
        if (all_sep) {
          const int i = k / 28, j = k - (k / 28) * 28;
          ex = tabR[m * TABR + j];
          ey = tabR[m * TABR + 28 + i];
        } else {
          glimpse_geom<false>(tabR, sth[m], m, k, C, ex, ey);
        }
      };
      auto gather = [&](int ks, float (&v)[4]) {
        float4 ex, ey;
        geom(ks, ex, ey);
        const int xb = __float_as_int(ex.x) + xo;
        const u32x2 r0 = __builtin_amdgcn_raw_buffer_load_b64(xr, xb + __float_as_int(ey.x), 0, 0);
        const u32x2 r1 = __builtin_amdgcn_raw_buffer_load_b64(xr, xb + __float_as_int(ey.y), 0, 0);
        v[0] = __uint_as_float(r0[0]);
        v[1] = __uint_as_float(r0[1]);
        v[2] = __uint_as_float(r1[0]);
        v[3] = __uint_as_float(r1[1]);
      };
      float* gdst = (save && m < nb) ? p.g + (size_t)(b0 + m) * W2 + kk : nullptr;
      const int so = LayF::TAB + (m * FSK + ((kk & 3) << 2) + (kk >> 2)) * 4;
      auto sample = [&](int ks, const float (&v)[4]) {
        float4 ex, ey;
        geom(ks, ex, ey);
        const int fl = __float_as_int(ex.y);
        const float Ia = (fl & 1) ? v[1] : v[0], Ib = (fl & 1) ? v[3] : v[2];
        const float Ic = (fl & 2) ? v[1] : v[0], Id = (fl & 2) ? v[3] : v[2];
        const int xlive = (fl ^ (fl >> 1)) & 1;
        const int ylive = __float_as_int(ey.x) != __float_as_int(ey.y) ? 1 : 0;
        const int live = (int)(m < nb) & (xlive | ylive);
        const float s = sample4(ex, ey, Ia, Ib, Ic, Id);
        const float val = live ? s : 0.0f;
        const int slab = (ks / FKG) & 1;
        *reinterpret_cast<float*>(arena + so + slab * LayF::KB + (ks % FKG) * 64) = val;
        if (gdst) st_stream(gdst + 16 * ks, val);
      };
#pragma unroll
      for (int k = 0; k < LA; ++k) gather(k, I[k]);
      static_for<0, FKS1>([&](auto kc) {
        constexpr int ks = decltype(kc)::value;
        sample(ks, I[ks % LA]);
        if constexpr (ks + LA < FKS1) gather(ks + LA, I[ks % LA]);
        if constexpr (ks % FKG == FKG - 1) lds_barrier();  // slab filled
      });
      lds_barrier();  // the MFMA waves are done with the last slab
    } else {
      const int rot = (int)(blockIdx.x >> 3);
      const __amdgpu_buffer_rsrc_t wr = frag_rsrc_f32(p.wt[0]);
      int wo[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        ct[c] = (wv + 8 * c + rot) % 32;
        wo[c] = frag_voff(ct[c], lane);
      }
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[rt][c] = floatx4{0.f, 0.f, 0.f, 0.f};
      constexpr int DB = 3;
      floatx4 q[DB][4];
      auto loadB = [&](int ks, floatx4* b) {
#pragma unroll
        for (int c = 0; c < 4; ++c) b[c] = load_frag_f32<32>(wr, wo[c], ks);
      };
#pragma unroll
      for (int d = 0; d < DB; ++d) loadB(d, q[d]);
      const int ao = LayF::TAB + (li * FSK + 4 * g) * 4;
      lds_barrier();  // slab 0 filled
      static_for<0, FKS1>([&](auto kc) {
        constexpr int ks = decltype(kc)::value;
        const unsigned char* sa = arena + ao + ((ks / FKG) & 1) * LayF::KB + (ks % FKG) * 64;
        floatx4 a[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) a[rt] = *reinterpret_cast<const floatx4*>(sa + rt * 16 * FSK * 4);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int c = 0; c < 4; ++c)
              acc[rt][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rt][kk], q[ks % DB][c][kk],
                                                                acc[rt][c], 0, 0, 0);
        if constexpr (ks + DB < FKS1) loadB(ks + DB, q[ks % DB]);
        if constexpr (ks % FKG == FKG - 1) lds_barrier();  // slab consumed / next filled
      });
    }
    STAMP(1);
    // a1 epilogue in two halves: the MFMA waves leave pre = acc + b1 in LDS
    // (the slabs are dead: every wave passed the last barrier), then all
    // sixteen waves take the exact softplus of a quarter row each (on the
    // eight MFMA waves alone this VALU-heavy part took 12.8 us per tile, now
    // 9.9; launch 648 -> 634 us at 24,576 rows)
    float* sA1 = reinterpret_cast<float*>(arena);
    if (wv < 8) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int n0 = ct[c] * 16 + (li & ~3);
        const floatx4 b = load_bias4(p.bias[0], n0, 512);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
          const int mrow = rt * 16 + g * 4 + (li & 3);
          const floatx4 v = quad_transpose(acc[rt][c], tid);
#pragma unroll
          for (int j = 0; j < 4; ++j) sA1[mrow * FS512 + kperm(n0 + j)] = v[j] + b[j];
        }
      }
    }
    lds_barrier();
#pragma unroll
    for (int it = 0; it < M * 128 / NTHR; ++it) {
      const int q = tid + it * NTHR, mrow = q >> 7, n0 = (q & 127) * 4;
      floatx4 pre, post;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pre[j] = sA1[mrow * FS512 + kperm(n0 + j)];
        post[j] = mog_softplusf(pre[j]);
        sA1[mrow * FS512 + kperm(n0 + j)] = post[j];
      }
      if (save && mrow < nb) {
        if (p.a1pre)
          st_stream(reinterpret_cast<floatx4*>(p.a1pre + (size_t)(b0 + mrow) * 512 + n0), pre);
        st_stream(reinterpret_cast<floatx4*>(p.a1 + (size_t)(b0 + mrow) * 512 + n0), post);
      }
    }
  }
  lds_barrier();
  STAMP(2);
  // softplus layer epilogue: pre / post rows to HBM, post into the next
  // layer's permuted LDS rows
  auto sp_epi = [&](float* dst, int ldd, float* gpre, float* gpost, int ldg) {
    return [=](int m, int n0, const floatx4& v, const floatx4& b) {
      floatx4 pre, post;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pre[j] = v[j] + b[j];
        post[j] = mog_softplusf(pre[j]);
        dst[m * ldd + kperm(n0 + j)] = post[j];
      }
      if (gpost != nullptr && m < nb) {
        if (gpre != nullptr)
          st_stream(reinterpret_cast<floatx4*>(gpre + (size_t)(b0 + m) * ldg + n0), pre);
        st_stream(reinterpret_cast<floatx4*>(gpost + (size_t)(b0 + m) * ldg + n0), post);
      }
    };
  };
  float* sR1 = reinterpret_cast<float*>(arena);
  float* sR2 = reinterpret_cast<float*>(arena + LayF::OFF_R2);
  // ---- 3. a2 = softplus(a1 W2 + b2) [M x 256] -> R2 ------------------------
  dense_f32<2, 32, 16, 1, 8>(sR1, FS512, p.wt[1], p.bias[1], 256, 0, 0, NW,
                             sp_epi(sR2, FS256, save ? p.a2pre : nullptr, save ? p.a2 : nullptr, 256), tid);
  lds_barrier();
  STAMP(3);
  // ---- 4. mu | lv = a2 W + b [M x 50] (waves 0-3 | 4-7) -> R1 -------------
  float* sMu = reinterpret_cast<float*>(arena + LayF::OFF_MU);
  float* sLv = reinterpret_cast<float*>(arena + LayF::OFF_LV);
  {
    auto epi50 = [&](float* dst) {
      return [dst](int m, int n0, const floatx4& v, const floatx4& b) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (n0 + j < 50) dst[m * FS50 + n0 + j] = v[j] + b[j];
      };
    };
    dense_f32<2, 16, 4, 1, 4>(sR2, FS256, p.wt[2], p.bias[2], 50, 0, 0, 4, epi50(sMu), tid);
    dense_f32<2, 16, 4, 1, 4>(sR2, FS256, p.wt[3], p.bias[3], 50, 0, 4, 4, epi50(sLv), tid);
  }
  lds_barrier();
  STAMP(4);
  // ---- 5. z = mu + eps sqrt(exp(lv)); VAE KL (vae.py:27-30) -> R1 ---------
  float* sKl = reinterpret_cast<float*>(arena + LayF::OFF_KL);
  float* sZ = reinterpret_cast<float*>(arena + LayF::OFF_Z);
  {
    const float* sEz = reinterpret_cast<const float*>(arena + LayF::OFF_EZ);
#pragma unroll
    for (int it = 0; it < M * 64 / NTHR; ++it) {
      const int i = tid + it * NTHR, m = i >> 6, k = i & 63;
      float zv = 0.0f;
      if (k < 50 && m < nb) {
        const size_t o = (size_t)(b0 + m) * 50 + k;
        const float l = sLv[m * FS50 + k];
        const float mv = sMu[m * FS50 + k];
        const float var = mog_expf(l);
        zv = mv + sEz[m * 50 + k] * sqrtf(var);
        st_stream(p.z + o, zv);
        if (save) {
          st_stream(p.mu + o, mv);
          st_stream(p.lv + o, l);
        }
        const float d = mv - p.v_pm;
        sKl[m * 50 + k] = (((p.v_plv - l) - 1.0f) + var / p.v_pv) + (d * d) / p.v_pv;
      }
      sZ[m * FSZ + kperm(k)] = zv;
    }
  }
  lds_barrier();
  if (tid < nb) {  // sequential KL sum per image (k order, as vae_sample_fwd_kernel)
    const int m = tid;
    const float rl = p.runloss ? p.runloss[b0 + m] : 0.0f;  // (latency under the sum)
    float sum = 0.0f;
    for (int k = 0; k < 50; ++k) sum = sum + sKl[m * 50 + k];
    const float vkl = 0.5f * sum;
    p.vkl[b0 + m] = vkl;
    if (p.runloss && smask[m]) p.runloss[b0 + m] = rl + vkl;
  }
  STAMP(5);
  // ---- 6. d1 = softplus(z Wg1 + b) [M x 256] -> R2 (K = 50 padded to 64) --
  dense_f32<2, 4, 16, 1, 4>(sZ, FSZ, p.wt[4], p.bias[4], 256, 0, 0, NW,
                            sp_epi(sR2, FS256, save ? p.d1pre : nullptr, save ? p.d1 : nullptr, 256), tid);
  lds_barrier();
  STAMP(6);
  // ---- 7. d2 = softplus(d1 Wg2 + b) [M x 512] -> R1 -------------------------
  dense_f32<2, 16, 32, 2, 6>(sR2, FS256, p.wt[5], p.bias[5], 512, 0, 0, NW,
                             sp_epi(sR1, FS512, save ? p.d2pre : nullptr, save ? p.d2 : nullptr, 512), tid);
  lds_barrier();
  STAMP(7);
  // ---- 8. r = sigmoid((d2 Wgo + b) + std eps) [M x 784] -> HBM ------------
  // (gemm_f32's EPI_SIGMOID_NOISE: eps_x from the Philox quad of (row, col / 4)
  // or read; 49 column tiles: 48 over the 16 waves, the last split by rows)
  {
    const float sd = p.lik_std;
    auto epi = [&](int m, int n0, const floatx4& v, const floatx4& b) {
      if (m >= nb) return;
      float e[4];
      const size_t q = (size_t)(b0 + m) * (W2 / 4) + (n0 >> 2);
      if (p.eps_gen) {
        mog_philox_quad(p.eps_seed, p.eps_offset + q, true, e);
      } else {
        const float4 e4 = reinterpret_cast<const float4*>(p.eps_x)[q];
        e[0] = e4.x; e[1] = e4.y; e[2] = e4.z; e[3] = e4.w;
      }
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float w = v[j] + b[j];
        o[j] = mog_sigmoidf(w + e[j] * sd);
      }
      reinterpret_cast<float4*>(p.r)[q] = make_float4(o[0], o[1], o[2], o[3]);
    };
    dense_f32<2, 32, 49, 3, 5>(sR1, FS512, p.wt[6], p.bias[6], W2, 0, 0, NW, epi, tid);
    if (wv >= 14) {  // column tile 48: row tile wv - 14
      const int rt = wv - 14;
      dense_f32<1, 32, 49, 1, 4>(sR1 + rt * 16 * FS512, FS512, p.wt[6], p.bias[6], W2, 48, 14, 1,
                                 [&](int m, int n0, const floatx4& v, const floatx4& b) {
                                   epi(m + rt * 16, n0, v, b);
                                 },
                                 tid - rt * 64);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // r stores done before other waves read it
  lds_barrier();
  STAMP(8);
  STAMP(9);
  // ---- 9. STN write: the bf16 kernel's (stn_write_tile) ---------------------
  stn_write_tile<NW>(p.r, p.part, p.part_rows, C, arena, LayF::WSLOT, sth, smask, ssep, szv, b0,
                     nb, wv, lane);
  if (p.tstamp) {
    lds_barrier();
    STAMP(10);
  }
}

// W [K][N] row-major fp32 -> B-fragment pack ((ks * NCT + ct) * 64 + lane) * 4
// + kk = W[16 ks + 4 kk + g][16 ct + li] (lane = 16 g + li), zero outside.
struct PackF32 {
  const float* W[8];
  float* out[8];
  int K[8], N[8];
};
__global__ __launch_bounds__(256) void pack_frag_f32_kernel(PackF32 a) {
  const int L = blockIdx.y;
  const int K = a.K[L], N = a.N[L], KS = (K + 15) / 16, NCT = (N + 15) / 16;
  const long total = (long)KS * NCT * 256;
  for (long o = (long)blockIdx.x * 256 + threadIdx.x; o < total; o += (long)gridDim.x * 256) {
    const int kk = (int)(o & 3), lane = (int)((o >> 2) & 63);
    const long f = o >> 8;
    const int ct = (int)(f % NCT), ks = (int)(f / NCT);
    const int k = 16 * ks + 4 * kk + (lane >> 4), n = 16 * ct + (lane & 15);
    a.out[L][o] = (k < K && n < N) ? a.W[L][(size_t)k * N + n] : 0.0f;
  }
}

}  // namespace


// The fused step kernels run one 16-wave workgroup per CU and would leave a
// few KiB of LDS free beside it; their launches pad the LDS request to the
// CU's whole 160 KiB, so no workgroup of another kernel that uses LDS -- every
// GEMM, the bf16 and x3 ones included -- can share a CU with them.  That is
// what lets this file build with SLP vectorization (compiler-packed
// v_pk_*_f32 arithmetic; without it the bf16 training step at 65,536 images
// took 472 instead of 452 us, scripts/ab_fused.py): DESIGN.md §2 traced wrong
// halves of packed fp32 pairs to bf16 MFMA waves of ANOTHER kernel on the same
// CU, which the padding rules out (tests/test_gpu_streams.py runs the fused
// kernels beside bf16 / x3 GEMMs and requires every output bit-identical).
constexpr size_t CU_LDS_BYTES = 160 * 1024;
template <class Kern>
long lds_pad(Kern k) {
  hipFuncAttributes a;
  if (hipFuncGetAttributes(&a, reinterpret_cast<const void*>(k)) != hipSuccess) return -1;
  return a.sharedSizeBytes < CU_LDS_BYTES ? (long)(CU_LDS_BYTES - a.sharedSizeBytes) : 0;
}

extern "C" int mog_stn_vae_step_forward(int B, int C, int W, int R1, int R2, int Z, int G1,
                                        int G2, const float* x, const float* theta_f,
                                        const float* theta_b, const float* mask,
                                        const float* zval, const float* eps_z,
                                        const float* eps_x, int eps_gen,
                                        unsigned long long eps_seed,
                                        unsigned long long eps_offset, const void* const* wt,
                                        const float* const* bias, float lik_std, float v_pm,
                                        float v_pv, float v_plv, float* canvas_part,
                                        int* part_rows, float* runloss, float* vkl, void* gb,
                                        void* a1b, void* a2b, float* mu, float* lv, float* z,
                                        void* zb, void* d1b, void* d2b, float* r, int x_period,
                                        void* stream) {
  MOG_CHECK_ARG(B >= 0 && C >= 2 && C * C <= 16384);
  // the tile shapes are compiled for the reference's default VAE
  MOG_CHECK_ARG(W == 28 && R1 == 512 && R2 == 256 && Z == 50 && G1 == 256 && G2 == 512);
  MOG_CHECK_ARG(x && theta_f && theta_b && mask && zval && eps_z && (eps_x || eps_gen) && wt && bias);
  MOG_CHECK_ARG(canvas_part && part_rows && vkl && r);
  // the saved activations: all given (train) or all NULL (forward only); gb
  // (the saved glimpse) may be given in either form
  const bool save = a1b != nullptr;
  MOG_CHECK_ARG(!save || (gb && a2b && mu && lv && z && zb && d1b && d2b));
  MOG_CHECK_ARG(save || !(a2b || mu || lv || zb || d1b || d2b));
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
  p.part = canvas_part; p.part_rows = part_rows; p.runloss = runloss; p.vkl = vkl;
  p.gb = reinterpret_cast<__bf16*>(gb); p.a1b = reinterpret_cast<__bf16*>(a1b);
  p.a2b = reinterpret_cast<__bf16*>(a2b); p.mu = mu; p.lv = lv; p.z = z;
  p.zb = reinterpret_cast<__bf16*>(zb); p.d1b = reinterpret_cast<__bf16*>(d1b);
  p.d2b = reinterpret_cast<__bf16*>(d2b); p.r = r;
  const char* ph = mog_prof_env("MOG_VS_PHASES");
  p.phases = ph ? atoi(ph) : 31;
  if (!save) p.phases &= ~16;
  p.B = B; p.C = C; p.lik_std = lik_std; p.v_pm = v_pm; p.v_pv = v_pv; p.v_plv = v_plv;
  p.x_period = x_period > 0 ? x_period : B;
  hipStream_t s = mog_stream(stream);
  // Tile height: the one with the shorter estimated launch, rounds of tiles
  // over the CUs x the measured per-tile time (one 16-wave workgroup per CU:
  // ~112 us per 64-image tile, ~73 us per 32-image tile on MI355X).  64-image
  // tiles halve the weight stream per image, but a partial last round (the
  // train step's T*B = 24,576 rows: 1.5 rounds of 64-image tiles, 3 of
  // 32-image ones) can cost more than they save: 225 -> 220 us, bf16 train
  // step 2.32 -> 2.28 ms.  MOG_VS_MT overrides (profiling build): 4 = 64 images x 16 waves,
  // 2 = 32 images x 8 waves, 3 = 32 images x 16 waves.
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      ncu = v;
    else
      ncu = 256;
  }
  const long r64 = ((long)B + 64L * ncu - 1) / (64L * ncu), r32 = ((long)B + 32L * ncu - 1) / (32L * ncu);
  int mt = r64 * 112 <= r32 * 73 ? 4 : 3;
  if (const char* e = mog_prof_env("MOG_VS_MT")) {  // (profiling build)
    const int v = atoi(e);
    if (v == 2 || v == 3 || v == 4) mt = v;
  }
  const int M = 16 * (mt == 3 ? 2 : mt);
  // a tile must not straddle two periods of x (one descriptor per tile);
  // several steps' rows in one launch also rule out the running loss
  // (rows of one image would race on it: mog_air_runloss replays it)
  MOG_CHECK_ARG(p.x_period == B || (p.x_period % M == 0 && !runloss));
  // MOG_VS_TIMING=1 (profiling build): per-phase durations, averaged over
  // blocks, printed to stderr (synchronizes the stream)
  static long long* tbuf = nullptr;
  static size_t tcap = 0;
  const unsigned nblk = mog_cdiv(B, M);
  p.tstamp = nullptr;
  if (mog_prof_env("MOG_VS_TIMING")) {
    if (tcap < (size_t)nblk * 16) {
      if (tbuf) (void)hipFree(tbuf);
      tcap = (size_t)nblk * 16;
      if (hipMalloc(&tbuf, tcap * sizeof(long long)) != hipSuccess) return MOG_ERR_INVALID;
    }
    p.tstamp = tbuf;
  }
  // (the LDS padding of the 16-wave forms: see lds_pad)
  static const long pad4 = lds_pad(stn_vae_step_kernel<4, 16, 4>);
  static const long pad3 = lds_pad(stn_vae_step_kernel<2, 16, 4>);
  if (pad4 < 0 || pad3 < 0) return MOG_ERR_INVALID;
#ifdef MOG_PROFILING
  // MOG_VS_LA (profiling build): sampler gather lookahead of the 64-image form
  static const int la = mog_prof_env("MOG_VS_LA") ? atoi(mog_prof_env("MOG_VS_LA")) : 3;
  if (mt == 4 && la == 4) stn_vae_step_kernel<4, 16, 4, 4><<<nblk, 1024, pad4, s>>>(p);
  else if (mt == 4 && la == 5) stn_vae_step_kernel<4, 16, 4, 5><<<nblk, 1024, pad4, s>>>(p);
  else if (mt == 2) stn_vae_step_kernel<2, 8, 4><<<nblk, 512, 0, s>>>(p);
  else
#endif
  if (mt == 4) stn_vae_step_kernel<4, 16, 4><<<nblk, 1024, pad4, s>>>(p);
  else stn_vae_step_kernel<2, 16, 4><<<nblk, 1024, pad3, s>>>(p);
  if (p.tstamp) {
    std::vector<long long> h((size_t)nblk * 16);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), tbuf, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
    static const char* names[10] = {"read+L1", "L1epi", "L2", "mu_lv", "sample",
                                    "g1", "g2", "go1", "go23", "write"};
    double acc[11] = {0}, pro = 0;
    long long t0 = h[0], t1 = h[10];
    for (unsigned b = 0; b < nblk; ++b) {
      for (int k = 0; k < 10; ++k) acc[k] += (double)(h[b * 16 + k + 1] - h[b * 16 + k]);
      acc[10] += (double)(h[b * 16 + 10] - h[b * 16]);
      pro += (double)(h[b * 16] - h[b * 16 + 11]);
      t0 = std::min(t0, h[b * 16]);
      t1 = std::max(t1, h[b * 16 + 10]);
    }
    fprintf(stderr, "stn_vae_step M=%d phases (us, mean over %u blocks; 100 MHz clock): prologue %.2f",
            M, nblk, pro / nblk / 100.0);
    for (int k = 0; k < 10; ++k) fprintf(stderr, " %s %.2f", names[k], acc[k] / nblk / 100.0);
    fprintf(stderr, " | block %.2f | span %.2f\n", acc[10] / nblk / 100.0, (t1 - t0) / 100.0);
  }
  MOG_LAUNCH_RET();
}

// fp32 B-fragment packs of n <= 8 weight matrices (W[i] [K[i]][N[i]] fp32 ->
// out[i], (K + 15) / 16 * (N + 15) / 16 KiB), see stn_vae_step_f32_kernel
extern "C" int mog_pack_frag_f32(int n, const float* const* W, const int* K, const int* N,
                                 float* const* out, void* stream) {
  MOG_CHECK_ARG(n >= 1 && n <= 8 && W && K && N && out);
  PackF32 a = {};
  long most = 0;
  for (int i = 0; i < n; ++i) {
    MOG_CHECK_ARG(W[i] && out[i] && K[i] > 0 && N[i] > 0);
    a.W[i] = W[i]; a.out[i] = out[i]; a.K[i] = K[i]; a.N[i] = N[i];
    most = std::max(most, (long)((K[i] + 15) / 16) * ((N[i] + 15) / 16) * 256);
  }
  const dim3 grid((unsigned)std::min<long>(1024, (most + 255) / 256), n);
  pack_frag_f32_kernel<<<grid, 256, 0, mog_stream(stream)>>>(a);
  MOG_LAUNCH_RET();
}

// The fp32 fused step (see stn_vae_step_f32_kernel): the arguments of
// mog_stn_vae_step_forward with fp32 weight packs (mog_pack_frag_f32) and the
// fp32 saved activations of the unfused sequence (g, a1pre, a1, a2pre, a2,
// mu, lv, d1pre, d1, d2pre, d2: all given, or all NULL for a forward-only
// step); z and r are always written.
extern "C" int mog_stn_vae_step_forward_f32(
    int B, int C, const float* x, const float* theta_f, const float* theta_b, const float* mask,
    const float* zval, const float* eps_z, const float* eps_x, int eps_gen,
    unsigned long long eps_seed, unsigned long long eps_offset, const float* const* wt,
    const float* const* bias, float lik_std, float v_pm, float v_pv, float v_plv,
    float* canvas_part, int* part_rows, float* runloss, float* vkl, float* g, float* a1pre,
    float* a1, float* a2pre, float* a2, float* mu, float* lv, float* z, float* d1pre, float* d1,
    float* d2pre, float* d2, float* r, int x_period, void* stream) {
  MOG_CHECK_ARG(B >= 0 && C >= 2 && C * C <= 16384);
  MOG_CHECK_ARG(x && theta_f && theta_b && mask && zval && eps_z && (eps_x || eps_gen) && wt && bias);
  MOG_CHECK_ARG(canvas_part && part_rows && vkl && z && r);
  const bool save = a1 != nullptr;
  // (the pre-activations are optional: the backward reads the outputs)
  MOG_CHECK_ARG(!save || (g && a1 && a2 && mu && lv && d1 && d2));
  MOG_CHECK_ARG(save || !(g || a1pre || a2pre || a2 || mu || lv || d1pre || d1 || d2pre || d2));
  if (B == 0) return 0;
  StepArgsF p;
  p.x = x; p.theta_f = theta_f; p.theta_b = theta_b; p.mask = mask; p.zval = zval;
  p.eps_z = eps_z; p.eps_x = eps_x;
  p.eps_gen = eps_gen; p.eps_seed = eps_seed; p.eps_offset = eps_offset;
  for (int i = 0; i < 7; ++i) {
    MOG_CHECK_ARG(wt[i] && bias[i]);
    p.wt[i] = wt[i];
    p.bias[i] = bias[i];
  }
  p.part = canvas_part; p.part_rows = part_rows; p.runloss = runloss; p.vkl = vkl;
  p.g = g; p.a1pre = a1pre; p.a1 = a1; p.a2pre = a2pre; p.a2 = a2; p.mu = mu; p.lv = lv; p.z = z;
  p.d1pre = d1pre; p.d1 = d1; p.d2pre = d2pre; p.d2 = d2; p.r = r;
  p.B = B; p.C = C; p.lik_std = lik_std; p.v_pm = v_pm; p.v_pv = v_pv; p.v_plv = v_plv;
  p.x_period = x_period > 0 ? x_period : B;
  p.phases = 31;
  // a tile must not straddle two periods of x; several steps' rows in one
  // launch rule out the running loss (mog_air_runloss replays it)
  MOG_CHECK_ARG(p.x_period == B || (p.x_period % FM == 0 && !runloss));
  hipStream_t s = mog_stream(stream);
  const unsigned nblk = mog_cdiv(B, FM);
  static long long* tbuf = nullptr;
  static size_t tcap = 0;
  p.tstamp = nullptr;
  if (mog_prof_env("MOG_VS_TIMING")) {
    if (tcap < (size_t)nblk * 16) {
      if (tbuf) (void)hipFree(tbuf);
      tcap = (size_t)nblk * 16;
      if (hipMalloc(&tbuf, tcap * sizeof(long long)) != hipSuccess) return MOG_ERR_INVALID;
    }
    p.tstamp = tbuf;
  }
  static const long padf = lds_pad(stn_vae_step_f32_kernel);  // (see lds_pad)
  if (padf < 0) return MOG_ERR_INVALID;
  stn_vae_step_f32_kernel<<<nblk, 1024, padf, s>>>(p);
  if (p.tstamp) {
    std::vector<long long> h((size_t)nblk * 16);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), tbuf, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
    static const char* names[10] = {"read+L1", "L1epi", "L2", "mu_lv", "sample",
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
    fprintf(stderr, "stn_vae_step_f32 M=%d phases (us, mean over %u blocks; 100 MHz clock): prologue %.2f",
            FM, nblk, pro / nblk / 100.0);
    for (int k = 0; k < 10; ++k) fprintf(stderr, " %s %.2f", names[k], acc[k] / nblk / 100.0);
    fprintf(stderr, " | block %.2f | span %.2f\n", acc[10] / nblk / 100.0, (t1 - t0) / 100.0);
  }
  MOG_LAUNCH_RET();
}
