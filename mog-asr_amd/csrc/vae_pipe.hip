// Fused per-object step, pipelined form: STN read -> glimpse VAE -> latent
// sample + KL -> STN write (air_model.py:500-588 + :718-736, vae.py:5-48,
// transformer.py:18-175) with two tiles in flight per CU.  Same arithmetic,
// element for element, as stn_vae_step_kernel (vae_step.hip) and the unfused
// bf16 sequence; SURVEY.md §8 D.3 prices it at 30,024 algorithmic HBM bytes
// per image-step.
//
// Why a second form.  The lockstep kernel runs every phase of a 64-image tile
// with all 16 waves of the CU's one workgroup, so a launch pays the SUM of the
// per-phase floors: the HBM gather of the STN read, the L2 -> CU weight stream
// of the dense layers, the canvas-part stores of the STN write and the tile
// bookkeeping.  Here one persistent workgroup per CU walks
// its tiles with the waves split by role, each role on a different tile:
//   * M role (waves 0-7): the seven dense layers of tile i -- recognition
//     layer (its glimpse operand brought back from L2 into an LDS slab ring
//     by LDS-DMA), mu / logvar, latent sample + VAE KL, decoder and output
//     layer with in-kernel Philox noise -> r (HBM);
//   * S role (waves 8-15): tile i+1's STN read (gather + bilinear sample ->
//     the saved glimpse gb, normal stores so that the M role's DMA finds it in
//     L2), tile i-1's STN write (r -> canvas part rows), tile i+2's
//     bookkeeping (theta, masks, read tables).
// The roles meet only through three LDS counters: "glimpse of tile i in L2"
// (S -> M), "r of tile i in L2" (M -> S) and each role's own barrier between
// the phases that reuse its LDS.  So the weight stream, the gathers and the
// part stores of different tiles overlap on one CU, and a launch pays roughly
// max(M role, S role) per tile plus one tile of fill and drain.
//
// Every spin has a bound (a role that never arrives cannot hang the GPU: the
// waiting waves give up after ~0.2 s and the results are garbage, which the
// parity tests catch).
#include "vae_tile.h"

namespace {

constexpr int PM = 64, PMT = 4;   // images per tile, 16-row MFMA tiles
#ifndef MOG_PIPE_WAVES
#define MOG_PIPE_WAVES 4
#endif
// waves per role: 4 + 4 (one of each per SIMD, 256 registers) or 8 + 8 (128)
constexpr int MW = MOG_PIPE_WAVES, SW = MOG_PIPE_WAVES;
constexpr int MTHR = MW * 64;     // M-role threads (tid 0..255)
constexpr int NTHR_P = (MW + SW) * 64;
constexpr int KGP = 5;            // recognition k-steps per DMA slab
constexpr int NGP = KS1 / KGP;    // slabs per tile
static_assert(KS1 % KGP == 0, "slabs");
constexpr int SSTG = 64 + 8;      // S staging row stride (bf16): 2 k-steps of one image
constexpr int SIMG = PM / SW;     // images per sampler wave (16)
constexpr int SNU = SIMG / 2;     // gather groups per lane (two images per wave-instruction)

// LDS map (bytes).  M region: the activation arena of Lay<4, *> (a1 / a2 /
// mu / lv / kl / z / d1 / d2), the recognition slab ring inside it (dead once
// a1 is written), eps_z of the tile behind it.  S region: read tables +
// per-wave sample staging, or (later in the period) the STN write slots.
// Records: two slots of per-tile scalars (the tile being sampled, the tile
// being written).
struct LayP {
  using L = Lay<PMT, 16>;
  static constexpr int ARENA = cmax(L::A1, L::OFF_D1 + L::A2);
  static constexpr int SLAB = KGP * PMT * 1024;  // 5 k-steps x 4 row tiles x 1 KiB
  static_assert(3 * SLAB <= ARENA, "slab ring inside the arena");
  static constexpr int OFF_EZ = ARENA;             // eps_z [64][50] fp32 (13 DMA pieces)
  static constexpr int S_BASE = OFF_EZ + 13 * 1024;
  static constexpr int TAB = PM * TABR * 16;
  static constexpr int STG = SW * SIMG * SSTG * 2;
  static constexpr int WS = SW * L::WSLOT;
  static constexpr int S_SIZE = cmax(TAB + STG, WS);
  static constexpr int REC = S_BASE + S_SIZE;
  static constexpr int REC_SLOT = PM * 12 * 4 + 4 * PM * 4;  // sth, szv, smask, ssep + flag
  static constexpr int CTR = REC + 2 * REC_SLOT;
  static constexpr int TOTAL = CTR + 64;
};
static_assert(LayP::TOTAL <= 160 * 1024, "LDS");

struct Rec {
  float (*sth)[12];
  float* szv;
  int* smask;
  int* ssep;
  int* flag;  // 1: some image of the tile has a non-axis-aligned theta_f
};
__device__ __forceinline__ Rec rec_slot(unsigned char* lds, int slot) {
  unsigned char* b = lds + LayP::REC + slot * LayP::REC_SLOT;
  Rec r;
  r.sth = reinterpret_cast<float(*)[12]>(b);
  r.szv = reinterpret_cast<float*>(b + PM * 48);
  r.smask = reinterpret_cast<int*>(b + PM * 52);
  r.ssep = reinterpret_cast<int*>(b + PM * 56);
  r.flag = reinterpret_cast<int*>(b + PM * 60);
  return r;
}

constexpr unsigned SPIN_MAX = 1u << 22;

// Counter barrier of one role's n waves (LDS counter, no s_barrier: the other
// role keeps running).  The generation is recovered from the value the
// wave's own add returns, so no per-wave state is needed.
// (LDS ordering only: a workgroup-scope fence builtin could also drain the
// wave's outstanding global loads and stores, which must stay in flight)
__device__ __forceinline__ void lds_release() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void lds_acquire() { asm volatile("" ::: "memory"); }
__device__ __forceinline__ void role_bar(unsigned* ctr, unsigned n) {
  lds_release();
  unsigned old = 0;
  if ((threadIdx.x & 63) == 0)
    old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = __builtin_amdgcn_readfirstlane(old);
  const unsigned target = (old / n + 1) * n;
  for (unsigned it = 0; it < SPIN_MAX; ++it) {
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
    __builtin_amdgcn_s_sleep(1);
  }
  lds_acquire();
}
// wait until a hand-off counter reaches `target`
__device__ __forceinline__ void role_wait(unsigned* ctr, unsigned target) {
  for (unsigned it = 0; it < SPIN_MAX; ++it) {
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
    __builtin_amdgcn_s_sleep(2);
  }
  lds_acquire();
}
// this wave's global stores are done (in L2), then count the wave in
__device__ __forceinline__ void role_signal(unsigned* ctr) {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct RoleBar {
  unsigned* ctr;
  __device__ __forceinline__ void operator()() const { role_bar(ctr, MW); }
};

__device__ __forceinline__ void stamp(const StepArgs& p, int li, int k) {
  if (p.tstamp && (threadIdx.x & 63) == 0)
    p.tstamp[((size_t)blockIdx.x * 8 + li) * 16 + k] = wall_clock64();
}

// Per-tile values the compiler must not hoist out of the persistent tile
// loop: the per-lane address math of every layer would otherwise be computed
// once before the loop and stay live across all of it (and spill).  The thread
// id passes through an empty asm once per tile; the mask restores its known
// range, so the address math stays 32-bit.
__device__ __forceinline__ int tile_tid() {
  int v = threadIdx.x;
  asm volatile("" : "+v"(v));
  return v & 1023;
}
// ---- M role: the dense layers of one tile ---------------------------------
__device__ __forceinline__ void m_tile(const StepArgs& p_, unsigned char* lds, unsigned* ctr, int b0,
                                       int nb, int li_tile) {
#pragma clang fp contract(off)
  using L = Lay<PMT, 16>;
  constexpr int M = PM;
  const StepArgs& p = p_;
  const int tid = tile_tid(), lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  unsigned* mctr = ctr;
  const RoleBar mbar{mctr};
  const bool save = (p.phases & 16) != 0;
  // the previous tile's last layer has read its LDS operand
  mbar();
  role_wait(ctr + 2, (unsigned)SW * (li_tile + 1));  // tile's glimpse in L2
  stamp(p, li_tile, 0);

  // eps_z of the tile -> LDS (13 x 1 KiB LDS-DMA pieces; past the tile: 0)
  {
    const __amdgpu_buffer_rsrc_t er = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.eps_z) + (size_t)b0 * 50, 0, nb * 50 * 4, 0x00020000);
    for (int q = w; q < 13; q += MW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          er, (__attribute__((address_space(3))) void*)(lds + LayP::OFF_EZ + q * 1024), 16,
          q * 1024 + lane * 16, 0, 0, 0);
  }
  // ---- recognition layer: A = the tile's glimpse (gb, written by the S
  // role, L2-resident) through a ring of three LDS slabs of KGP k-steps,
  // filled by LDS-DMA two slabs ahead.  Piece (ks, rt) of a slab is 1 KiB:
  // lane (li, g) brings row rt*16 + li, k = 32 ks + 8 g .. +7 -- exactly its
  // MFMA A operand, so the fragment read is one linear ds_read_b128.  k past
  // 784 (the zero padding to 800) and rows past the batch read 0.
  // (descriptor over the tile's rows: rows past the batch read 0; the lane's
  // part of the offset is one register, the piece's part a scalar offset)
  const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
      p.gb + (size_t)b0 * W2, 0, nb * W2 * 2, 0x00020000);
  const int dvo = (li * W2 + 8 * g) * 2;                // k < 784 everywhere but the last k-step
  const int dvo_last = g < 2 ? dvo : 0x7ffffff0;        // k-step 24: k 784.. read 0
  auto dma_slab = [&](int s) {
    for (int j = w; j < KGP * PMT; j += MW) {
      const int ksl = j / PMT, rt = j - (j / PMT) * PMT, ks = s * KGP + ksl;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          gr, (__attribute__((address_space(3))) void*)(lds + (s % 3) * LayP::SLAB + j * 1024), 16,
          ks == KS1 - 1 ? dvo_last : dvo, (rt * 16 * W2 + ks * 32) * 2, 0, 0);
    }
  };
  constexpr int TW = 32 / MW, DB = 2;
  floatx4 acc[PMT][TW];
  int ct[TW];
  floatx4 b1q[TW];
  {
    const int rot = (int)(blockIdx.x >> 3);
    const __amdgpu_buffer_rsrc_t wr = weight_rsrc(p.wt[0]);
    int wo[TW];
#pragma unroll
    for (int c = 0; c < TW; ++c) {
      ct[c] = (w + MW * c + rot) % 32;
      wo[c] = frag_voff(ct[c], lane);
    }
    bf16x8 q[DB][TW];
    auto loadB = [&](int ks, bf16x8* b) {
#pragma unroll
      for (int c = 0; c < TW; ++c) b[c] = load_frag<32>(wr, wo[c], ks);
    };
    auto mfma = [&](int ks, const bf16x8* b) {
      const int s = ks / KGP, ksl = ks - s * KGP;
      const unsigned char* sl = lds + (s % 3) * LayP::SLAB + ksl * PMT * 1024 + lane * 16;
#pragma unroll
      for (int rt = 0; rt < PMT; ++rt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(sl + rt * 1024);
#pragma unroll
        for (int c = 0; c < TW; ++c)
          acc[rt][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[c], acc[rt][c], 0, 0, 0);
      }
    };
#pragma unroll
    for (int rt = 0; rt < PMT; ++rt)
#pragma unroll
      for (int c = 0; c < TW; ++c) acc[rt][c] = floatx4{0.f, 0.f, 0.f, 0.f};
    dma_slab(0);
    dma_slab(1);
#pragma unroll
    for (int d = 0; d < DB; ++d) loadB(d, q[d]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    mbar();  // slabs 0, 1 landed everywhere
    static_for<0, KS1>([&](auto kc) {
      constexpr int ks = decltype(kc)::value;
      if constexpr (ks % KGP == 0 && ks / KGP + 2 < NGP) {
        // slab s+2 into the slot slab s-1 used (consumed before the last barrier)
        __builtin_amdgcn_sched_barrier(0);
        dma_slab(ks / KGP + 2);
        __builtin_amdgcn_sched_barrier(0);
      }
      mfma(ks, q[ks % DB]);
      if constexpr (ks + DB < KS1) loadB(ks + DB, q[ks % DB]);
      // (k-step boundary: keeps the scheduler from hoisting later weight
      // loads, whose registers the ring does not have)
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (ks % KGP == KGP - 1) {
        // own DMAs of the next slab landed, then every wave's (and this slab
        // is consumed by all before its slot is refilled)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        mbar();
      }
    });
#pragma unroll
    for (int c = 0; c < TW; ++c) b1q[c] = load_bias4(p.bias[0], ct[c] * 16 + (li & ~3), 512);
  }
  stamp(p, li_tile, 1);
  __bf16* sA1 = reinterpret_cast<__bf16*>(lds);
#pragma unroll
  for (int c = 0; c < TW; ++c) {
    const int n0 = ct[c] * 16 + (li & ~3);
#pragma unroll
    for (int rt = 0; rt < PMT; ++rt)
      store_softplus4(sA1 + (rt * 16 + g * 4 + (li & 3)) * S512 + n0, quad_transpose(acc[rt][c], tid),
                      b1q[c]);
  }
  mbar();
  stamp(p, li_tile, 8);
  // ---- a2 = softplus(a1 W2 + b2) [64 x 256], in place; a1's saved copy
  // flushed inside the k loop
  __bf16* sA2 = sA1;
  {
    RowFlush<__bf16, 512, MTHR> fl(sA1, S512, p.a1b + (size_t)b0 * 512, 512, nb, save, tid);
    dense_tiles<PMT, 512, 256, 16 / MW, 4, true>(sA1, S512, p.wt[1], p.bias[1], 0, 0, MW,
                                           [&](int m, int n0, const floatx4& v, const floatx4& b) {
                                             store_softplus4(sA2 + m * S256 + n0, v, b);
                                           },
                                           mbar, fl, tid);
  }
  mbar();
  stamp(p, li_tile, 9);
  // ---- mu | lv = a2 W + b [64 x 50] fp32 (first | second half of the waves), then a2's copy
  float* sMu = reinterpret_cast<float*>(lds + L::OFF_MU);
  float* sLv = reinterpret_cast<float*>(lds + L::OFF_LV);
  {
    auto epi_f32 = [&](float* dst) {
      return [dst](int m, int n0, const floatx4& v, const floatx4& b) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (n0 + k < 50) dst[m * 50 + n0 + k] = v[k] + b[k];
      };
    };
    dense_tiles<PMT, 256, 50, 8 / MW, 4, false>(sA2, S256, p.wt[2], p.bias[2], 0, 0, MW / 2,
                                                epi_f32(sMu), mbar,
                                           NoHook{}, tid);
    dense_tiles<PMT, 256, 50, 8 / MW, 4, false>(sA2, S256, p.wt[3], p.bias[3], 0, MW / 2, MW / 2,
                                                epi_f32(sLv), mbar,
                                           NoHook{}, tid);
    if (save) flush_rows<MTHR>(sA2, S256, p.a2b + (size_t)b0 * 256, 256, 256, nb, tid);
  }
  mbar();
  stamp(p, li_tile, 10);
  // ---- z = mu + eps sqrt(exp(lv)); VAE KL (vae.py:27-30) -------------------
  float* sKl = reinterpret_cast<float*>(lds + L::OFF_KL);
  __bf16* sZ = reinterpret_cast<__bf16*>(lds + L::OFF_Z);
  {
    constexpr int NS = M * 64 / MTHR;
    const float* sEz = reinterpret_cast<const float*>(lds + LayP::OFF_EZ);
    float ez[NS];
#pragma unroll
    for (int it = 0; it < NS; ++it) {
      const int i = tid + it * MTHR, m = i >> 6, k = i & 63;
      ez[it] = (k < 50 && m < nb) ? sEz[m * 50 + k] : 0.0f;
    }
#pragma unroll
    for (int it = 0; it < NS; ++it) {
      const int i = tid + it * MTHR, m = i >> 6, k = i & 63;
      float zv = 0.0f;
      if (k < 50 && m < nb) {
        const size_t o = (size_t)(b0 + m) * 50 + k;
        const float l = sLv[m * 50 + k];
        const float mv = sMu[m * 50 + k];
        const float var = mog_expf(l);
        zv = mv + ez[it] * sqrtf(var);
        if (p.z) st_stream(p.z + o, zv);
        if (save) {
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
  mbar();
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
    if (p.runloss && p.mask[b0 + m] != 0.0f) p.runloss[b0 + m] = p.runloss[b0 + m] + vkl;
  }
  stamp(p, li_tile, 11);
  // ---- d1 = softplus(z Wg1 + b) [64 x 256] (over mu | lv) -------------------
  __bf16* sD1 = reinterpret_cast<__bf16*>(lds + L::OFF_D1);
  dense_tiles<PMT, 64, 256, 16 / MW, 2, false>(sZ, SZ, p.wt[4], p.bias[4], 0, 0, MW,
                                         [&](int m, int n0, const floatx4& v, const floatx4& b) {
                                           store_softplus4(sD1 + m * S256 + n0, v, b);
                                         },
                                         mbar, NoHook{}, tid);
  mbar();
  stamp(p, li_tile, 12);
  // ---- d2 = softplus(d1 Wg2 + b) [64 x 512] at 0 (in place over d1) --------
  __bf16* sD2 = reinterpret_cast<__bf16*>(lds);
  {
    RowFlush<__bf16, 256, MTHR> fl(sD1, S256, p.d1b + (size_t)b0 * 256, 256, nb, save, tid);
    dense_tiles<PMT, 256, 512, 32 / MW, 2, true>(sD1, S256, p.wt[5], p.bias[5], 0, 0, MW,
                                           [&](int m, int n0, const floatx4& v, const floatx4& b) {
                                             store_softplus4(sD2 + m * S512 + n0, v, b);
                                           },
                                           mbar, fl, tid);
  }
  mbar();
  stamp(p, li_tile, 2);
  // ---- r = sigmoid(d2 Wgo + b + std eps) [64 x 784] fp32 -> HBM ------------
  // 49 column tiles: three passes of 16 (2 per wave, Philox quads inside the
  // k loop) + 1 split over the row tiles; d2's copy flushed in the first pass
  {
    const float sd = p.lik_std;
    auto epi = [&](int m, int n, const floatx4& v, const floatx4& b) {
      if (m < nb) {
        float ev[4];
        const size_t qi = (size_t)(b0 + m) * (W2 / 4) + (n >> 2);
        if (p.eps_gen) {
          mog_philox_quad(p.eps_seed, p.eps_offset + qi, true, ev);
        } else {
          const float4 e4 = reinterpret_cast<const float4*>(p.eps_x)[qi];
          ev[0] = e4.x; ev[1] = e4.y; ev[2] = e4.z; ev[3] = e4.w;
        }
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float y = __builtin_fmaf(ev[k], sd, v[k] + b[k]);
          o[k] = mog_sigmoid_hw(y);
        }
        reinterpret_cast<float4*>(p.r)[qi] = make_float4(o[0], o[1], o[2], o[3]);
      }
    };
    RowFlush<__bf16, 512, MTHR> fl(sD2, S512, p.d2b + (size_t)b0 * 512, 512, nb, save, tid);
    dense_out<PMT, 16 / MW, 4>(sD2, S512, p, 0, 0, MW, b0, nb, tid, fl);
    dense_out<PMT, 16 / MW, 4>(sD2, S512, p, 16, 0, MW, b0, nb, tid);
    dense_out<PMT, 16 / MW, 4>(sD2, S512, p, 32, 0, MW, b0, nb, tid);
    dense_rowsplit<PMT, 512, W2>(sD2, S512, p.wt[6], p.bias[6], 48, epi, tid);
  }
  stamp(p, li_tile, 3);
  role_signal(ctr + 3);  // r of the tile (and every saved activation) in L2
}

// ---- S role ---------------------------------------------------------------
// Bookkeeping of one tile into a record slot + the read tables (S waves only)
__device__ __forceinline__ void s_prologue(const StepArgs& p, unsigned char* lds, unsigned* sctr,
                                           const Rec& rc, int b0, int nb) {
  const int ts = threadIdx.x - MTHR;  // 0..511
  constexpr int STHR = SW * 64;
  const int C = p.C;
  for (int i = ts; i < PM * 12; i += STHR) {
    const int m = i / 12, k = i % 12;
    float v = 0.0f;
    if (m < nb) v = k < 6 ? p.theta_f[(size_t)(b0 + m) * 6 + k] : p.theta_b[(size_t)(b0 + m) * 6 + k - 6];
    rc.sth[m][k] = v;
  }
  if (ts < PM) {
    const bool act = ts < nb && p.mask[b0 + ts] != 0.0f;
    rc.smask[ts] = act;
    rc.szv[ts] = act ? p.zval[b0 + ts] : 0.0f;
  }
  if (ts == 0) *rc.flag = 0;
  role_bar(sctr, SW);
  if (ts < PM) {
    const bool sep_f = stn_separable(&rc.sth[ts][0]);
    rc.ssep[ts] = (sep_f ? 1 : 0) | (stn_separable(&rc.sth[ts][6]) && C <= CTAB_MAX ? 2 : 0);
    if (!sep_f) __hip_atomic_fetch_or(rc.flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  float4* tabR = reinterpret_cast<float4*>(lds + LayP::S_BASE);
  for (int i = ts; i < PM * TABR; i += STHR) {
    const int m = i / TABR, n = i - (i / TABR) * TABR;
    const float* th = rc.sth[m];
    tabR[i] = n < 28 ? col_pair4(axis_col(th, C, C, 28, 28, n), C)
                     : axis4(axis_row(th, C, C, 28, 28, n - 28), 4 * C);
  }
  role_bar(sctr, SW);
}

// STN read of one tile (transformer.py:18-175) -> gb.  Sampler wave sw owns
// images 16 sw .. 16 sw + 15; lane (kk = lane & 31, h = lane >> 5) samples
// pixel 32 ks + kk of images 16 sw + 2u + h, u < 8, gathering LA k-steps ahead.
// Samples are staged per wave two k-steps at a time and leave as 16-byte
// stores (normal policy: the M role reads them back from L2).
template <bool SEP, int LA>
__device__ __forceinline__ void s_sample(const StepArgs& p, unsigned char* lds, const Rec& rc,
                                         int b0, int nb) {
#pragma clang fp contract(off)
  constexpr int NU = SNU;
  const int tid = threadIdx.x, lane = tid & 63;
  const int sw = __builtin_amdgcn_readfirstlane((tid >> 6) - MW);
  const int C = p.C, C2 = C * C;
  const float4* tabR = reinterpret_cast<const float4*>(lds + LayP::S_BASE);
  auto opaque = [](int v) {
    asm volatile("" : "+v"(v));
    return v;
  };
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(p.x) + (size_t)(b0 % p.x_period) * C2, 0, nb * C2 * 4, 0x00020000);
  const int kk = lane & 31, h = lane >> 5;
  const int mw = sw * SIMG + h;                                // the lane's first image
  const int tabo = LayP::S_BASE + mw * TABR * 16;
  __bf16* stg = reinterpret_cast<__bf16*>(lds + LayP::S_BASE + LayP::TAB + sw * SIMG * SSTG * 2);
  float I[LA][NU][4];
  auto gather = [&](int ks, float (&I)[NU][4]) {
    const int k = 32 * ks + kk;
    const int i = min(k / 28, 27), j = k - (k / 28) * 28;
    const float4* tc = reinterpret_cast<const float4*>(lds + opaque(tabo + j * 16));
    const float4* tr = reinterpret_cast<const float4*>(lds + opaque(tabo + (28 + i) * 16));
    int xo = mw * C2 * 4;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int m = mw + 2 * u;
      float4 ex, ey;
      if constexpr (SEP) {
        ex = tc[2 * u * TABR];
        ey = tr[2 * u * TABR];
      } else {
        glimpse_geom<false>(tabR, rc.sth[m], m, k, C, ex, ey);
      }
      const int xb = __float_as_int(ex.x) + xo;
      const u32x2 r0 = __builtin_amdgcn_raw_buffer_load_b64(xr, xb + __float_as_int(ey.x), 0, 0);
      const u32x2 r1 = __builtin_amdgcn_raw_buffer_load_b64(xr, xb + __float_as_int(ey.y), 0, 0);
      I[u][0] = __uint_as_float(r0[0]);
      I[u][1] = __uint_as_float(r0[1]);
      I[u][2] = __uint_as_float(r1[0]);
      I[u][3] = __uint_as_float(r1[1]);
      xo += 2 * C2 * 4;
    }
  };
  auto sample = [&](int ks, const float (&I)[NU][4]) {
    const int k = 32 * ks + kk;
    const int i = min(k / 28, 27), j = k - (k / 28) * 28;
    asm volatile("" ::: "memory");  // re-read the tables instead of keeping them live
    const float4* tc = reinterpret_cast<const float4*>(lds + opaque(tabo + j * 16));
    const float4* tr = reinterpret_cast<const float4*>(lds + opaque(tabo + (28 + i) * 16));
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int m = mw + 2 * u;
      float4 ex, ey;
      if constexpr (SEP) {
        ex = tc[2 * u * TABR];
        ey = tr[2 * u * TABR];
      } else {
        glimpse_geom<false>(tabR, rc.sth[m], m, k, C, ex, ey);
      }
      const int fl = __float_as_int(ex.y);
      const float Ia = (fl & 1) ? I[u][1] : I[u][0], Ib = (fl & 1) ? I[u][3] : I[u][2];
      const float Ic = (fl & 2) ? I[u][1] : I[u][0], Id = (fl & 2) ? I[u][3] : I[u][2];
      const int xlive = (fl ^ (fl >> 1)) & 1;
      const int ylive = __float_as_int(ey.x) != __float_as_int(ey.y) ? 1 : 0;
      const int live = (int)(k < W2) & (int)(m < nb) & (xlive | ylive);
      const float v = sample4(ex, ey, Ia, Ib, Ic, Id);
      stg[(2 * u + h) * SSTG + (ks & 1) * 32 + kk] = (__bf16)(live ? v : 0.0f);
    }
  };
  // k-steps 2q, 2q+1 (staged) -> gb[:, 64 q ..]: lane -> images (l >> 3) and
  // (l >> 3) + 8 of the wave, 16-byte chunk l & 7
  auto flush = [&](int q) {
    wave_lds_sync();
    const int c = lane & 7, k0 = 64 * q + 8 * c;
#pragma unroll
    for (int hh = 0; hh < SIMG / 8; ++hh) {
      const int row = (lane >> 3) + 8 * hh;
      const u32x4 v = *reinterpret_cast<const u32x4*>(stg + row * SSTG + 8 * c);
      if (k0 < W2 && sw * SIMG + row < nb)
        *reinterpret_cast<u32x4*>(p.gb + (size_t)(b0 + sw * SIMG + row) * W2 + k0) = v;
    }
    wave_lds_sync();
  };
#pragma unroll
  for (int k = 0; k < LA; ++k) gather(k, I[k]);
  static_for<0, KS1>([&](auto kc) {
    constexpr int ks = decltype(kc)::value;
    sample(ks, I[ks % LA]);
    if constexpr (ks + LA < KS1) gather(ks + LA, I[ks % LA]);
    if constexpr (ks % 2 == 1 || ks == KS1 - 1) flush(ks / 2);
    __builtin_amdgcn_sched_barrier(0);
  });
}

// The persistent pipelined kernel: one 16-wave workgroup per CU, tiles
// blockIdx.x, blockIdx.x + gridDim.x, ... (at most 8 per workgroup).
template <int LA>
__global__ __launch_bounds__(NTHR_P, 8 / MW) void stn_vae_step_pipe_kernel(StepArgs p) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LayP::TOTAL];
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  unsigned* ctr = reinterpret_cast<unsigned*>(lds + LayP::CTR);  // M bar, S bar, glimpse, r
  if (tid < 4) ctr[tid] = 0;
  __syncthreads();
  const int ntiles = (p.B + PM - 1) / PM;
  const int G = (int)gridDim.x;
  const int n = ((int)blockIdx.x < ntiles) ? (ntiles - 1 - (int)blockIdx.x) / G + 1 : 0;
  auto tile_b0 = [&](int i) { return ((int)blockIdx.x + i * G) * PM; };
  if (wv < MW) {
    for (int i = 0; i < n; ++i) {
      const int b0 = tile_b0(i);
      m_tile(p, lds, ctr, b0, min(PM, p.B - b0), i);
    }
  } else {
    unsigned* sctr = ctr + 1;
    const int sw = wv - MW;
    if (n > 0) {
      const Rec r0 = rec_slot(lds, 0);
      s_prologue(p, lds, sctr, r0, tile_b0(0), min(PM, p.B - tile_b0(0)));
    }
    for (int i = 0; i <= n; ++i) {
      if (i < n) {
        const int b0 = tile_b0(i), nb = min(PM, p.B - b0);
        const Rec rc = rec_slot(lds, i & 1);
        stamp(p, i, 4);
        if (*rc.flag) s_sample<false, 3>(p, lds, rc, b0, nb);
        else s_sample<true, LA>(p, lds, rc, b0, nb);
        stamp(p, i, 5);
        role_signal(ctr + 2);  // glimpse of tile i in L2
      }
      if (i >= 1) {
        // STN write of tile i-1 once its r is in L2 (the write slots overlap
        // the read tables, which tile i's sampling is done with)
        const int b0 = tile_b0(i - 1), nb = min(PM, p.B - b0);
        const Rec rc = rec_slot(lds, (i - 1) & 1);
        role_bar(sctr, SW);
        role_wait(ctr + 3, (unsigned)MW * i);
        stamp(p, i - 1, 6);
        if (p.phases & 8)
          stn_write_tile<SW>(p.r, p.part, p.part_rows, p.C, lds + LayP::S_BASE,
                             Lay<PMT, 16>::WSLOT, rc.sth, rc.smask, rc.ssep, rc.szv, b0, nb, sw,
                             lane);
        stamp(p, i - 1, 7);
      }
      if (i + 1 < n) {
        role_bar(sctr, SW);  // write slots free again
        const int b0 = tile_b0(i + 1);
        s_prologue(p, lds, sctr, rec_slot(lds, (i + 1) & 1), b0, min(PM, p.B - b0));
      }
    }
  }
}

}  // namespace

// Launch of the pipelined form (called by mog_stn_vae_step_forward, which
// validated the arguments).  Requires the saved glimpse buffer (gb) and a
// 16-byte aligned eps_z; the caller checks that.  grid: workgroups (<= the
// CU count; tiles per workgroup <= 8).
int mog_internal_stn_vae_pipe(const StepArgs& p, int grid, int la, hipStream_t s) {
  if (p.gb == nullptr || (reinterpret_cast<size_t>(p.eps_z) & 15) != 0) return MOG_ERR_INVALID;
  if (la == 2) stn_vae_step_pipe_kernel<2><<<grid, NTHR_P, 0, s>>>(p);
  else if (la == 4) stn_vae_step_pipe_kernel<4><<<grid, NTHR_P, 0, s>>>(p);
  else stn_vae_step_pipe_kernel<3><<<grid, NTHR_P, 0, s>>>(p);
  return (int)hipGetLastError();
}
