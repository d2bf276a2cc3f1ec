// Tile-level building blocks of the fused STN-read -> glimpse-VAE ->
// STN-write step kernels (vae_step.hip): MFMA dense layers over LDS-resident activation
// tiles with weights streamed from L2 in B-fragment order, the STN read
// sampler and the STN write of a tile's canvas parts.  Everything is in an
// anonymous namespace: each translation unit gets its own copies.
// (air_model.py:500-588, vae.py:5-48, transformer.py:18-175)
#pragma once
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>
#include <vector>

#include "bf16_epi.h"
#include "philox.h"
#include "stn_geom.h"

// launch arguments of the bf16 fused step kernels (shared by both forms:
// outside the anonymous namespace, one type across translation units)
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
  float* part;               // [B, C*C] this step's canvas contribution (rows in part_rows)
  int* part_rows;            // [B] rows [lo, hi) of part that were stored: lo | hi << 16
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
  int x_period;             // image of row b is x[b % x_period] (all T steps in one launch)
  float lik_std, v_pm, v_pv, v_plv;
  int phases;               // profiling aid: bit mask of the phases to run (all by default)
  long long* tstamp;        // profiling aid: per-block phase timestamps (or null)
};

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <int V>
using IC = std::integral_constant<int, V>;

// waves per workgroup: a kernel template parameter NW, 16 (one workgroup per
// CU) or 8 (two per CU)
constexpr int W2 = 784;       // 28 x 28 glimpse
constexpr int KS1 = 25;       // recognition-layer k-steps (k padded to 800)
constexpr int S512 = 512 + 8, S256 = 256 + 8, SZ = 64 + 8;  // LDS row strides (bf16)
constexpr int KG = 5;          // recognition k-steps per glimpse slab (one barrier per slab)
constexpr int NG = KS1 / KG;   // slabs
constexpr int SK = 32 * KG + 8;  // slab row stride (bf16)
static_assert(KS1 % KG == 0, "slabs");
constexpr int TABR = 56;      // read-table entries per image: 28 columns, then 28 rows
constexpr int CTAB_MAX = 64;  // write tables for canvases up to 64 x 64

constexpr int cmax(int a, int b) { return a > b ? a : b; }

// f(IC<K>{}), f(IC<K+1>{}) ... f(IC<N-1>{}): a fully unrolled loop whose index
// is a compile-time constant in every copy (the waitcnt pass then knows
// exactly which loads are still in flight; at a rolled loop's header it
// falls back to waiting for all of them)
template <int K, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (K < N) {
    f(IC<K>{});
    static_for<K + 1, N>(f);
  }
}

// LDS arena layout (bytes) for M = 16*MT images.
//   read:   tables [M][56] float4 at 0, glimpse slabs 3 x [M][SK] bf16 behind them
//   then:   a1 [M][S512] at 0 -> a2 [M][S256] at 0 (in place), mu | lv fp32 behind a2
//   sample: kl [M][50] fp32 at 0, z [M][SZ] bf16 behind it, d1 [M][S256] at A2
//   then:   d2 [M][S512] at 0 (in place over d1)
//   write:  one slot per wave at wv * WSLOT: r [784] fp32, write tables [2C] float4
template <int MT, int NW>
struct Lay {
  static constexpr int M = 16 * MT;
  static constexpr int A1 = M * S512 * 2;
  static constexpr int TAB = M * TABR * 16;
  static constexpr int KB = M * SK * 2;  // one glimpse slab (KG k-steps)
  static constexpr int A2 = M * S256 * 2;
  static constexpr int OFF_MU = A2, OFF_LV = A2 + M * 50 * 4;
  static constexpr int OFF_KL = 0, OFF_Z = M * 50 * 4;
  static constexpr int OFF_D1 = A2;
  // STN write: one slot per wave (r of one image + its 2C write tables)
  static constexpr int WSLOT = W2 * 4 + 2 * CTAB_MAX * 16;
  static constexpr int ARENA0 =
      cmax(cmax(A1, TAB + 3 * KB), cmax(OFF_D1 + A2, cmax(OFF_LV + M * 50 * 4, NW * WSLOT)));
  static constexpr int OFF_EZ = ARENA0;        // eps_z [M][50] fp32, staged in the prologue
  static constexpr int ARENA = ARENA0 + M * 50 * 4;
  static_assert(OFF_Z + M * SZ * 2 <= A2, "kl / z behind a2");
  static_assert(OFF_LV + M * 50 * 4 <= OFF_D1 + A2, "mu / lv");
};


// Workgroup barrier for LDS hand-offs only: unlike __syncthreads() it does not
// drain the wave's global stores (activation flushes, canvas parts), which stay
// in flight across phases.  The one global hand-off (r, output layer -> STN
// write) waits for its stores explicitly.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// wave-local LDS ordering (a wave's DS operations complete in order; this
// keeps the compiler from moving LDS accesses across the point)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


// value of lane (lane ^ 1) / (lane ^ 2) of the same quad
__device__ __forceinline__ float quad_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float quad_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}

// 4 x 4 transpose inside lane quads (two DPP exchanges): on entry lane
// (li = lane & 15, g = lane >> 4) holds an MFMA 16 x 16 accumulator's rows
// g*4 + r, r < 4, of column li; on exit it holds row g*4 + (li & 3) at the
// four consecutive columns (li & ~3) + r.
__device__ __forceinline__ floatx4 quad_transpose(const floatx4& a, int tid = threadIdx.x) {
  const int e = tid & 3;
  float r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3];
  {
    const bool hi = (e & 2) != 0;
    const float t0 = quad_xor2(hi ? r0 : r2), t1 = quad_xor2(hi ? r1 : r3);
    if (hi) { r0 = t0; r1 = t1; } else { r2 = t0; r3 = t1; }
  }
  {
    const bool od = (e & 1) != 0;
    const float t0 = quad_xor1(od ? r0 : r1), t1 = quad_xor1(od ? r2 : r3);
    if (od) { r0 = t0; r2 = t1; } else { r1 = t0; r3 = t1; }
  }
  return floatx4{r0, r1, r2, r3};
}

// Weight fragments (1 KiB per wave per k-step) through a buffer descriptor:
// the per-lane offset is fixed per column tile and the k-step goes into the
// scalar offset, so a fragment load costs no vector ALU address arithmetic.
// Layout k-step major (mog_cvt_bf16_batch transpose 2): fragment (ks, ct) at
// (ks * NCT + ct) KiB, NCT = the layer's 16-column tiles -- the column tiles
// that the waves and CUs stream at the same k-step are adjacent in memory
// (spread over the L2 channels) instead of a column tile's K-long run apart.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t weight_rsrc(const __bf16* W) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(W), 0, 0x7ffffff0, 0x00020000);
}
__device__ __forceinline__ int frag_voff(int ct, int lane) { return (ct * 64 + lane) * 16; }
template <int NCT>
__device__ __forceinline__ bf16x8 load_frag(__amdgpu_buffer_rsrc_t r, int voff, int ks) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, ks * NCT * 1024, 0);
  return __builtin_bit_cast(bf16x8, v);
}
constexpr int nct(int N) { return (N + 15) / 16; }

// Streaming stores (saved activations, canvas parts: written once, read by
// later launches) carry the non-temporal hint so they do not evict the bf16
// weights, which every tile of every CU re-streams, from the XCD's L2.  r stays
// a normal store: the STN write phase reads it back.
template <class T>
__device__ __forceinline__ void st_stream(T* p, T v) {
  __builtin_nontemporal_store(v, p);
}

// bias[n0 .. n0+3] (0 past N): four loads from clamped indices, selected
// afterwards (a branch between a vector and a scalar form compiled to a load
// under exec masking with a vmcnt(0) wait inside it)
__device__ __forceinline__ floatx4 load_bias4(const float* __restrict__ bias, int n0, int N) {
  floatx4 b;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float v = bias[min(n0 + k, N - 1)];
    b[k] = n0 + k < N ? v : 0.0f;
  }
  return b;
}

// softplus of v + b as four bf16 -> one 8-byte LDS store
__device__ __forceinline__ void store_softplus4(__bf16* dst, const floatx4& v, const floatx4& b) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = (__bf16)mog_softplus_hw(v[k] + b[k]);
  *reinterpret_cast<bf16x4*>(dst) = o;
}

// Axis tables of `nimg` images' transforms (th at sth[m0 + m][th_off]):
// tab[m*per + n], n < Wout columns then Hout rows, as {coordinate, lo | hi<<16}.
template <int NTHR>
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

// Column tiles tile_base + (w + nw*c + rot) % (nw*TPW) of one dense layer over
// the M = 16*MT rows held in LDS, for waves wbase .. wbase+nw-1.  A: LDS
// [M][lda] bf16, zero-padded to K.  W: the layer's W^T in B-fragment order
// (mog_cvt_bf16_batch transpose 2; N padded to 16, K to 32, zeros outside), so
// each B fragment is one 1-KiB contiguous wave load streamed from L2 straight
// into the MFMA, with a register prefetch ring of D k-steps (rolled,
// branch-free body; the ragged tail is peeled at compile time).  SYNC: the
// whole workgroup meets after the k loop (the epilogue overwrites A; requires
// nw == NW).  Epilogue per 16 x 16 accumulator tile, quad-transposed:
// epi(m, n0, v, b) with v = row m's columns n0 .. n0+3 and b = their biases
// (loaded before the k loop; 0 at or past N).
struct LdsBarrier {
  __device__ __forceinline__ void operator()() const { lds_barrier(); }
};
struct NoHook {
  __device__ __forceinline__ void operator()() const {}
  __device__ __forceinline__ void step() {}
};

// The LDS -> HBM copy of a saved activation (rows [nb] x NCOL of T, LDS row
// stride lds) spread over the k loop of the NEXT dense layer: every k-step
// each thread moves one 16-byte chunk (the waves wait on the weight stream
// there), finish() moves what is left before that layer overwrites its input.
template <class T, int NCOL, int NTHR>
struct RowFlush {
  static constexpr int V = 16 / sizeof(T), CPR = NCOL / V;
  const T* s;
  T* g;
  int lds, ldg, total, i;
  __device__ __forceinline__ RowFlush(const T* s_, int lds_, T* g_, int ldg_, int nb, bool on,
                                      int tid)
      : s(s_), g(g_), lds(lds_), ldg(ldg_), total(on ? nb * CPR : 0), i(tid) {}
  __device__ __forceinline__ void step() {
    if (i < total) {
      const int m = i / CPR, c = i - (i / CPR) * CPR;
      __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(s + m * lds + c * V),
                                  reinterpret_cast<u32x4*>(g + (size_t)m * ldg + c * V));
      i += NTHR;
    }
  }
  __device__ __forceinline__ void operator()() {
    while (i < total) step();
  }
};

// Bar: the barrier SYNC uses; Hook: step() once per k-step (a RowFlush
// spreading the previous activation's copy over the k loop), operator() by
// every participating wave right after its last read of A (before the
// epilogue).
template <int MT, int K, int N, int TPW, int D, bool SYNC, class Epi, class Bar = LdsBarrier,
          class Hook = NoHook>
__device__ __forceinline__ void dense_tiles(const __bf16* A, int lda, const __bf16* __restrict__ W,
                                            const float* __restrict__ bias, int tile_base,
                                            int wbase, int nw, Epi epi, Bar bar = Bar{},
                                            Hook hook = Hook{}, int tid = threadIdx.x) {
  constexpr int KS = K / 32, NCT = nct(N);
  static_assert(K % 32 == 0, "K padding");
  const int rot = (int)(blockIdx.x >> 3);  // spread the CUs of one XCD over the weight columns
  const int lane = tid & 63, w = (tid >> 6) - wbase;
  const bool on = w >= 0 && w < nw;
  const int li = lane & 15, g = lane >> 4;
  int ct[TPW], wo[TPW];
  const __amdgpu_buffer_rsrc_t wr = weight_rsrc(W);
#pragma unroll
  for (int c = 0; c < TPW; ++c) {
    ct[c] = tile_base + (w + nw * c + rot) % (nw * TPW);
    wo[c] = frag_voff(ct[c], lane);
  }
  // biases loaded before the k loop (their latency off the epilogue), except
  // for four or more column tiles per wave, where those registers would push
  // the k loop's accumulators + weight ring past the 128-register budget
  constexpr bool LATE_BIAS = TPW >= 4;
  floatx4 bq[TPW];
  if constexpr (!LATE_BIAS) {
#pragma unroll
    for (int c = 0; c < TPW; ++c) bq[c] = on ? load_bias4(bias, ct[c] * 16 + (li & ~3), N) : floatx4{};
  }
  floatx4 acc[MT][TPW];
#pragma unroll
  for (int rt = 0; rt < MT; ++rt)
#pragma unroll
    for (int c = 0; c < TPW; ++c) acc[rt][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto loadB = [&](int ks, bf16x8* b) {
#pragma unroll
    for (int c = 0; c < TPW; ++c) b[c] = load_frag<NCT>(wr, wo[c], ks);
  };
  auto step = [&](int ks, const bf16x8* b) {
    const int k = ks * 32 + 8 * g;
#pragma unroll
    for (int rt = 0; rt < MT; ++rt) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(&A[(rt * 16 + li) * lda + k]);
#pragma unroll
      for (int c = 0; c < TPW; ++c)
        acc[rt][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[c], acc[rt][c], 0, 0, 0);
    }
    hook.step();
  };
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
  hook();
  if constexpr (SYNC) bar();
  if (!on) return;
  if constexpr (LATE_BIAS) {
#pragma unroll
    for (int c = 0; c < TPW; ++c) bq[c] = load_bias4(bias, ct[c] * 16 + (li & ~3), N);
  }
#pragma unroll
  for (int c = 0; c < TPW; ++c)
#pragma unroll
    for (int rt = 0; rt < MT; ++rt)
      epi(rt * 16 + g * 4 + (li & 3), ct[c] * 16 + (li & ~3), quad_transpose(acc[rt][c], tid), bq[c]);
}

// One column tile `ct` of a dense layer split by rows: wave w < MT computes
// row tile w (for a last, odd column tile that would otherwise leave seven
// waves idle).
template <int MT, int K, int N, class Epi>
__device__ __forceinline__ void dense_rowsplit(const __bf16* A, int lda, const __bf16* __restrict__ W,
                                               const float* __restrict__ bias, int ct, Epi epi,
                                               int tid = threadIdx.x) {
  constexpr int KS = K / 32, D = 4, NCT = nct(N);
  static_assert(KS % D == 0, "ring");
  const int lane = tid & 63, rt = tid >> 6;
  if (rt >= MT) return;
  const int li = lane & 15, g = lane >> 4;
  const floatx4 bq = load_bias4(bias, ct * 16 + (li & ~3), N);
  const __amdgpu_buffer_rsrc_t wr = weight_rsrc(W);
  const int wo = frag_voff(ct, lane);
  floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
  bf16x8 q[D];
#pragma unroll
  for (int d = 0; d < D; ++d) q[d] = load_frag<NCT>(wr, wo, d);
#pragma unroll 1
  for (int ks = 0; ks < KS; ks += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(&A[(rt * 16 + li) * lda + (ks + d) * 32 + 8 * g]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, q[d], acc, 0, 0, 0);
      q[d] = load_frag<NCT>(wr, wo, min(ks + d + D, KS - 1));
    }
  }
  epi(rt * 16 + g * 4 + (li & 3), ct * 16 + (li & ~3), quad_transpose(acc, tid), bq);
}

// The VAE output layer r = sigmoid(d2 Wgo + b + std * eps_x) (vae.py:44-46)
// over column tiles tile_base + .. (dense_tiles' assignment, K = 512, N = 784)
// with the likelihood noise produced INSIDE the k loop: the waves wait on the
// weight stream there with the VALU idle, so each odd k-step computes one
// Philox4x32-10 quad of eps_x (or loads the injected one) for an accumulator
// tile of the lane -- the quads the epilogue needs after the quad transpose
// (lane row g*4 + (li & 3), columns (li & ~3) .. +3: one quad).  Same
// counters, same arithmetic as the epilogue form: bit-identical.
template <int MT, int TPW, int D, class Hook = NoHook>
__device__ __forceinline__ void dense_out(const __bf16* A, int lda, const StepArgs& p, int tile_base,
                                          int wbase, int nw, int b0, int nb, int tid,
                                          Hook hook = Hook{}) {
#pragma clang fp contract(off)
  constexpr int K = 512, N = W2, KS = K / 32, NCT = nct(N), NQ = MT * TPW;
  static_assert(NQ <= KS, "one noise quad per k-step at most");
  const int rot = (int)(blockIdx.x >> 3);
  const int lane = tid & 63, w = (tid >> 6) - wbase;
  const bool on = w >= 0 && w < nw;
  const int li = lane & 15, g = lane >> 4;
  int ct[TPW], wo[TPW];
  const __amdgpu_buffer_rsrc_t wr = weight_rsrc(p.wt[6]);
#pragma unroll
  for (int c = 0; c < TPW; ++c) {
    ct[c] = tile_base + (w + nw * c + rot) % (nw * TPW);
    wo[c] = frag_voff(ct[c], lane);
  }
  floatx4 bq[TPW];
#pragma unroll
  for (int c = 0; c < TPW; ++c) bq[c] = on ? load_bias4(p.bias[6], ct[c] * 16 + (li & ~3), N) : floatx4{};
  floatx4 acc[MT][TPW];
#pragma unroll
  for (int rt = 0; rt < MT; ++rt)
#pragma unroll
    for (int c = 0; c < TPW; ++c) acc[rt][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  float ev[NQ][4];
  auto noise = [&](int idx) {
    const int rt = idx / TPW, c = idx - (idx / TPW) * TPW;
    const int m = rt * 16 + g * 4 + (li & 3), n = ct[c] * 16 + (li & ~3);
    const size_t q = (size_t)(b0 + m) * (W2 / 4) + (n >> 2);
    if (p.eps_gen) {
      mog_philox_quad(p.eps_seed, p.eps_offset + q, true, ev[idx]);
    } else {
      const float4 e4 = m < nb ? reinterpret_cast<const float4*>(p.eps_x)[q] : float4{};
      ev[idx][0] = e4.x; ev[idx][1] = e4.y; ev[idx][2] = e4.z; ev[idx][3] = e4.w;
    }
  };
  if (on) {
    bf16x8 q[D][TPW];
    auto loadB = [&](int ks, bf16x8* b) {
#pragma unroll
      for (int c = 0; c < TPW; ++c) b[c] = load_frag<NCT>(wr, wo[c], ks);
    };
#pragma unroll
    for (int d = 0; d < D; ++d) loadB(d, q[d]);
    static_for<0, KS>([&](auto kc) {
      constexpr int ks = decltype(kc)::value;
      const int k = ks * 32 + 8 * g;
#pragma unroll
      for (int rt = 0; rt < MT; ++rt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&A[(rt * 16 + li) * lda + k]);
#pragma unroll
        for (int c = 0; c < TPW; ++c)
          acc[rt][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, q[ks % D][c], acc[rt][c], 0, 0, 0);
      }
      if constexpr (ks + D < KS) loadB(ks + D, q[ks % D]);
      if constexpr (ks % (KS / NQ) == KS / NQ - 1) noise(ks / (KS / NQ));
      if constexpr (ks % 4 == 1) hook.step();  // (the rest of a flush: hook())
    });
  }
  hook();
  if (!on) return;
  const float sd = p.lik_std;
#pragma unroll
  for (int c = 0; c < TPW; ++c)
#pragma unroll
    for (int rt = 0; rt < MT; ++rt) {
      const int m = rt * 16 + g * 4 + (li & 3), n = ct[c] * 16 + (li & ~3);
      const floatx4 v = quad_transpose(acc[rt][c], tid);
      const float* e = ev[rt * TPW + c];
      if (m < nb) {
        float o[4];
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) {
          const float y = __builtin_fmaf(e[kq], sd, v[kq] + bq[c][kq]);
          o[kq] = mog_sigmoid_hw(y);
        }
        reinterpret_cast<float4*>(p.r)[(size_t)(b0 + m) * (W2 / 4) + (n >> 2)] =
            make_float4(o[0], o[1], o[2], o[3]);
      }
    }
}

// LDS tile [nb][lds] -> HBM rows [nb][ldg] with 16-byte stores (ncols * sizeof(T) % 16 == 0).
template <int NTHR, class T>
__device__ __forceinline__ void flush_rows(const T* s, int lds, T* g, int ldg, int ncols, int nb,
                                           int tid = threadIdx.x) {
  constexpr int V = 16 / sizeof(T);
  const int cpr = ncols / V;
  for (int i = tid; i < nb * cpr; i += NTHR) {
    const int m = i / cpr, c = i - (i / cpr) * cpr;
    st_stream(reinterpret_cast<u32x4*>(g + (size_t)m * ldg + c * V),
              *reinterpret_cast<const u32x4*>(s + m * lds + c * V));
  }
}

#define STAMP(k) \
  if (p.tstamp && threadIdx.x == 0) p.tstamp[blockIdx.x * 16 + (k)] = wall_clock64()

// Column entry of the STN read in pair form: the two corner columns lo, hi
// (hi == lo + 1, or lo == hi when clipped) are always inside the pixel pair
// (xb, xb + 1), xb = min(lo, Win - 2), which one 8-byte load per corner row
// fetches: {xb * 4 (byte offset), lo != xb | (hi != xb) << 1 (int bits),
// hi - c, c - lo}.  Corner values: U[y][lo] = pair[flag0], U[y][hi] = pair[flag1];
// lo == hi exactly when the two flags agree.
__device__ __forceinline__ float4 col_pair4(float2 e, int Win) {
  const int lo = axis_lo(e), hi = axis_hi(e), xb = min(lo, Win - 2);
  return make_float4(__int_as_float(xb * 4), __int_as_float((lo != xb ? 1 : 0) | (hi != xb ? 2 : 0)),
                     (float)hi - e.x, e.x - (float)lo);
}

// Glimpse sample geometry (transformer.py:48-116) for glimpse pixel k < 800 of
// image m: column entry in pair form (col_pair4), row entry {lo, hi (byte
// offsets, int bits), hi - c, c - lo}: from the LDS tables (axis-aligned
// transforms) or per sample.
template <bool SEP>
__device__ __forceinline__ void glimpse_geom(const float4* tabR, const float* th, int m, int k, int C,
                                             float4& ex, float4& ey) {
  const int i = min(k / 28, 27), j = k - (k / 28) * 28;
  if constexpr (SEP) {
    ex = tabR[m * TABR + j];
    ey = tabR[m * TABR + 28 + i];
  } else {
    const Tap t = stn_tap(th, C, C, mog_linspace(j, 28), mog_linspace(i, 28));
    ex = col_pair4(make_float2(t.x, __int_as_float((int)t.x0f | ((int)t.x1f << 16))), C);
    ey = make_float4(__int_as_float((int)t.y0f * C * 4), __int_as_float((int)t.y1f * C * 4),
                     t.y1f - t.y, t.y - t.y0f);
  }
}

// STN read pipelined into the recognition layer a1 = softplus(g W1 + b1),
// with the workgroup split by role: waves 8-15 (samplers) gather and sample
// the glimpse, waves 0-7 (MFMA waves, four of the 32 column tiles each) run
// the MFMAs, so the sampling VALU work and the matrix work overlap.  The
// glimpse passes through a ring of three LDS slabs of KG k-steps (KG*32
// pixels of all M images): while the MFMA waves consume slab g, the samplers
// fill slab g+1 and flush slab g-1 to HBM (the saved glimpse); one workgroup
// barrier per slab.  The samplers' gathers run LA k-steps ahead of the
// samples (HBM latency).  A sampler lane samples pixel 32ks + (lane&31) of its
// wave's images sw*M/8 + 2u + (lane>>5), u < M/16.
template <int MT, int NW, bool SEP, int LA = 3>
__device__ __forceinline__ void read_recognition(const StepArgs& p, unsigned char* arena,
                                                 const float (*sth)[12], int b0, int nb,
                                                 floatx4 (&acc)[MT][64 / NW], int (&ct)[64 / NW],
                                                 floatx4 (&b1q)[64 / NW]) {
#pragma clang fp contract(off)
  using Ly = Lay<MT, NW>;
  constexpr int M = Ly::M;
  constexpr int NTHR = NW * 64;
  constexpr int TW = 64 / NW;          // recognition column tiles per MFMA wave (32 over NW/2)
  constexpr int NU = M / NW;           // gather instructions (two images each) per sampler lane
  constexpr int DB = NW == 16 ? 2 : 1; // weight-fragment ring depth (register budget)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bool sampler = wv >= NW / 2;
  const int li = lane & 15, g = lane >> 4;
  const int C = p.C, C2 = C * C;
  const float4* tabR = reinterpret_cast<const float4*>(arena);
  const bool rd = (p.phases & 1) != 0, mm = (p.phases & 2) != 0;
  auto opaque = [](int v) {
    asm volatile("" : "+v"(v));
    return v;
  };
  if (sampler) {
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(p.x) + (size_t)(b0 % p.x_period) * C2, 0, nb * C2 * 4, 0x00020000);
    const int kk = lane & 31;
    const int mw = (wv - NW / 2) * (2 * M / NW) + (lane >> 5);
    // Per-lane LDS bases made opaque to the compiler, so that image u of the
    // lane (mw + 2u) is a small immediate offset from them instead of one
    // materialized address register per u (the arena is larger than the 64 KiB
    // reach of a DS instruction's offset field).
    const int tabo = mw * TABR * 16;                       // the lane's first table
    const int kbo = Ly::TAB + (mw * SK + kk) * 2;          // its first sample in slab 0
    float I[LA][NU][4];
    auto gather = [&](int ks, float (&I)[NU][4]) {
      const int k = 32 * ks + kk;
      const int i = min(k / 28, 27), j = k - (k / 28) * 28;
      const float4* tc = reinterpret_cast<const float4*>(arena + opaque(tabo + j * 16));
      const float4* tr = reinterpret_cast<const float4*>(arena + opaque(tabo + (28 + i) * 16));
      int xo = mw * C2 * 4;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int m = mw + 2 * u;
        float4 ex, ey;
        if constexpr (SEP) {
          ex = tc[2 * u * TABR];
          ey = tr[2 * u * TABR];
        } else {
          glimpse_geom<false>(tabR, sth[m], m, k, C, ex, ey);
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
      const float4* tc = reinterpret_cast<const float4*>(arena + opaque(tabo + j * 16));
      const float4* tr = reinterpret_cast<const float4*>(arena + opaque(tabo + (28 + i) * 16));
      const int grp = ks / KG;
      __bf16* kd = reinterpret_cast<__bf16*>(
          arena + opaque(kbo + (grp % 3) * Ly::KB + (ks - grp * KG) * 64));
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int m = mw + 2 * u;
        float4 ex, ey;
        if constexpr (SEP) {
          ex = tc[2 * u * TABR];
          ey = tr[2 * u * TABR];
        } else {
          glimpse_geom<false>(tabR, sth[m], m, k, C, ex, ey);
        }
        // corners from the two pairs (rows y0: I[u][0..1], y1: I[u][2..3])
        const int fl = __float_as_int(ex.y);
        const float Ia = (fl & 1) ? I[u][1] : I[u][0], Ib = (fl & 1) ? I[u][3] : I[u][2];
        const float Ic = (fl & 2) ? I[u][1] : I[u][0], Id = (fl & 2) ? I[u][3] : I[u][2];
        // dead: corners coincide on both axes (flags agree, rows equal).
        // Evaluated with bitwise ops: short-circuit forms made the compiler
        // branch around a separate LDS load of the row entry.
        const int xlive = (fl ^ (fl >> 1)) & 1;
        const int ylive = __float_as_int(ey.x) != __float_as_int(ey.y) ? 1 : 0;
        const int live = (int)rd & (int)(k < W2) & (int)(m < nb) & (xlive | ylive);
        const float v = sample4(ex, ey, Ia, Ib, Ic, Id);
        kd[2 * u * SK] = (__bf16)(live ? v : 0.0f);
      }
    };
    // glimpse slab grp -> gb[:, 160grp ..] (16-byte pieces inside the 784 columns)
    auto flush = [&](int grp) {
      if (!(p.phases & 16)) return;
      const __bf16* kb = reinterpret_cast<const __bf16*>(arena + Ly::TAB + (grp % 3) * Ly::KB);
      constexpr int CPR = KG * 4;  // 16-byte pieces per slab row
      for (int i = tid - NTHR / 2; i < M * CPR; i += NTHR / 2) {
        const int m = i / CPR, c = i - (i / CPR) * CPR, k = 32 * KG * grp + 8 * c;
        if (m < nb && k < W2)
          st_stream(reinterpret_cast<u32x4*>(p.gb + (size_t)(b0 + m) * W2 + k),
                    *reinterpret_cast<const u32x4*>(kb + m * SK + 8 * c));
      }
    };
    // k-step ks uses gather register set ks % LA; the sample loop is unrolled
    // by LA so the set index is a compile-time constant
#pragma unroll
    for (int k = 0; k < LA; ++k)
      if (rd) gather(k, I[k]);
    static_for<0, KS1>([&](auto kc) {
      constexpr int ks = decltype(kc)::value;
      sample(ks, I[ks % LA]);
      if constexpr (ks + LA < KS1)
        if (rd) gather(ks + LA, I[ks % LA]);
      if constexpr (ks % KG == KG - 1) {  // slab complete
        if constexpr (ks >= 2 * KG - 1) flush(ks / KG - 1);
        lds_barrier();
      }
    });
    flush(NG - 1);
    lds_barrier();
  } else {
    // MFMA waves: column tiles (wv + (NW/2) c + rot) % 32, c < TW
    const int rot = (int)(blockIdx.x >> 3);
    const __amdgpu_buffer_rsrc_t wr = weight_rsrc(p.wt[0]);
    int wo[TW];
#pragma unroll
    for (int c = 0; c < TW; ++c) {
      ct[c] = (wv + (NW / 2) * c + rot) % 32;
      wo[c] = frag_voff(ct[c], lane);
    }
    bf16x8 q[DB][TW];
    auto loadB = [&](int ks, bf16x8* b) {
#pragma unroll
      for (int c = 0; c < TW; ++c) b[c] = load_frag<32>(wr, wo[c], ks);
    };
    const int kao = Ly::TAB + (li * SK + 8 * g) * 2;
    auto mfma = [&](int ks, const bf16x8* b) {
      if (!mm) return;
      const int grp = ks / KG;
      const __bf16* ka = reinterpret_cast<const __bf16*>(
          arena + opaque(kao + (grp % 3) * Ly::KB + (ks - grp * KG) * 64));
#pragma unroll
      for (int rt = 0; rt < MT; ++rt) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&ka[rt * 16 * SK]);
#pragma unroll
        for (int c = 0; c < TW; ++c)
          acc[rt][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[c], acc[rt][c], 0, 0, 0);
      }
    };
#pragma unroll
    for (int rt = 0; rt < MT; ++rt)
#pragma unroll
      for (int c = 0; c < TW; ++c) acc[rt][c] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < DB; ++d) loadB(d, q[d]);
    lds_barrier();  // slab 0 filled
    static_for<0, KS1>([&](auto kc) {
      constexpr int ks = decltype(kc)::value;
      mfma(ks, q[ks % DB]);
      if constexpr (ks + DB < KS1) loadB(ks + DB, q[ks % DB]);
      if constexpr (ks % KG == KG - 1) lds_barrier();  // slab consumed / next slab filled
    });
#pragma unroll
    for (int c = 0; c < TW; ++c) b1q[c] = load_bias4(p.bias[0], ct[c] * 16 + (li & ~3), 512);
  }
}

// ---- STN write (air_model.py:580-588): this step's canvas part -----------
// part = active ? z * w : 0 (mog_recon_loss sums the parts in step order).
// r is staged back one image per wave into the wave's LDS slot; the lanes
// walk the image's pixel pairs and store 8 bytes each.  Only rows whose
// clipped corner rows differ can be nonzero; the even-aligned range of them
// is stored and recorded.  Shared by the bf16 and fp32 step kernels.
template <int NW>
__device__ __forceinline__ void stn_write_tile(const float* __restrict__ r, float* part,
                                               int* part_rows, int C, unsigned char* arena,
                                               int wslot, const float (*sth)[12],
                                               const int* smask, const int* ssep,
                                               const float* szv, int b0, int nb, int wv,
                                               int lane) {
#pragma clang fp contract(off)
  const int C2 = C * C;
  // Wave-private: wave wv writes images wv, wv + NW, ... from its own LDS
  // slot (r of one image); the next image's r is
  // fetched into registers while the current one is computed, and the
  // waves meet no workgroup barrier, so their memory and VALU phases drift
  // apart and overlap.
  const bool vec = (C2 & 3) == 0;  // even C: 16-byte aligned image rows of parts
  unsigned char* slot = arena + wv * wslot;
  float* sRw = reinterpret_cast<float*>(slot);
  constexpr int NQ = (W2 / 4 + 63) / 64;
  // (native vectors, unconditional loads at clamped indices: with HIP's
  // float4 and a predicated load the array went to scratch and every fetch
  // waited for its loads on the spot)
  floatx4 tmp[NQ];
  auto fetch = [&](int m) {
    const floatx4* src = reinterpret_cast<const floatx4*>(r + (size_t)(b0 + m) * W2);
#pragma unroll
    for (int it = 0; it < NQ; ++it) tmp[it] = src[min(lane + it * 64, W2 / 4 - 1)];
  };
  if (wv < nb) fetch(wv);
  for (int m = wv; m < nb; m += NW) {
#pragma unroll
    for (int it = 0; it < NQ; ++it) {
      const int i = lane + it * 64;
      if (i < W2 / 4) reinterpret_cast<floatx4*>(sRw)[i] = tmp[it];
    }
    wave_lds_sync();
    if (m + NW < nb) fetch(m + NW);
    float* om = part + (size_t)(b0 + m) * C2;
    float4* om4 = reinterpret_cast<float4*>(om);
    const float* U = sRw;
    const bool act = smask[m] != 0, tab = (ssep[m] & 2) != 0;
    const float zn = szv[m];
    if (!act) {  // inactive: the whole part is +0 -- nothing stored
      if (lane == 0) part_rows[b0 + m] = 0;
    } else if (tab && vec && C <= CTAB_MAX) {
      // Only rows whose clipped corner rows differ can be nonzero (a row
      // with coinciding corner rows samples exactly +0 at every column:
      // the y weights are exact negatives on one source row, and within
      // a live row no sample is dead): store the even-aligned range
      // [rlo, rhi) of such rows and record it.  Lane i holds row entry i
      // in registers; a pass reads rows r, r + 1 with readlane.
      const float4 el = axis4(axis_row(&sth[m][6], 28, 28, C, C, lane < C ? lane : 0), 4 * 28);
      const unsigned long long lm =
          __builtin_amdgcn_ballot_w64(lane < C && __float_as_int(el.x) != __float_as_int(el.y));
      const int rlo = lm ? (__builtin_ctzll(lm) & ~1) : 0;
      const int rhi = lm ? min(C, (64 - __builtin_clzll(lm) + 1) & ~1) : 0;
      if (lane == 0) part_rows[b0 + m] = rlo | (rhi << 16);
      // Lane -> pixel pair pr of row r + half (PR pairs per row, two rows
      // per pass; C = 50 leaves 14 lanes idle): the column geometry stays
      // in registers, and a corner pair (x0, x0 + 1) of a source row is
      // one ds_read2 -- a live column has x1 = x0 + 1, a dead one x1 = x0
      // (its second corner is the first).  Same products and summation
      // order as sample4, per pixel.
      const int PR = C >> 1, half = lane >= PR ? 1 : 0, pr = lane - half * PR;
      const bool on = lane < 2 * PR;
      const float4 e0 = axis4(axis_col(&sth[m][6], 28, 28, C, C, on ? 2 * pr : 0), 4);
      const float4 e1 = axis4(axis_col(&sth[m][6], 28, 28, C, C, on ? 2 * pr + 1 : 0), 4);
      const int a0 = __float_as_int(e0.x), a1 = __float_as_int(e1.x);
      const bool dd0 = a0 == __float_as_int(e0.y), dd1 = a1 == __float_as_int(e1.y);
      typedef float f2 __attribute__((ext_vector_type(2)));
      const f2 xz = {e0.z, e1.z}, xw = {e0.w, e1.w};
      const char* Ub = reinterpret_cast<const char*>(sRw);
      auto ld = [Ub](int a, int b) { return *reinterpret_cast<const float*>(Ub + a + b); };
      f2* dst = reinterpret_cast<f2*>(om + (rlo + half) * C) + pr;
      const int eyx = __float_as_int(el.x), eyy = __float_as_int(el.y);
      const int eyz = __float_as_int(el.z), eyw = __float_as_int(el.w);
      for (int r = rlo; r < rhi; r += 2) {
        // (readlane takes a uniform lane: both rows' entries, then select)
        const int y0a = __builtin_amdgcn_readlane(eyx, r), y0b = __builtin_amdgcn_readlane(eyx, r + 1);
        const int y1a = __builtin_amdgcn_readlane(eyy, r), y1b = __builtin_amdgcn_readlane(eyy, r + 1);
        const int za = __builtin_amdgcn_readlane(eyz, r), zb = __builtin_amdgcn_readlane(eyz, r + 1);
        const int wa_ = __builtin_amdgcn_readlane(eyw, r), wb_ = __builtin_amdgcn_readlane(eyw, r + 1);
        const int y0 = half ? y0b : y0a, y1 = half ? y1b : y1a;
        const float ez = __int_as_float(half ? zb : za), ew = __int_as_float(half ? wb_ : wa_);
        if (on) {
          const f2 Ia = {ld(y0, a0), ld(y0, a1)}, Ib = {ld(y1, a0), ld(y1, a1)};
          const f2 In = {ld(y0, a0 + 4), ld(y0, a1 + 4)}, Jn = {ld(y1, a0 + 4), ld(y1, a1 + 4)};
          const f2 Ic = {dd0 ? Ia.x : In.x, dd1 ? Ia.y : In.y};
          const f2 Id = {dd0 ? Ib.x : Jn.x, dd1 ? Ib.y : Jn.y};
          const f2 wa = xz * ez, wb = xz * ew, wc = xw * ez, wd = xw * ew;
          const f2 sv = ((wa * Ia + wb * Ib) + wc * Ic) + wd * Id;
          st_stream(dst, zn * sv);
        }
        dst += C;  // two rows of C / 2 pairs
      }
    } else {  // general transform or odd C: per-pixel geometry, flat order
      if (lane == 0) part_rows[b0 + m] = C << 16;
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
        if (vec) st_stream(reinterpret_cast<floatx4*>(om4 + q), floatx4{v[0], v[1], v[2], v[3]});
        else st_stream(om + q, v[0]);
      }
    }
    wave_lds_sync();  // the slot is rewritten for the next image
  }
}

}  // namespace
