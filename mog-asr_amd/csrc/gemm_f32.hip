// Generic fp32 GEMM on the gfx950 fp32-input MFMA (v_mfma_f32_16x16x4_f32).
//
// C[m][n] = epilogue( chain_k A(m,k) B(k,n) ), optionally batched over up to
// MAXB independent problems (pointer arrays) and split over K.
//
// Bit-exactness contract: with splitk == 1 each output
// element is ONE fp32 fma chain over k in natural order, starting from 0 (or
// from Cin), exactly like the oracle's dense() loop — the 16x16x4 f32 MFMA is
// a k-ordered fma chain on gfx950 and the k loop below walks k upward.  The
// bias is added with a separate rounding (TF matmul + bias_add,
// contrib/layers fully_connected as used at vae.py:18-41, air_model.py:462-499).
//
// Tiles: 64x64 or 128x128 per 256-thread workgroup (2x2 waves, each wave
// (BM/2)x(BN/2) of 16x16 MFMA tiles), BK = 16, operands through raw buffer
// descriptors, register-staged double buffering (next tile's global loads in
// flight during the MFMAs), k-permuted LDS rows read as one ds_read_b128 per
// fragment per k-tile.
//
// Weight-gradient form: transA + EPI_ATOMIC + split-K computes dW += X^T dY;
// when `colsum` is given the workgroups of the first M-tile row also add the
// column sums of their dY tiles into colsum[n] (the bias gradient, TF
// BiasAddGrad), so no separate reduction pass re-reads dY.
//
// Replaces the TF-1.12 MatMul / BiasAdd / Softplus / Relu / Sigmoid op groups
// of the hot path (SURVEY.md §2 table "TF op group on the hot path").
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "mog_common.h"
#include "philox.h"

namespace {

enum {
  EPI_STORE = 0,          // C = acc (+ bias)
  EPI_RELU = 1,           // C = relu(acc + bias), Cpre = acc + bias
  EPI_SOFTPLUS = 2,       // C = softplus_tf(acc + bias), Cpre = acc + bias
  EPI_SIGMOID_NOISE = 3,  // C = sigmoid((acc + bias) + aux*scale), Cpre = acc + bias
  EPI_SOFTPLUS_BWD = 4,   // C = acc * (1 - exp(-aux))     (dX through softplus; aux = its
                          //  output: sigmoid(x) = 1 - exp(-softplus(x)))
  EPI_ATOMIC = 5,         // C += acc  (atomic; split-K / batch reduction)
  EPI_RELU_BWD = 6,       // C = aux > 0 ? acc : 0          (dX through relu)
};

constexpr int MAXB = 8;
struct GemmPtrs {
  const float* A[MAXB];
  const float* B[MAXB];
  float* C[MAXB];
  const float* bias[MAXB];
  const float* Cin[MAXB];
  float* Cpre[MAXB];
  const float* aux[MAXB];
  float* colsum[MAXB];
};
struct GemmDims {
  int M, N, K, lda, ldb, ldc, ldaux, splitk, kchunk, vecA, vecB, nx, ny;
  int kseg;  // > 0: K is nseg segments of kseg, segment s read from A[s] / B[s]
  // (kseg) problem z of the batch owns segments segoff[z] .. segoff[z+1]-1
  // (its K = that count * kseg; D.K is the largest problem's)
  int segoff[5];
  int vecC;  // C / Cpre / aux 16-byte aligned with ldc, ldaux % 4 == 0 (row-staged epilogue)
  float aux_scale;
  // EPI_SIGMOID_NOISE with in-kernel noise (eps_gen): the noise of element
  // (row, col) is lane col % 4 of Philox quad eps_off + row * N / 4 + col / 4,
  // bit-identical to mog_rng_fill(seed, eps_off) of a [M][N] buffer
  int eps_gen;
  unsigned long long eps_seed, eps_off;
};

// noise quad of output row `row`, columns col .. col + 3 (col % 4 == 0)
__device__ __forceinline__ void noise_quad(const GemmDims& D, int row, int col, float v[4]) {
  mog_philox_quad(D.eps_seed, D.eps_off + (unsigned long long)row * (D.N / 4) + col / 4, true, v);
}

// LDS image of a BK-deep slice of an operand: one row of Lay<BK>::S floats
// per m (A) or n (B).  The BK k values of a row are stored PERMUTED: k =
// 4 kk + g lives in 4-float chunk ci = g (BK/16) + kk / 4 (XOR-swizzled by the
// row), position kk % 4, so lane (row, g) of a 16x16x4 MFMA fragment reads four
// consecutive k-steps with ONE ds_read_b128.  Strides / swizzles were searched
// to be conflict-free for those reads and for the tile writes under the gfx950
// LDS lane grouping (MI355X_MICROARCH.md §LDS): BK = 16 -> S = 24, no
// swizzle; BK = 32 -> S = 48, chunk ^= row & 7.
template <int BK>
struct Lay;
template <>
struct Lay<16> {
  static constexpr int S = 24;
  __device__ static __forceinline__ int sw(int) { return 0; }
};
template <>
struct Lay<32> {
  static constexpr int S = 48;
  __device__ static __forceinline__ int sw(int row) { return row & 7; }
};
template <int BK>
__device__ __forceinline__ int lpos(int row, int g, int kk) {  // float index of (row, k = 4 kk + g)
  return row * Lay<BK>::S + 4 * ((g * (BK / 16) + (kk >> 2)) ^ Lay<BK>::sw(row)) + (kk & 3);
}

// bijective XCD-grouping remap of the linear workgroup id (guide §5, T1):
// consecutive ids (same A row-panel, neighbouring N tiles) share one XCD's L2
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t frsrc(const float* p, long elems) {
  // raw buffer over [p, p + elems): loads past the end return 0 (no fault)
  const long bytes = elems * 4;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0,
                                           (int)(bytes < 0x7ffffff0L ? bytes : 0x7ffffff0L),
                                           0x00020000);
}

// One operand tile (ROWS x BK) moving global -> registers -> LDS, through a
// raw buffer descriptor (32-bit offsets; rows past the operand's extent read
// 0).  Interior k-tiles (`full`) load without per-element checks; only the
// ragged last k-tile of a split masks k >= kend.
//   KC (k-contiguous in memory: A [M][K], B^T [N][K]): float4 loads along k,
//     four ds_write_b32 into the permuted row.
//   otherwise (row-contiguous: A^T [K][M], B [K][N]): per (row, g) BK/4 dword
//     loads at k = g, 4+g, 8+g, ... (coalesced over rows across lanes), one
//     ds_write_b128 per four of them.
// Elements masked off (k >= kend of a split-K chunk, still inside the
// operand) are read at an offset past every descriptor's extent, so the
// hardware returns 0: the mask is applied to the address, never to the loaded
// value, and nothing waits for a load before its k-tile is written to LDS.
constexpr int OOB = 0x7ffffff0;

template <int ROWS, bool KC, int BK>
struct TileIO {
  static constexpr int KK = BK / 4;
  static constexpr int NV = ROWS * BK / 1024;  // KC: float4 per thread
  static constexpr int NP = ROWS * 4 / 256;    // row-contiguous: (row, g) pairs per thread
  static constexpr int NR = KC ? NV * 4 : NP * KK;
  float r[NR];
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, int ld, int r0, int k0,
                                       int kend, bool vec, bool full, int t) {
    if constexpr (KC) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int q = t + 256 * i;
        const int row = q / KK, c = q % KK;  // KK float4 chunks per BK-deep row
        const int gk = k0 + 4 * c;
        const int off = ((r0 + row) * ld + gk) * 4;
        if (full && vec) {
          const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
#pragma unroll
          for (int j = 0; j < 4; ++j) r[4 * i + j] = __uint_as_float(v[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            r[4 * i + j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                rs, (full || gk + j < kend) ? off + 4 * j : OOB, 0, 0));
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int q = t + 256 * i;
        const int row = q % ROWS, g = q / ROWS;  // lanes run along the contiguous rows
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          const int gk = k0 + 4 * kk + g;
          r[KK * i + kk] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
              rs, (full || gk < kend) ? (gk * ld + r0 + row) * 4 : OOB, 0, 0));
        }
      }
    }
  }
  __device__ __forceinline__ void store(float* S, int t) const {
    if constexpr (KC) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int q = t + 256 * i;
        const int row = q / KK, c = q % KK;  // chunk c holds kk = c for g = 0..3
#pragma unroll
        for (int g = 0; g < 4; ++g) S[lpos<BK>(row, g, c)] = r[4 * i + g];
      }
    } else {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int q = t + 256 * i;
        const int row = q % ROWS, g = q / ROWS;
#pragma unroll
        for (int h = 0; h < KK / 4; ++h)
          *reinterpret_cast<floatx4*>(&S[lpos<BK>(row, g, 4 * h)]) =
              floatx4{r[KK * i + 4 * h], r[KK * i + 4 * h + 1], r[KK * i + 4 * h + 2],
                      r[KK * i + 4 * h + 3]};
      }
    }
  }
};

// Epilogue of one wave's (16 MI) x (16 NI) accumulator block at output rows
// r0 + ..., columns c0 + ... (16x16 MFMA layout: lane (li, g) holds rows
// 4g .. 4g+3 of column li of each tile).
// RA / RB: the LDS-DMA kernel's remapped fragments (row-contiguous operands
// read as one vector per k-step, gemm_f32_dma_kernel): accumulator row i of
// tile mi is output row MI i + mi, column j of tile ni is column NI j + ni.
template <int MI, int NI, bool RA, bool RB>
__device__ __forceinline__ int acc_row(int mi, int i) {
  return RA ? MI * i + mi : mi * 16 + i;
}
template <int MI, int NI, bool RA, bool RB>
__device__ __forceinline__ int acc_col(int ni, int j) {
  return RB ? NI * j + ni : ni * 16 + j;
}

template <int MI, int NI, int EPI, bool RA = false, bool RB = false>
__device__ __forceinline__ void store_tile(const floatx4 (&acc)[MI][NI], const GemmPtrs& P,
                                           const GemmDims& D, int z, int r0, int c0, int lane) {
#pragma clang fp contract(off)
  const int M = D.M, N = D.N;
  float* C = P.C[z];
  const float* bias = P.bias[z];
  const float* aux = P.aux[z];
  float* Cpre = P.Cpre[z];
  constexpr bool HAS_AUX = EPI == EPI_SOFTPLUS_BWD || EPI == EPI_RELU_BWD || EPI == EPI_SIGMOID_NOISE;
  // every bias / aux operand of the lane loaded up front from clamped indices
  // (a load under the per-element bounds test below compiles to a branch with
  // a vmcnt(0) wait inside: one memory latency per element)
  float bq[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
    bq[ni] = bias != nullptr ? bias[min(c0 + acc_col<MI, NI, RA, RB>(ni, lane & 15), N - 1)] : 0.0f;
  float xq[MI][NI][4];
  if (HAS_AUX && !(EPI == EPI_SIGMOID_NOISE && D.eps_gen)) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = min(r0 + acc_row<MI, NI, RA, RB>(mi, (lane >> 4) * 4 + r), M - 1);
          const int col = min(c0 + acc_col<MI, NI, RA, RB>(ni, lane & 15), N - 1);
          xq[mi][ni][r] = aux[(size_t)row * D.ldaux + col];
        }
  }
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + acc_row<MI, NI, RA, RB>(mi, (lane >> 4) * 4 + r);
        const int col = c0 + acc_col<MI, NI, RA, RB>(ni, lane & 15);
        if (row >= M || col >= N) continue;
        const size_t o = (size_t)row * D.ldc + col;
        float v = acc[mi][ni][r];
        if (EPI == EPI_ATOMIC) {
          atomicAdd(C + o, v);
          continue;
        }
        if (EPI == EPI_SOFTPLUS_BWD) {
          C[o] = v * -mog_expm1f(-xq[mi][ni][r]);
          continue;
        }
        if (EPI == EPI_RELU_BWD) {
          C[o] = xq[mi][ni][r] > 0.0f ? v : 0.0f;
          continue;
        }
        if (bias != nullptr) v = v + bq[ni];
        if (EPI == EPI_STORE) {
          C[o] = v;
        } else {
          if (Cpre != nullptr) Cpre[o] = v;
          if (EPI == EPI_RELU) C[o] = v > 0.0f ? v : 0.0f;
          if (EPI == EPI_SOFTPLUS) C[o] = mog_softplusf(v);
          if (EPI == EPI_SIGMOID_NOISE) {
            float nz;
            if (D.eps_gen) {
              float q[4];
              noise_quad(D, row, col & ~3, q);
              nz = q[col & 3];
            } else {
              nz = xq[mi][ni][r];
            }
            C[o] = mog_sigmoidf(v + nz * D.aux_scale);
          }
        }
      }
}

// Epilogue of the whole BM x BN workgroup tile staged through LDS (the k
// loop's stage buffers, free by now): the waves' 16x16 accumulator layout
// (a store instruction writes 64-byte row pieces) is re-read as whole rows,
// so every store / aux load / atomic instruction covers full 256-byte row
// segments.  Elementwise math identical to store_tile.
template <int BM, int BN, int EPI, bool RA = false, bool RB = false>
__device__ __forceinline__ void store_tile_rows(const floatx4 (&acc)[BM / 32][BN / 32],
                                                float* sC, const GemmPtrs& P, const GemmDims& D,
                                                int z, int m0, int n0, int wm, int wn) {
#pragma clang fp contract(off)
  constexpr int MI = BM / 32, NI = BN / 32, LDC = BN + 4;
  const int t = threadIdx.x, lane = t & 63;
  __syncthreads();  // every wave is done with the stage buffers
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sC[(wm + acc_row<MI, NI, RA, RB>(mi, (lane >> 4) * 4 + r)) * LDC + wn +
           acc_col<MI, NI, RA, RB>(ni, lane & 15)] = acc[mi][ni][r];
  __syncthreads();
  const int M = D.M, N = D.N;
  float* C = P.C[z];
  if constexpr (EPI == EPI_ATOMIC) {
    // one element per lane: a wave-instruction adds 64 consecutive columns
    for (int q = t; q < BM * BN; q += 256) {
      const int row = q / BN, col = q - row * BN;
      if (m0 + row < M && n0 + col < N)
        atomicAdd(C + (size_t)(m0 + row) * D.ldc + n0 + col, sC[row * LDC + col]);
    }
  } else {
    const float* bias = P.bias[z];
    const float* aux = P.aux[z];
    float* Cpre = P.Cpre[z];
    constexpr int C4 = BN / 4, RSTEP = 256 / C4, ITER = BM / RSTEP;
    static_assert(256 % C4 == 0 && BM % RSTEP == 0, "epilogue row mapping");
    constexpr bool HAS_PRE = EPI == EPI_RELU || EPI == EPI_SOFTPLUS || EPI == EPI_SIGMOID_NOISE;
    constexpr bool HAS_AUX = EPI == EPI_SOFTPLUS_BWD || EPI == EPI_RELU_BWD ||
                             EPI == EPI_SIGMOID_NOISE;
    // the thread's column quad is the same in every row it visits: its bias
    // quad is loaded once, and every aux quad up front, from clamped
    // (in-bounds) indices, unconditionally -- a load under the bounds test
    // compiles to a branch with a vmcnt(0) wait inside
    const int c4 = t % C4, r00 = t / C4, gcol = n0 + 4 * c4;
    float bq[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias != nullptr) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bq[e] = bias[min(gcol + e, N - 1)];
    }
    float xq[ITER][4];
    const bool aux_ld = HAS_AUX && !(EPI == EPI_SIGMOID_NOISE && D.eps_gen);
    if (aux_ld) {
      // a quad is read whole only where N and ldaux are multiples of 4 (a
      // uniform test): the quad then never passes column N - 1 of the row
      const int ac = gcol < N ? gcol : 0;
#pragma unroll
      for (int i = 0; i < ITER; ++i) {
        const float* ar = aux + (size_t)min(m0 + r00 + RSTEP * i, M - 1) * D.ldaux;
        if (D.ldaux % 4 == 0 && N % 4 == 0) {
          const float4 x4 = *reinterpret_cast<const float4*>(ar + ac);
          xq[i][0] = x4.x; xq[i][1] = x4.y; xq[i][2] = x4.z; xq[i][3] = x4.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) xq[i][e] = ar[min(ac + e, N - 1)];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int row = r00 + RSTEP * i;
      const int grow = m0 + row;
      if (grow >= M || gcol >= N) continue;
      const bool full = gcol + 4 <= N;
      const float4 a4 = *reinterpret_cast<const float4*>(&sC[row * LDC + 4 * c4]);
      const float v[4] = {a4.x, a4.y, a4.z, a4.w};
      float x[4] = {0.f, 0.f, 0.f, 0.f};
      if (EPI == EPI_SIGMOID_NOISE && D.eps_gen) {
        noise_quad(D, grow, gcol, x);  // N % 4 == 0: the quad lies inside the row
      } else if constexpr (HAS_AUX) {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = xq[i][e];
      }
      float o[4], pre[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float w = v[e];
        pre[e] = w;
        if (EPI == EPI_SOFTPLUS_BWD) {
          o[e] = w * -mog_expm1f(-x[e]);
        } else if (EPI == EPI_RELU_BWD) {
          o[e] = x[e] > 0.0f ? w : 0.0f;
        } else {
          if (bias != nullptr) w = w + bq[e];
          pre[e] = w;
          if (EPI == EPI_STORE) o[e] = w;
          if (EPI == EPI_RELU) o[e] = w > 0.0f ? w : 0.0f;
          if (EPI == EPI_SOFTPLUS) o[e] = mog_softplusf(w);
          if (EPI == EPI_SIGMOID_NOISE) o[e] = mog_sigmoidf(w + x[e] * D.aux_scale);
        }
      }
      float* cr = C + (size_t)grow * D.ldc + gcol;
      float* pr = (HAS_PRE && Cpre) ? Cpre + (size_t)grow * D.ldc + gcol : nullptr;
      // the pre-activation is read only by the backward, long after: stored
      // non-temporal so it does not displace the next layer's operands
      if (full) {
        *reinterpret_cast<float4*>(cr) = make_float4(o[0], o[1], o[2], o[3]);
        if (pr)
          __builtin_nontemporal_store(floatx4{pre[0], pre[1], pre[2], pre[3]},
                                      reinterpret_cast<floatx4*>(pr));
      } else {
        for (int e = 0; e < 4; ++e)
          if (gcol + e < N) {
            cr[e] = o[e];
            if (pr) __builtin_nontemporal_store(pre[e], pr + e);
          }
      }
    }
  }
}

template <int BM, int BN, int BK, int PF, bool TA, bool TB, int EPI, bool KSEG>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmPtrs P, GemmDims D) {
#pragma clang fp contract(off)
  constexpr int MI = BM / 32, NI = BN / 32;     // 16x16 tiles per wave (2x2 waves)
  constexpr int KK = BK / 4;                    // MFMA k-steps per tile
  constexpr int A_SZ = BM * Lay<BK>::S, STAGE = (BM + BN) * Lay<BK>::S;
  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];
  const int nwg = gridDim.x * gridDim.y * gridDim.z;
  const int wg = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), nwg);
  const int bx = wg % D.nx, by = (wg / D.nx) % D.ny, bz = wg / (D.nx * D.ny);
  const int z = bz / D.splitk, ks = bz - z * D.splitk;
  const int m0 = by * BM, n0 = bx * BN;
  const int kbeg = ks * D.kchunk;
  const int sb = KSEG ? D.segoff[z] : 0;  // (kseg) problem z's first segment
  const int kend = min(KSEG ? (D.segoff[z + 1] - sb) * D.kseg : D.K, kbeg + D.kchunk);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);
  const int M = D.M, N = D.N;
  float* colsum = P.colsum[z];
  const bool do_cs = colsum != nullptr && by == 0 && t < BN;
  float cs = 0.0f;

  floatx4 acc[MI][NI];
  const float* Cin = P.Cin[z];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // clamped, unconditional loads (a per-element `if` around a load
        // compiles to a branch with a vmcnt(0) wait inside: one memory
        // latency per element); the out-of-range elements are never stored
        float v = 0.0f;
        if (Cin != nullptr && ks == 0) {
          const int row = min(m0 + wm + mi * 16 + (lane >> 4) * 4 + r, M - 1);
          const int col = min(n0 + wn + ni * 16 + (lane & 15), N - 1);
          v = Cin[(size_t)row * D.ldc + col];
        }
        acc[mi][ni][r] = v;
      }

  // operand extents (elements) behind the buffer descriptors: A rows < M
  // (TA: k rows < K of lda), B likewise; per K-segment when KSEG
  const int ka = KSEG ? D.kseg : D.K;
  const long extA = TA ? (long)(ka - 1) * D.lda + M : (long)(M - 1) * D.lda + ka;
  const long extB = TB ? (long)(N - 1) * D.ldb + ka : (long)(ka - 1) * D.ldb + N;
  __amdgpu_buffer_rsrc_t ra = frsrc(P.A[KSEG ? sb : z], extA);
  __amdgpu_buffer_rsrc_t rb = frsrc(P.B[KSEG ? sb : z], extB);
  int seg = 0;

  // PF register sets of staged tiles: tile j+1 is loaded PF iterations
  // before it is written to LDS (PF = 2 hides an HBM miss behind two k-tiles)
  TileIO<BM, !TA, BK> ta[PF];
  TileIO<BN, TB, BK> tb[PF];
  auto load_tiles = [&](int k0, TileIO<BM, !TA, BK>& A_, TileIO<BN, TB, BK>& B_) {
    int kl = k0, kl_end = kend;
    if (KSEG) {  // a BK tile never straddles two segments (kseg % BK == 0)
      const int sg = k0 / D.kseg;
      if (sg != seg) {
        seg = sg;
        ra = frsrc(P.A[sb + sg], extA);
        rb = frsrc(P.B[sb + sg], extB);
      }
      kl = k0 - sg * D.kseg;
      kl_end = kend - sg * D.kseg;
    }
    const bool full = k0 + BK <= kend;
    A_.load(ra, D.lda, m0, kl, kl_end, D.vecA, full, t);
    B_.load(rb, D.ldb, n0, kl, kl_end, D.vecB, full, t);
  };
  auto store_tiles = [&](int stage, const TileIO<BM, !TA, BK>& A_,
                         const TileIO<BN, TB, BK>& B_) {
    float* As = lds + stage * STAGE;
    A_.store(As, t);
    B_.store(As + A_SZ, t);
  };
  const int fr = lane & 15, fg = lane >> 4;
  floatx4 fa[MI][KK / 4], fb[NI][KK / 4];
  auto read_frags = [&](int stage) {
    const float* As = lds + stage * STAGE;
    const float* Bs = As + A_SZ;
#pragma unroll
    for (int h = 0; h < KK / 4; ++h) {
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
        fa[mi][h] = *reinterpret_cast<const floatx4*>(&As[lpos<BK>(wm + mi * 16 + fr, fg, 4 * h)]);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        fb[ni][h] = *reinterpret_cast<const floatx4*>(&Bs[lpos<BK>(wn + ni * 16 + fr, fg, 4 * h)]);
    }
    if (do_cs) {
#pragma unroll
      for (int k = 0; k < BK; ++k) cs += Bs[t * Lay<BK>::S + k];
    }
  };
  auto mfmas = [&]() {
    // k = 4 kk + g: MFMA kk consumes k-slots 4kk..4kk+3 in order -> one
    // k-ordered fma chain per output element
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(
              fa[mi][kk >> 2][kk & 3], fb[ni][kk >> 2][kk & 3], acc[mi][ni], 0, 0, 0);
  };

  // two LDS stages, PF register sets, one barrier per k-tile: after the
  // barrier of iteration it the wave reads tile it's fragments (stage it&1),
  // writes the register set holding tile it+1 (set it % PF) to the other
  // stage (last read in iteration it-1, before this barrier), re-issues tile
  // it+1+PF's loads into that set and then runs its MFMAs.  The k order of
  // every fma chain is unchanged.
  const int nk = kbeg < kend ? (kend - kbeg + BK - 1) / BK : 0;
  auto body = [&](int it, auto sc) {
    constexpr int S = decltype(sc)::value;
    __syncthreads();
    read_frags(it & 1);
    if (it + 1 < nk) {
      store_tiles((it + 1) & 1, ta[S], tb[S]);
      if (it + 1 + PF < nk) load_tiles(kbeg + (it + 1 + PF) * BK, ta[S], tb[S]);
    }
    mfmas();
  };
  if (nk > 0) {
    load_tiles(kbeg, ta[0], tb[0]);
    store_tiles(0, ta[0], tb[0]);
#pragma unroll
    for (int j = 1; j <= PF; ++j)
      if (j < nk) load_tiles(kbeg + j * BK, ta[j - 1], tb[j - 1]);
    for (int it = 0; it < nk; it += PF) {
      body(it, std::integral_constant<int, 0>{});
      if constexpr (PF > 1)
        if (it + 1 < nk) body(it + 1, std::integral_constant<int, 1>{});
    }
  }
  if (do_cs && n0 + t < N) atomicAdd(colsum + n0 + t, cs);

  store_tile<MI, NI, EPI>(acc, P, D, z, m0 + wm, n0 + wn, lane);
}

// ---------------------------------------------------------------------------
// LDS-DMA form: operand k-tiles go global -> LDS by buffer_load_dwordx4 ... lds
// (no register staging, no LDS store instructions), NS stages deep, with the
// DMA of tile it+NS-1 issued right after the barrier of iteration it and a
// counted vmcnt keeping NS-2 tiles in flight across every barrier.  A DMA
// wave-instruction writes 64 x 16 B lane-linearly, so the LDS images are laid
// out by choosing each lane's SOURCE address (MI355X guide §5 rule 21):
//   KC image (operand k-contiguous: A [M][K], B^T [N][K]): ROWS rows of 16 k;
//     16-B chunk c of row r holds k = 4 (c ^ kcs(r)) .. +3 (one instruction
//     fills 16 rows, 64 B of each);
//   RC image (operand row-contiguous: A^T [K][M], B [K][N]): 16 k-rows of
//     ROWS floats; element n of k-row k sits at n ^ rcs(k).
// KC fragments: element (row, k = 4 kk + g) is one ds_read_b32 (2-way, the
// minimum for 4-B reads of a 16-float row).  RC fragments are REMAPPED: the
// wave's (16 MI) rows are assigned so that lane (fr, g) owns rows
// w0 + MI fr .. + MI - 1, which sit side by side in the k-row: one ds_read_b64
// (MI = 2) / ds_read_b128 (MI = 4) per k-step instead of MI ds_read_b32 (those
// run at half the LDS rate, gfx950 LDS table of MI355X_MICROARCH.md); the
// epilogue maps accumulator rows back (acc_row / acc_col).  rcs() makes the
// vector reads conflict-free under the b64 (2 x 32 lanes) / b128 (4 x 16
// lanes) lane groups: 64-float rows swap their halves on odd k, 128-float rows
// need no swizzle.  The k order of every MFMA chain is unchanged.
// The MFMA sequence, and so every fma chain, is the register-staged kernel's.
// KC chunk swizzle: BK = 16 -> 4 chunks per row, (r >> 1) & 3; BK = 32 -> 8
// chunks, r & 7 (both the 2-way minimum for 4-B reads)
template <int BK>
__device__ __forceinline__ int kcs(int r) {
  return BK == 16 ? (r >> 1) & 3 : r & 7;
}

template <int ROWS, bool KC, int BK>
struct DmaOperand {
  static constexpr int NQ = ROWS * BK * 4 / 1024;  // 1-KiB DMA instructions per k-tile
  static constexpr int NWQ = NQ / 4;               // per wave
  static constexpr int CPR = BK / 4;               // KC: 16-B chunks per row
  static_assert(NQ % 4 == 0, "four waves share a tile's DMAs");
  static_assert(KC || ROWS == 32 || ROWS == 64 || ROWS == 128, "RC swizzle");
  // RC: float offset XOR of k-row k (32-float rows: the two k-rows a b32 lane
  // group reads land in opposite 16-bank halves)
  __device__ static __forceinline__ int rcs(int k) {
    return ROWS == 64 ? (k & 1) << 5 : ROWS == 32 ? (k & 1) << 4 : 0;
  }
  int voff[NWQ];  // this lane's source byte offset at k0 = 0
  int kof[NWQ];   // its k within the tile (KC: first of its 4; RC: its k-row)
  __device__ __forceinline__ void init(int w, int lane, int r0, int ld) {
#pragma unroll
    for (int j = 0; j < NWQ; ++j) {
      const int q = w + 4 * j;
      if constexpr (KC) {
        const int row = (64 / CPR) * q + lane / CPR;
        const int kc = 4 * ((lane % CPR) ^ kcs<BK>(row));
        voff[j] = ((r0 + row) * ld + kc) * 4;
        kof[j] = kc;
      } else {
        constexpr int PER = ROWS / 4;  // 16-B chunks per k-row
        const int k = q * (256 / ROWS) + lane / PER;
        const int n = (4 * (lane % PER)) ^ rcs(k);
        voff[j] = (k * ld + r0 + n) * 4;
        kof[j] = k;
      }
    }
  }
  // this wave's DMAs of the k-tile at k0 into `img`; k >= kend reads 0
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, float* img, int w, int k0,
                                        int kend, bool full, int ld) const {
#pragma unroll
    for (int j = 0; j < NWQ; ++j) {
      int o = voff[j] + (KC ? k0 * 4 : k0 * ld * 4);
      if (!full && k0 + kof[j] >= kend) o = OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(img + (w + 4 * j) * 256), 16, o, 0, 0, 0);
    }
  }
  // image index of element (row, k = 4 kk + g)
  __device__ static __forceinline__ int at(int row, int kk, int g) {
    if constexpr (KC) return row * BK + 4 * (kk ^ kcs<BK>(row)) + g;
    else return (4 * kk + g) * ROWS + (row ^ rcs(g));
  }
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int BK, int NS, bool TA, bool TB, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_f32_dma_kernel(GemmPtrs P, GemmDims D) {
#pragma clang fp contract(off)
  constexpr int MI = BM / 32, NI = BN / 32, KK = BK / 4;
  constexpr int A_SZ = BM * BK, STAGE = (BM + BN) * BK;  // floats
  using OpA = DmaOperand<BM, !TA, BK>;
  using OpB = DmaOperand<BN, TB, BK>;
  constexpr bool RA = TA, RB = !TB;  // row-contiguous operands: remapped vector fragments
  typedef float fva __attribute__((ext_vector_type(MI)));
  typedef float fvb __attribute__((ext_vector_type(NI)));
  constexpr int DPT = OpA::NWQ + OpB::NWQ;  // DMA instructions per wave per k-tile
  // the stage buffers, reused by the row-staged epilogue
  constexpr int LDS_F = NS * STAGE > BM * (BN + 4) ? NS * STAGE : BM * (BN + 4);
  __shared__ __attribute__((aligned(1024))) float lds[LDS_F];
  const int nwg = gridDim.x * gridDim.y * gridDim.z;
  const int wg = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), nwg);
  const int bx = wg % D.nx, by = (wg / D.nx) % D.ny, bz = wg / (D.nx * D.ny);
  const int z = bz / D.splitk, ks = bz - z * D.splitk;
  const int m0 = by * BM, n0 = bx * BN;
  const int kbeg = ks * D.kchunk;
  const int kend = min(D.K, kbeg + D.kchunk);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);
  const int M = D.M, N = D.N;
  float* colsum = P.colsum[z];
  const bool do_cs = colsum != nullptr && by == 0 && t < BN;
  float cs = 0.0f;

  floatx4 acc[MI][NI];
  const float* Cin = P.Cin[z];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = 0.0f;  // (clamped, unconditional: see gemm_f32_kernel)
        if (Cin != nullptr && ks == 0) {
          const int row = min(m0 + wm + acc_row<MI, NI, RA, RB>(mi, (lane >> 4) * 4 + r), M - 1);
          const int col = min(n0 + wn + acc_col<MI, NI, RA, RB>(ni, lane & 15), N - 1);
          v = Cin[(size_t)row * D.ldc + col];
        }
        acc[mi][ni][r] = v;
      }

  const long extA = TA ? (long)(D.K - 1) * D.lda + M : (long)(M - 1) * D.lda + D.K;
  const long extB = TB ? (long)(N - 1) * D.ldb + D.K : (long)(D.K - 1) * D.ldb + N;
  const __amdgpu_buffer_rsrc_t ra = frsrc(P.A[z], extA);
  const __amdgpu_buffer_rsrc_t rb = frsrc(P.B[z], extB);
  OpA da;
  OpB db;
  da.init(w, lane, m0, D.lda);
  db.init(w, lane, n0, D.ldb);

  const int nk = kbeg < kend ? (kend - kbeg + BK - 1) / BK : 0;
  auto issue = [&](int j, int stage) {
    const int k0 = kbeg + j * BK;
    const bool full = k0 + BK <= kend;
    float* st = lds + stage * STAGE;
    da.issue(ra, st, w, k0, kend, full, D.lda);
    db.issue(rb, st + A_SZ, w, k0, kend, full, D.ldb);
  };
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < nk) issue(j, j);

  const int fr = lane & 15, fg = lane >> 4;
  // fragment registers: FP = 2 sets (tile it+1's fragments are read from LDS
  // while tile it's MFMAs run), FP = 1 set (read after the barrier)
  constexpr int FP = NS >= 4 ? 2 : 1;
  float fa[FP][KK][MI], fb[FP][KK][NI];
  auto read_frags = [&](int stage, auto fs) {
    constexpr int F = decltype(fs)::value;
    const float* As = lds + stage * STAGE;
    const float* Bs = As + A_SZ;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      if constexpr (RA) {
        const fva v = *reinterpret_cast<const fva*>(&As[OpA::at(wm + MI * fr, kk, fg)]);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) fa[F][kk][mi] = v[mi];
      } else {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) fa[F][kk][mi] = As[OpA::at(wm + mi * 16 + fr, kk, fg)];
      }
      if constexpr (RB) {
        const fvb v = *reinterpret_cast<const fvb*>(&Bs[OpB::at(wn + NI * fr, kk, fg)]);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) fb[F][kk][ni] = v[ni];
      } else {
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) fb[F][kk][ni] = Bs[OpB::at(wn + ni * 16 + fr, kk, fg)];
      }
    }
    if constexpr (!TB) {
      if (do_cs) {
#pragma unroll
        for (int k = 0; k < BK; ++k) cs += Bs[k * BN + (t ^ OpB::rcs(k))];
      }
    }
  };
  auto mfmas = [&](auto fs) {
    constexpr int F = decltype(fs)::value;
    // k = 4 kk + g: MFMA kk consumes k-slots 4kk..4kk+3 in order
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[F][kk][mi], fb[F][kk][ni],
                                                             acc[mi][ni], 0, 0, 0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto next = [](int s) { return s == NS - 1 ? 0 : s + 1; };
  if constexpr (FP == 1) {
    int st = 0;  // stage of tile it
    for (int it = 0; it < nk; ++it) {
      // this wave's DMAs of tile it have landed (NS-2 later tiles may stay in
      // flight), then every wave's have, and every wave is done reading the
      // stage the next DMA overwrites (tile it-1's)
      if (it + NS - 2 < nk) wait_vm<DPT * (NS - 2)>();
      else wait_vm<0>();
      asm volatile("s_barrier" ::: "memory");
      if (it + NS - 1 < nk) issue(it + NS - 1, st == 0 ? NS - 1 : st - 1);
      read_frags(st, I0{});
      mfmas(I0{});
      st = next(st);
    }
  } else {
    // iteration it: tile it+1 has landed everywhere (NS-3 later tiles stay in
    // flight); tile it's fragments are in registers (read in iteration
    // it-1); the DMA of tile it+NS-1 overwrites tile it-1's stage, whose
    // fragment reads every wave completed before this barrier
    if (nk > 0) {
      if (NS - 2 < nk) wait_vm<DPT * (NS - 2)>();
      else wait_vm<0>();
      asm volatile("s_barrier" ::: "memory");
      read_frags(0, I0{});
    }
    int st = 0;
    auto body = [&](int it, auto fs) {
      constexpr int F = decltype(fs)::value;
      if (it + 1 < nk) {
        if (it + NS - 2 < nk) wait_vm<DPT * (NS - 3)>();
        else wait_vm<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (it + NS - 1 < nk) issue(it + NS - 1, st == 0 ? NS - 1 : st - 1);
      if (it + 1 < nk) read_frags(next(st), std::integral_constant<int, 1 - F>{});
      mfmas(fs);
      st = next(st);
    };
    for (int it = 0; it < nk; it += 2) {
      body(it, I0{});
      if (it + 1 < nk) body(it + 1, I1{});
    }
  }
  if (do_cs && n0 + t < N) atomicAdd(colsum + n0 + t, cs);

  if (D.vecC) {
    store_tile_rows<BM, BN, EPI, RA, RB>(acc, lds, P, D, z, m0, n0, wm, wn);
    return;
  }
  store_tile<MI, NI, EPI, RA, RB>(acc, P, D, z, m0 + wm, n0 + wn, lane);
}

template <int BM, int BN, int BK, int PF, bool TA, bool TB, bool KS>
void launch_epi(int epi, dim3 g, hipStream_t s, const GemmPtrs& P, const GemmDims& D) {
#define MOG_GEMM_LAUNCH(E) gemm_f32_kernel<BM, BN, BK, PF, TA, TB, E, KS><<<g, 256, 0, s>>>(P, D)
  if constexpr (KS) {  // K-segment form: only the plain and the accumulate epilogues
    if (epi == EPI_ATOMIC) MOG_GEMM_LAUNCH(EPI_ATOMIC);
    else MOG_GEMM_LAUNCH(EPI_STORE);
    return;
  } else {
  switch (epi) {
    case EPI_STORE: MOG_GEMM_LAUNCH(EPI_STORE); break;
    case EPI_RELU: MOG_GEMM_LAUNCH(EPI_RELU); break;
    case EPI_SOFTPLUS: MOG_GEMM_LAUNCH(EPI_SOFTPLUS); break;
    case EPI_SIGMOID_NOISE: MOG_GEMM_LAUNCH(EPI_SIGMOID_NOISE); break;
    case EPI_SOFTPLUS_BWD: MOG_GEMM_LAUNCH(EPI_SOFTPLUS_BWD); break;
    case EPI_ATOMIC: MOG_GEMM_LAUNCH(EPI_ATOMIC); break;
    case EPI_RELU_BWD: MOG_GEMM_LAUNCH(EPI_RELU_BWD); break;
  }
  }
#undef MOG_GEMM_LAUNCH
}

template <int BM, int BN, int BK, int PF>
void launch_tile(bool ta, bool tb, int epi, hipStream_t s, const GemmPtrs& P, GemmDims D,
                 int batch) {
  int kchunk = (D.K + D.splitk - 1) / D.splitk;
  kchunk = ((kchunk + BK - 1) / BK) * BK;
  if (kchunk == 0) kchunk = BK;
  D.kchunk = kchunk;
  D.splitk = (D.K + kchunk - 1) / kchunk;
  if (D.splitk < 1) D.splitk = 1;
  D.nx = mog_cdiv(D.N, BN);
  D.ny = mog_cdiv(D.M, BM);
  dim3 g(D.nx, D.ny, batch * D.splitk);
  if (D.kseg > 0) {  // heads' dh = sum_z dhid_z W1_z^T (NT form only)
    if (!ta && tb) launch_epi<BM, BN, BK, PF, false, true, true>(epi, g, s, P, D);
    else launch_epi<BM, BN, BK, PF, false, false, true>(epi, g, s, P, D);
    return;
  }
  if (!ta && !tb) launch_epi<BM, BN, BK, PF, false, false, false>(epi, g, s, P, D);
  else if (!ta && tb) launch_epi<BM, BN, BK, PF, false, true, false>(epi, g, s, P, D);
  else if (ta && !tb) launch_epi<BM, BN, BK, PF, true, false, false>(epi, g, s, P, D);
  else launch_epi<BM, BN, BK, PF, true, true, false>(epi, g, s, P, D);
}

template <int BM, int BN, int BK, int NS, bool TA, bool TB>
void launch_dma_epi(int epi, dim3 g, hipStream_t s, const GemmPtrs& P, const GemmDims& D) {
#define MOG_GEMM_LAUNCH(E) gemm_f32_dma_kernel<BM, BN, BK, NS, TA, TB, E><<<g, 256, 0, s>>>(P, D)
  switch (epi) {
    case EPI_STORE: MOG_GEMM_LAUNCH(EPI_STORE); break;
    case EPI_RELU: MOG_GEMM_LAUNCH(EPI_RELU); break;
    case EPI_SOFTPLUS: MOG_GEMM_LAUNCH(EPI_SOFTPLUS); break;
    case EPI_SIGMOID_NOISE: MOG_GEMM_LAUNCH(EPI_SIGMOID_NOISE); break;
    case EPI_SOFTPLUS_BWD: MOG_GEMM_LAUNCH(EPI_SOFTPLUS_BWD); break;
    case EPI_ATOMIC: MOG_GEMM_LAUNCH(EPI_ATOMIC); break;
    case EPI_RELU_BWD: MOG_GEMM_LAUNCH(EPI_RELU_BWD); break;
  }
#undef MOG_GEMM_LAUNCH
}

// Returns MOG_ERR_INVALID (nothing launched) for a transposed A with BM < 64:
// a transposed A is a row-contiguous LDS image, which needs >= 64 rows.
template <int BM, int BN, int BK, int NS>
int launch_dma(bool ta, bool tb, int epi, hipStream_t s, const GemmPtrs& P, GemmDims D,
               int batch) {
  int kchunk = (D.K + D.splitk - 1) / D.splitk;
  kchunk = ((kchunk + BK - 1) / BK) * BK;
  if (kchunk == 0) kchunk = BK;
  D.kchunk = kchunk;
  D.splitk = (D.K + kchunk - 1) / kchunk;
  if (D.splitk < 1) D.splitk = 1;
  D.nx = mog_cdiv(D.N, BN);
  D.ny = mog_cdiv(D.M, BM);
  dim3 g(D.nx, D.ny, batch * D.splitk);
  if (!ta && !tb) {
    launch_dma_epi<BM, BN, BK, NS, false, false>(epi, g, s, P, D);
  } else if (!ta && tb) {
    launch_dma_epi<BM, BN, BK, NS, false, true>(epi, g, s, P, D);
  } else if constexpr (BM >= 64) {  // (a transposed A is a row-contiguous image: >= 64 rows)
    if (!tb) launch_dma_epi<BM, BN, BK, NS, true, false>(epi, g, s, P, D);
    else launch_dma_epi<BM, BN, BK, NS, true, true>(epi, g, s, P, D);
  } else {
    return MOG_ERR_INVALID;
  }
  return 0;
}

// Tile shape (measured on MI355X, scripts/bench_gemm_f32.py):
// 64x64 (2x2 waves of 32x32) wins on every train-step shape except the long-K
// x-projection (K = 2500), where 128x128 keeps more MFMAs per barrier and
// still gives every CU two workgroups.  Operands that allow it go through the
// LDS-DMA kernel (x-projection 457 -> 379 us, its gradient 385 -> 369 us,
// the dh GEMM 65 -> 49 us against register staging); register staging
// remains for unaligned / K % 4 operands and K segments.  Measured and not
// kept: BK = 32 (register staging -5..-25 %, LDS-DMA -3..-20 % on most
// shapes), 128x64 / 64x128 tiles, a 3-stage register pipeline with fragment
// prefetch (1 wave per SIMD at 128x128).  Profiling build (mog_prof_env):
// MOG_GEMM_TILE ("64" / "128") forces a tile, MOG_GEMM_DMA=0 the
// register-staged kernel.
int launch_auto(bool ta, bool tb, int epi, hipStream_t s, const GemmPtrs& P, const GemmDims& D,
                int batch) {
  static const char* force = mog_prof_env("MOG_GEMM_TILE");
  const long big = (long)mog_cdiv(D.M, 128) * mog_cdiv(D.N, 128) * batch * D.splitk;
  bool b128 = !ta && D.K >= 2048 && D.M >= 128 && D.N >= 128 && big >= 512;
  if (force != nullptr) b128 = atoi(force) == 128;
  // LDS-DMA form: 16-B source chunks must be aligned and lie wholly inside or
  // outside the k range and the operand's last row (K % 4 for k-contiguous
  // operands, M / N % 4 for row-contiguous ones); no K segments; the fused
  // bias-gradient column sum only from a row-contiguous B
  static const char* dma_env = mog_prof_env("MOG_GEMM_DMA");
  const bool dma = (dma_env == nullptr || atoi(dma_env) != 0) && D.kseg == 0 && D.vecA &&
                   D.vecB && (ta ? D.M % 4 == 0 : D.K % 4 == 0) &&
                   (tb ? D.K % 4 == 0 : D.N % 4 == 0) && !(tb && P.colsum[0] != nullptr);
  if (dma) {
    // Small M (the reference's batch of 64: M = 64 / 192 rows): the 64 x 64
    // grid leaves most CUs idle and every workgroup walks the whole K (no
    // split-K in a bit-exact forward chain), so 32 x 64 tiles (one 16-row
    // MFMA tile per wave, 32-deep k-tiles) double the workgroups and halve
    // each one's MFMA chain per k-step.  Same k order: same bits.
    const long t64 = (long)mog_cdiv(D.M, 64) * mog_cdiv(D.N, 64) * batch * D.splitk;
    const long t3264 = (long)mog_cdiv(D.M, 32) * mog_cdiv(D.N, 64) * batch * D.splitk;
    bool small = !ta && t64 < 128;
    // still under 128 workgroups at 32 x 64 (M = 64 x N = 1024 x-projection
    // of the reference's batch): 32 x 32 tiles, one 16 x 16 MFMA tile per wave
    bool tiny = small && t3264 < 128;
    if (force != nullptr) {
      small = !ta && (atoi(force) == 3264 || atoi(force) == 3232);
      tiny = !ta && atoi(force) == 3232;
    }
    // Four stages with fragment double-buffering: each workgroup walks a long
    // serial k chain (no split-K), so two k-tiles of DMA stay in flight and a
    // tile's fragments are read while the previous one's MFMAs run (captured
    // batch-64 step 0.396 -> 0.391 ms, AIR-ASR 1.355 -> 1.347 ms; three stages,
    // without the fragment double-buffering, 0.438 ms).  MOG_GEMM_TNS=2
    // (profiling build) keeps the two-stage form.
    static const char* tns_env = mog_prof_env("MOG_GEMM_TNS");
    const bool tns2 = tns_env != nullptr && atoi(tns_env) == 2;
    if (tiny) {
      if (tns2) return launch_dma<32, 32, 32, 2>(ta, tb, epi, s, P, D, batch);
      return launch_dma<32, 32, 32, 4>(ta, tb, epi, s, P, D, batch);
    }
    if (small) {
      if (tns2) return launch_dma<32, 64, 32, 2>(ta, tb, epi, s, P, D, batch);
      return launch_dma<32, 64, 32, 4>(ta, tb, epi, s, P, D, batch);
    }
    // stages (measured, scripts/bench_gemm_f32.py): 4 with fragment
    // double-buffering for the split-K weight gradients (transA), 3 for the
    // rest, where a fifth/sixth workgroup per CU beats the deeper pipeline
    // 128x64 (4 waves of 64x32: twice the MFMAs per barrier of 64x64, still
    // >= 3 workgroups per CU) for the tall non-transposed-A GEMMs: the
    // T*B-row forward layers and input gradients, the recurrent GEMM
    // (scripts/bench_gemm_f32.py: dX 196 -> 188 / 190 -> 182 us, recurrent
    // 54 -> 48 us; N = 256 layers and split-K weight gradients lose)
    bool t12864 = !ta && !b128 && D.N >= 512 && (long)D.M * D.N >= 8192L * 1024;
    if (force != nullptr) t12864 = atoi(force) == 12864;
    // 32-deep k-tiles in two stages (the LDS bytes of 16-deep x 4): half the
    // barriers per MFMA.  Measured (scripts/bench_gemm_f32.py):
    // faster for the weight gradients (transA, +1..6 %) and the transB input
    // gradients (dh +15 %), slower for the forward layers (recurrent -18 %,
    // T*B-row layers -2..5 %).  MOG_GEMM_BK=16|32 forces one depth.
    static const char* bk_env = mog_prof_env("MOG_GEMM_BK");
    bool bk32 = ta || tb;
    if (bk_env != nullptr) bk32 = atoi(bk_env) == 32;
    if (bk32 && !b128) {
      // MOG_GEMM_NS=3|4: deeper 32-deep pipelines (48 / 64 KB per workgroup)
      static const char* ns_env = mog_prof_env("MOG_GEMM_NS");
      const int ns = ns_env != nullptr ? atoi(ns_env) : 2;
      if (t12864) return launch_dma<128, 64, 32, 2>(ta, tb, epi, s, P, D, batch);
      else if (ns == 4) return launch_dma<64, 64, 32, 4>(ta, tb, epi, s, P, D, batch);
      else if (ns == 3) return launch_dma<64, 64, 32, 3>(ta, tb, epi, s, P, D, batch);
      else return launch_dma<64, 64, 32, 2>(ta, tb, epi, s, P, D, batch);
    }
    if (t12864) {
      if (ta) return launch_dma<128, 64, 16, 4>(ta, tb, epi, s, P, D, batch);
      else return launch_dma<128, 64, 16, 3>(ta, tb, epi, s, P, D, batch);
    } else if (b128) {
      if (ta) return launch_dma<128, 128, 16, 4>(ta, tb, epi, s, P, D, batch);
      else return launch_dma<128, 128, 16, 3>(ta, tb, epi, s, P, D, batch);
    } else {
      if (ta) return launch_dma<64, 64, 16, 4>(ta, tb, epi, s, P, D, batch);
      else return launch_dma<64, 64, 16, 3>(ta, tb, epi, s, P, D, batch);
    }
  }
  // k-segment NT chains of a small batch (AIR / AIR-ASR's per-step head
  // gradients at the reference's batch of 64: a 64 x 64 grid of a dozen
  // workgroups, each a serial K = 64..320 chain): 32 x 32 tiles 32 deep --
  // four times the workgroups, half the barriers per k.  Same k order: same
  // bits.  MOG_KSEG_SMALL=0 keeps 64 x 64 x 16.
  static const char* ks_env = mog_prof_env("MOG_KSEG_SMALL");
  if (D.kseg > 0 && !ta && tb && D.kseg % 32 == 0 && (ks_env == nullptr || atoi(ks_env) != 0) &&
      (long)mog_cdiv(D.M, 64) * mog_cdiv(D.N, 64) * batch < 128) {
    GemmDims E = D;
    E.kchunk = ((E.K + 31) / 32) * 32;
    E.splitk = 1;
    E.nx = mog_cdiv(E.N, 32);
    E.ny = mog_cdiv(E.M, 32);
    launch_epi<32, 32, 32, 1, false, true, true>(epi, dim3(E.nx, E.ny, batch), s, P, E);
    return 0;
  }
  // the NT form of a small batch off the LDS-DMA path (an operand off the
  // 16-byte alignment, e.g. K = Z = 50: the latent layer's input gradient at the
  // batch of 64): 32 x 32 x 32 tiles as above.  MOG_NT_SMALL=0 keeps 64 x 64 x 16.
  static const char* nt_env = mog_prof_env("MOG_NT_SMALL");
  if (D.kseg == 0 && !ta && tb && D.splitk == 1 && (nt_env == nullptr || atoi(nt_env) != 0) &&
      (long)mog_cdiv(D.M, 64) * mog_cdiv(D.N, 64) * batch < 128) {
    GemmDims E = D;
    E.kchunk = ((E.K + 31) / 32) * 32;
    if (E.kchunk == 0) E.kchunk = 32;
    E.nx = mog_cdiv(E.N, 32);
    E.ny = mog_cdiv(E.M, 32);
    launch_epi<32, 32, 32, 1, false, true, false>(epi, dim3(E.nx, E.ny, batch), s, P, E);
    return 0;
  }
  if (b128) launch_tile<128, 128, 16, 1>(ta, tb, epi, s, P, D, batch);
  else launch_tile<64, 64, 16, 1>(ta, tb, epi, s, P, D, batch);
  return 0;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int mog_gemm_f32(int batch, const float* const* A, const float* const* B,
                            float* const* C, const float* const* bias,
                            const float* const* Cin, float* const* Cpre,
                            const float* const* aux, float* const* colsum, int M, int N, int K,
                            int lda, int ldb, int ldc, int ldaux, int transA, int transB,
                            int epi, float aux_scale, int splitk, void* stream) {
  MOG_CHECK_ARG(batch >= 1 && batch <= MAXB);
  MOG_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && splitk >= 1);
  MOG_CHECK_ARG(epi >= EPI_STORE && epi <= EPI_RELU_BWD);
  MOG_CHECK_ARG(splitk == 1 || epi == EPI_ATOMIC);
  MOG_CHECK_ARG(colsum == nullptr || epi == EPI_ATOMIC);
  MOG_CHECK_ARG(C && (K == 0 || (A && B)));
  if (M == 0 || N == 0) return 0;
  GemmPtrs P;
  bool va = true, vb = true;
  for (int i = 0; i < MAXB; ++i) {
    const bool on = i < batch;
    P.A[i] = (on && A) ? A[i] : nullptr;
    P.B[i] = (on && B) ? B[i] : nullptr;
    P.C[i] = on ? C[i] : nullptr;
    P.bias[i] = (on && bias) ? bias[i] : nullptr;
    P.Cin[i] = (on && Cin) ? Cin[i] : nullptr;
    P.Cpre[i] = (on && Cpre) ? Cpre[i] : nullptr;
    P.aux[i] = (on && aux) ? aux[i] : nullptr;
    P.colsum[i] = (on && colsum) ? colsum[i] : nullptr;
    if (on) {
      MOG_CHECK_ARG(P.C[i] && (K == 0 || (P.A[i] && P.B[i])));
      va = va && aligned16(P.A[i]);
      vb = vb && aligned16(P.B[i]);
      if (epi == EPI_SIGMOID_NOISE || epi == EPI_SOFTPLUS_BWD || epi == EPI_RELU_BWD)
        MOG_CHECK_ARG(P.aux[i] != nullptr);
    }
  }
  // operands are addressed through raw buffer descriptors (32-bit byte offsets)
  const long extA = transA ? (long)(K - 1) * lda + M : (long)(M - 1) * lda + K;
  const long extB = transB ? (long)(N - 1) * ldb + K : (long)(K - 1) * ldb + N;
  MOG_CHECK_ARG(extA * 4 < 0x7ffffff0L && extB * 4 < 0x7ffffff0L);
  GemmDims D;
  D.M = M; D.N = N; D.K = K; D.lda = lda; D.ldb = ldb; D.ldc = ldc; D.ldaux = ldaux;
  D.aux_scale = aux_scale;
  D.vecA = va && (lda % 4 == 0);
  D.vecB = vb && (ldb % 4 == 0);
  bool vc = ldc % 4 == 0 && (ldaux % 4 == 0 || aux == nullptr);
  for (int i = 0; i < batch; ++i)
    vc = vc && aligned16(P.C[i]) && (!P.Cpre[i] || aligned16(P.Cpre[i])) &&
         (!P.aux[i] || aligned16(P.aux[i]));
  D.vecC = vc;
  D.splitk = splitk;
  D.kchunk = 0;
  D.kseg = 0;
  D.eps_gen = 0;
  D.eps_seed = D.eps_off = 0;
  MOG_TRY(launch_auto(transA, transB, epi, mog_stream(stream), P, D, batch));
  MOG_LAUNCH_RET();
}

// C = sigmoid((A B + bias) + scale * eps), eps standard normal from Philox
// (seed, offset) in [M][N] fill order (vae.py:44-46, air_model.py:548-550 with
// the noise of mog_rng_fill generated in the epilogue instead of read)
extern "C" int mog_gemm_f32_sigmoid_philox(const float* A, const float* B, float* C,
                                           const float* bias, int M, int N, int K, int lda,
                                           int ldb, int ldc, float scale,
                                           unsigned long long seed, unsigned long long offset,
                                           void* stream) {
  MOG_CHECK_ARG(A && B && C && M >= 0 && N >= 0 && K >= 0 && N % 4 == 0);
  if (M == 0 || N == 0) return 0;
  MOG_CHECK_ARG((long)(K - 1) * ldb + N < 0x1ffffffcL && (long)(M - 1) * lda + K < 0x1ffffffcL);
  GemmPtrs P = {};
  P.A[0] = A; P.B[0] = B; P.C[0] = C; P.bias[0] = bias;
  GemmDims D;
  D.M = M; D.N = N; D.K = K; D.lda = lda; D.ldb = ldb; D.ldc = ldc; D.ldaux = 0;
  D.aux_scale = scale;
  D.vecA = aligned16(A) && lda % 4 == 0;
  D.vecB = aligned16(B) && ldb % 4 == 0;
  D.vecC = aligned16(C) && ldc % 4 == 0;
  D.splitk = 1;
  D.kchunk = 0;
  D.kseg = 0;
  D.eps_gen = 1;
  D.eps_seed = seed;
  D.eps_off = offset;
  MOG_TRY(launch_auto(false, false, EPI_SIGMOID_NOISE, mog_stream(stream), P, D, 1));
  MOG_LAUNCH_RET();
}

// C = epi( sum_s A_s op(B_s) ) as ONE k-ordered chain over the concatenated
// K = nseg * kseg (segment s read from A[s] / B[s]): e.g. the hidden-state
// gradient of the five heads, dh = sum_z dhid_z W1_z^T (air_model.py:462-499
// backward), without atomics.
extern "C" int mog_gemm_f32_kseg(int nseg, const float* const* A, const float* const* B,
                                 float* C, const float* bias, const float* Cin, int M, int N,
                                 int kseg, int lda, int ldb, int ldc, int transA, int transB,
                                 int epi, void* stream) {
  MOG_CHECK_ARG(nseg >= 1 && nseg <= MAXB && kseg > 0 && kseg % 16 == 0);
  MOG_CHECK_ARG(M >= 0 && N >= 0 && A && B && C);
  MOG_CHECK_ARG(epi == EPI_STORE || epi == EPI_ATOMIC);
  MOG_CHECK_ARG(!transA);
  if (M == 0 || N == 0) return 0;
  GemmPtrs P = {};
  bool va = true, vb = true;
  for (int i = 0; i < nseg; ++i) {
    MOG_CHECK_ARG(A[i] && B[i]);
    P.A[i] = A[i];
    P.B[i] = B[i];
    va = va && aligned16(A[i]);
    vb = vb && aligned16(B[i]);
  }
  P.C[0] = C;
  P.bias[0] = bias;
  P.Cin[0] = Cin;
  GemmDims D;
  D.M = M; D.N = N; D.K = nseg * kseg; D.lda = lda; D.ldb = ldb; D.ldc = ldc; D.ldaux = 0;
  D.aux_scale = 0.0f;
  D.vecA = va && (lda % 4 == 0);
  D.vecB = vb && (ldb % 4 == 0);
  D.vecC = 0;
  D.splitk = 1;
  D.kchunk = 0;
  D.kseg = kseg;
  D.segoff[0] = 0;
  D.segoff[1] = nseg;
  D.eps_gen = 0;
  D.eps_seed = D.eps_off = 0;
  MOG_TRY(launch_auto(transA, transB, epi, mog_stream(stream), P, D, 1));
  MOG_LAUNCH_RET();
}

// nprob independent k-segment chains of one shape in ONE launch: problem z
// is C_z = Cin_z + sum_s A_s B_s^T over its nseg[z] segments (A / B hold the
// problems' segments back to back): e.g. one AIR-ASR loop step's dh (five
// heads), dhg (two generative heads) and dhg_{t-1} (the z_pres prior).
extern "C" int mog_gemm_f32_kseg_group(int nprob, const int* nseg, const float* const* A,
                                       const float* const* B, float* const* C,
                                       const float* const* Cin, int M, int N, int kseg, int lda,
                                       int ldb, int ldc, int transB, void* stream) {
  MOG_CHECK_ARG(nprob >= 1 && nprob <= 4 && nseg && A && B && C && kseg > 0 && kseg % 16 == 0);
  MOG_CHECK_ARG(M >= 0 && N >= 0);
  if (M == 0 || N == 0) return 0;
  GemmPtrs P = {};
  GemmDims D;
  bool va = true, vb = true;
  int tot = 0, most = 0;
  for (int z = 0; z < nprob; ++z) {
    MOG_CHECK_ARG(nseg[z] >= 1 && C[z]);
    D.segoff[z] = tot;
    tot += nseg[z];
    most = nseg[z] > most ? nseg[z] : most;
    P.C[z] = C[z];
    P.Cin[z] = Cin ? Cin[z] : nullptr;
  }
  MOG_CHECK_ARG(tot <= MAXB);
  D.segoff[nprob] = tot;
  for (int i = 0; i < tot; ++i) {
    MOG_CHECK_ARG(A[i] && B[i]);
    P.A[i] = A[i];
    P.B[i] = B[i];
    va = va && aligned16(A[i]);
    vb = vb && aligned16(B[i]);
  }
  D.M = M; D.N = N; D.K = most * kseg; D.lda = lda; D.ldb = ldb; D.ldc = ldc; D.ldaux = 0;
  D.aux_scale = 0.0f;
  D.vecA = va && (lda % 4 == 0);
  D.vecB = vb && (ldb % 4 == 0);
  D.vecC = 0;
  D.splitk = 1;
  D.kchunk = 0;
  D.kseg = kseg;
  D.eps_gen = 0;
  D.eps_seed = D.eps_off = 0;
  MOG_TRY(launch_auto(false, transB != 0, EPI_STORE, mog_stream(stream), P, D, nprob));
  MOG_LAUNCH_RET();
}
