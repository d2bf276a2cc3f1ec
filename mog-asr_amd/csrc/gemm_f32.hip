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
// (BM/2)x(BN/2) of 16x16 MFMA tiles), BK = 16, register-staged double
// buffering (next tile's global loads in flight during the MFMAs).
//
// Weight-gradient form: transA + EPI_ATOMIC + split-K computes dW += X^T dY;
// when `colsum` is given the workgroups of the first M-tile row also add the
// column sums of their dY tiles into colsum[n] (the bias gradient, TF
// BiasAddGrad), so no separate reduction pass re-reads dY.
//
// Replaces the TF-1.12 MatMul / BiasAdd / Softplus / Relu / Sigmoid op groups
// of the hot path (SURVEY.md §2 table "TF op group on the hot path").
#include "mog_common.h"

namespace {

enum {
  EPI_STORE = 0,          // C = acc (+ bias)
  EPI_RELU = 1,           // C = relu(acc + bias), Cpre = acc + bias
  EPI_SOFTPLUS = 2,       // C = softplus_tf(acc + bias), Cpre = acc + bias
  EPI_SIGMOID_NOISE = 3,  // C = sigmoid((acc + bias) + aux*scale), Cpre = acc + bias
  EPI_SOFTPLUS_BWD = 4,   // C = acc * sigmoid(aux)        (dX through softplus)
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
  float aux_scale;
};

constexpr int BK = 16, PADF = 16;

// bijective XCD-grouping remap of the linear workgroup id (guide §5, T1):
// consecutive ids (same A row-panel, neighbouring N tiles) share one XCD's L2
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

template <int BM, int BN, bool TA, bool TB, int EPI>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmPtrs P, GemmDims D) {
#pragma clang fp contract(off)
  constexpr int MI = BM / 32, NI = BN / 32;     // 16x16 tiles per wave
  constexpr int NA = BM * BK / 1024, NB = BN * BK / 1024;  // float4 loads per thread
  constexpr int CPR = BK / 4;                              // float4 chunks per k-row
  constexpr int LDA_S = BM + PADF, LDB_S = BN + PADF;
  constexpr int STAGE = BK * (LDA_S + LDB_S);
  // two pipeline stages in ONE shared array: [stage][A: BK x LDA_S | B: BK x LDB_S]
  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];
  const int nwg = gridDim.x * gridDim.y * gridDim.z;
  const int wg = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), nwg);
  const int bx = wg % D.nx, by = (wg / D.nx) % D.ny, bz = wg / (D.nx * D.ny);
  const int z = bz / D.splitk, ks = bz - z * D.splitk;
  const float* __restrict__ A = P.A[z];
  const float* __restrict__ Bm = P.B[z];
  const int m0 = by * BM, n0 = bx * BN;
  const int kbeg = ks * D.kchunk;
  const int kend = min(D.K, kbeg + D.kchunk);
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
        float v = 0.0f;
        if (Cin != nullptr && ks == 0) {
          const int row = m0 + wm + mi * 16 + (lane >> 4) * 4 + r;
          const int col = n0 + wn + ni * 16 + (lane & 15);
          if (row < M && col < N) v = Cin[(size_t)row * D.ldc + col];
        }
        acc[mi][ni][r] = v;
      }

  float ra[NA][4], rb[NB][4];
  auto load_tiles = [&](int k0) {
    const float* __restrict__ Aq = A;
    const float* __restrict__ Bq = Bm;
    int koff = 0;
    if (D.kseg > 0) {  // a BK tile never straddles two segments (kseg % BK == 0)
      const int sg = k0 / D.kseg;
      Aq = P.A[sg];
      Bq = P.B[sg];
      koff = sg * D.kseg;
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int q = t + 256 * i;
      if (!TA) {
        const int row = q / CPR, kc = (q % CPR) * 4;
        const int gm = m0 + row, gk = k0 + kc;
        if (D.vecA && gm < M && gk + 3 < kend) {
          const float4 v = *reinterpret_cast<const float4*>(Aq + (size_t)gm * D.lda + (gk - koff));
          ra[i][0] = v.x; ra[i][1] = v.y; ra[i][2] = v.z; ra[i][3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ra[i][j] = (gm < M && gk + j < kend) ? Aq[(size_t)gm * D.lda + (gk - koff) + j] : 0.0f;
        }
      } else {
        const int k = q / (BM / 4), mc = (q % (BM / 4)) * 4;
        const int gk = k0 + k, gm = m0 + mc;
        if (D.vecA && gk < kend && gm + 3 < M) {
          const float4 v = *reinterpret_cast<const float4*>(Aq + (size_t)(gk - koff) * D.lda + gm);
          ra[i][0] = v.x; ra[i][1] = v.y; ra[i][2] = v.z; ra[i][3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ra[i][j] = (gk < kend && gm + j < M) ? Aq[(size_t)(gk - koff) * D.lda + gm + j] : 0.0f;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = t + 256 * i;
      if (!TB) {
        const int k = q / (BN / 4), nc = (q % (BN / 4)) * 4;
        const int gk = k0 + k, gn = n0 + nc;
        if (D.vecB && gk < kend && gn + 3 < N) {
          const float4 v = *reinterpret_cast<const float4*>(Bq + (size_t)(gk - koff) * D.ldb + gn);
          rb[i][0] = v.x; rb[i][1] = v.y; rb[i][2] = v.z; rb[i][3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            rb[i][j] = (gk < kend && gn + j < N) ? Bq[(size_t)(gk - koff) * D.ldb + gn + j] : 0.0f;
        }
      } else {
        const int n = q / CPR, kc = (q % CPR) * 4;
        const int gn = n0 + n, gk = k0 + kc;
        if (D.vecB && gn < N && gk + 3 < kend) {
          const float4 v = *reinterpret_cast<const float4*>(Bq + (size_t)gn * D.ldb + (gk - koff));
          rb[i][0] = v.x; rb[i][1] = v.y; rb[i][2] = v.z; rb[i][3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            rb[i][j] = (gn < N && gk + j < kend) ? Bq[(size_t)gn * D.ldb + (gk - koff) + j] : 0.0f;
        }
      }
    }
  };
  auto store_tiles = [&](int stage) {
    float* As = lds + stage * STAGE;
    float* Bs = As + BK * LDA_S;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int q = t + 256 * i;
      if (!TA) {
        const int row = q / CPR, kc = (q % CPR) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) As[(kc + j) * LDA_S + row] = ra[i][j];
      } else {
        const int k = q / (BM / 4), mc = (q % (BM / 4)) * 4;
        *reinterpret_cast<floatx4*>(&As[k * LDA_S + mc]) =
            floatx4{ra[i][0], ra[i][1], ra[i][2], ra[i][3]};
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = t + 256 * i;
      if (!TB) {
        const int k = q / (BN / 4), nc = (q % (BN / 4)) * 4;
        *reinterpret_cast<floatx4*>(&Bs[k * LDB_S + nc]) =
            floatx4{rb[i][0], rb[i][1], rb[i][2], rb[i][3]};
      } else {
        const int n = q / CPR, kc = (q % CPR) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) Bs[(kc + j) * LDB_S + n] = rb[i][j];
      }
    }
  };
  auto compute = [&](int stage) {
    const float* As = lds + stage * STAGE;
    const float* Bs = As + BK * LDA_S;
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const int k = kk * 4 + (lane >> 4);
      float a[MI], b[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) a[mi] = As[k * LDA_S + wm + mi * 16 + (lane & 15)];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) b[ni] = Bs[k * LDB_S + wn + ni * 16 + (lane & 15)];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
    }
    if (do_cs) {
#pragma unroll
      for (int k = 0; k < BK; ++k) cs += Bs[k * LDB_S + t];
    }
  };

  // two-stage pipeline: tile it is multiplied from stage it&1 while tile it+1
  // is written to the other stage and tile it+2's global loads are in flight;
  // one barrier per k-tile.  The k order of every fma chain is unchanged.
  const int nk = kbeg < kend ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    load_tiles(kbeg);
    store_tiles(0);
    if (nk > 1) load_tiles(kbeg + BK);
    __syncthreads();
    for (int it = 0; it < nk; ++it) {
      const int cur = it & 1;
      compute(cur);
      if (it + 1 < nk) {
        store_tiles(cur ^ 1);
        if (it + 2 < nk) load_tiles(kbeg + (it + 2) * BK);
      }
      __syncthreads();
    }
  }
  if (do_cs && n0 + t < N) atomicAdd(colsum + n0 + t, cs);

  float* C = P.C[z];
  const float* bias = P.bias[z];
  const float* aux = P.aux[z];
  float* Cpre = P.Cpre[z];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + mi * 16 + (lane >> 4) * 4 + r;
        const int col = n0 + wn + ni * 16 + (lane & 15);
        if (row >= M || col >= N) continue;
        const size_t o = (size_t)row * D.ldc + col;
        float v = acc[mi][ni][r];
        if (EPI == EPI_ATOMIC) {
          atomicAdd(C + o, v);
          continue;
        }
        if (EPI == EPI_SOFTPLUS_BWD) {
          C[o] = v * mog_sigmoidf(aux[(size_t)row * D.ldaux + col]);
          continue;
        }
        if (EPI == EPI_RELU_BWD) {
          C[o] = aux[(size_t)row * D.ldaux + col] > 0.0f ? v : 0.0f;
          continue;
        }
        if (bias != nullptr) v = v + bias[col];
        if (EPI == EPI_STORE) {
          C[o] = v;
        } else {
          if (Cpre != nullptr) Cpre[o] = v;
          if (EPI == EPI_RELU) C[o] = v > 0.0f ? v : 0.0f;
          if (EPI == EPI_SOFTPLUS) C[o] = mog_softplusf(v);
          if (EPI == EPI_SIGMOID_NOISE)
            C[o] = mog_sigmoidf(v + aux[(size_t)row * D.ldaux + col] * D.aux_scale);
        }
      }
}

template <int BM, int BN, bool TA, bool TB>
void launch_epi(int epi, dim3 g, hipStream_t s, const GemmPtrs& P, const GemmDims& D) {
  switch (epi) {
    case EPI_STORE: gemm_f32_kernel<BM, BN, TA, TB, EPI_STORE><<<g, 256, 0, s>>>(P, D); break;
    case EPI_RELU: gemm_f32_kernel<BM, BN, TA, TB, EPI_RELU><<<g, 256, 0, s>>>(P, D); break;
    case EPI_SOFTPLUS:
      gemm_f32_kernel<BM, BN, TA, TB, EPI_SOFTPLUS><<<g, 256, 0, s>>>(P, D); break;
    case EPI_SIGMOID_NOISE:
      gemm_f32_kernel<BM, BN, TA, TB, EPI_SIGMOID_NOISE><<<g, 256, 0, s>>>(P, D); break;
    case EPI_SOFTPLUS_BWD:
      gemm_f32_kernel<BM, BN, TA, TB, EPI_SOFTPLUS_BWD><<<g, 256, 0, s>>>(P, D); break;
    case EPI_ATOMIC: gemm_f32_kernel<BM, BN, TA, TB, EPI_ATOMIC><<<g, 256, 0, s>>>(P, D); break;
    case EPI_RELU_BWD:
      gemm_f32_kernel<BM, BN, TA, TB, EPI_RELU_BWD><<<g, 256, 0, s>>>(P, D); break;
  }
}

template <int BM, int BN>
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
  if (!ta && !tb) launch_epi<BM, BN, false, false>(epi, g, s, P, D);
  else if (!ta && tb) launch_epi<BM, BN, false, true>(epi, g, s, P, D);
  else if (ta && !tb) launch_epi<BM, BN, true, false>(epi, g, s, P, D);
  else launch_epi<BM, BN, true, true>(epi, g, s, P, D);
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
  GemmDims D;
  D.M = M; D.N = N; D.K = K; D.lda = lda; D.ldb = ldb; D.ldc = ldc; D.ldaux = ldaux;
  D.aux_scale = aux_scale;
  D.vecA = va && (lda % 4 == 0);
  D.vecB = vb && (ldb % 4 == 0);
  D.splitk = splitk;
  D.kchunk = 0;
  D.kseg = 0;
  hipStream_t s = mog_stream(stream);
  // 128x128 tiles once both output dims fill them and the grid still covers
  // the chip (>= 512 workgroups); 64x64 otherwise.
  // (measured: 128x128 is on par for the large NN GEMMs and slower for the
  // split-K weight-gradient form, so the transposed-A form stays on 64x64)
  const long big_tiles = (long)mog_cdiv(M, 128) * mog_cdiv(N, 128) * batch * splitk;
  if (!transA && M >= 128 && N >= 128 && big_tiles >= 512)
    launch_tile<128, 128>(transA, transB, epi, s, P, D, batch);
  else
    launch_tile<64, 64>(transA, transB, epi, s, P, D, batch);
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
  MOG_CHECK_ARG(nseg >= 1 && nseg <= MAXB && kseg > 0 && kseg % BK == 0);
  MOG_CHECK_ARG(M >= 0 && N >= 0 && A && B && C);
  MOG_CHECK_ARG(epi == EPI_STORE || epi == EPI_ATOMIC);
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
  D.splitk = 1;
  D.kchunk = 0;
  D.kseg = kseg;
  launch_tile<64, 64>(transA, transB, epi, mog_stream(stream), P, D, 1);
  MOG_LAUNCH_RET();
}
