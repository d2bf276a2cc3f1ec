// bf16-operand GEMM (fp32 accumulate) on gfx950 v_mfma_f32_16x16x32_bf16 —
// the glimpse-VAE layers of the bf16 configuration (BASELINE.json configs[1]).
//
// Two operand forms, chosen so no layout conversion happens at run time:
//   NT:  C[m][n] = sum_k A[m][k] * B[n][k]        (A rows and B rows k-contiguous)
//        forward   Y  = X  W   with B = W^T packed  ([out][in] bf16)
//        backward  dX = dY W^T with B = W  packed   ([in][out] bf16)
//   TN:  C[m][n] = sum_k A[k][m] * B[k][n]        (both operands k-major)
//        weight gradient dW = X^T dY over the batch rows (split-K, fp32 atomics,
//        fused bias-gradient column sums); fragments come out of the k-major
//        LDS images with the gfx950 transpose read ds_read_b64_tr_b16.
// All k extents are multiples of 8 (buffers are padded with zeros), so every
// global load is a 16-byte vector.
//
// Pipeline: BK = 64, two LDS stages in ONE __shared__ array, register-staged
// prefetch of tile i+2 while tile i is multiplied and tile i+1 is written to
// the other stage — one barrier per k-iteration.  Workgroup ids are remapped
// so that the workgroups sharing an A row-panel run on one XCD (shared L2).
#include <cstdlib>

#include "bf16_epi.h"
#include "mog_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

enum {
  B_STORE = 0,           // C = acc (+bias)                       fp32 or bf16 out
  B_SOFTPLUS = 1,        // C = softplus(acc + bias)              bf16 out
  B_SIGMOID_NOISE = 2,   // C = sigmoid(acc + bias + aux*scale)   fp32 out (aux fp32)
  B_SOFTPLUS_BWD = 3,    // C = acc * (1 - exp(-aux))  [aux = softplus output, bf16]
  B_ATOMIC = 4,          // C += acc (fp32 atomics), optional colsum of B
};

constexpr int MAXB = 8;
struct BPtrs {
  const __bf16* A[MAXB];
  const __bf16* B[MAXB];
  void* C[MAXB];
  const float* bias[MAXB];
  const float* Cin[MAXB];
  const void* aux[MAXB];
  float* colsum[MAXB];
};
struct BDims {
  int M, N, K, lda, ldb, ldc, ldaux, splitk, kchunk, out_bf16, nx, ny;
  float aux_scale;
};

constexpr int BKK = 64;

__device__ __forceinline__ float bf2f(__bf16 v) { return (float)v; }

// bijective XCD-grouping remap of the linear workgroup id (guide §5, T1)
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

template <int BM, int BN, bool TN, int EPI>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(BPtrs P, BDims D) {
  constexpr int MI = BM / 32, NI = BN / 32;
  // LDS images.  NT: [rows][BKK+8] (k contiguous).  TN: [BKK][cols+8].
  constexpr int A_ELEMS = TN ? BKK * (BM + 8) : BM * (BKK + 8);
  constexpr int B_ELEMS = TN ? BKK * (BN + 8) : BN * (BKK + 8);
  constexpr int STAGE = A_ELEMS + B_ELEMS;
  constexpr int NA = (BM * BKK / 8) / 256;  // 16-byte chunks per thread
  constexpr int NB = (BN * BKK / 8) / 256;
  constexpr int CPR = BKK / 8;              // 16-byte chunks per k-row (NT)
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * STAGE];

  const int nwg = gridDim.x * gridDim.y * gridDim.z;
  const int orig = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const int wg = xcd_remap(orig, nwg);
  const int bx = wg % D.nx, by = (wg / D.nx) % D.ny, bz = wg / (D.nx * D.ny);

  const int z = bz / D.splitk, ks = bz - z * D.splitk;
  const __bf16* __restrict__ A = P.A[z];
  const __bf16* __restrict__ Bm = P.B[z];
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

  u32x4 ra[NA], rb[NB];
  const u32x4 zero4 = {0u, 0u, 0u, 0u};
  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int q = t + 256 * i;
      if (!TN) {
        const int row = q / CPR, kc = (q % CPR) * 8;
        const int gm = m0 + row, gk = k0 + kc;
        ra[i] = (gm < M && gk < kend)
                    ? *reinterpret_cast<const u32x4*>(A + (size_t)gm * D.lda + gk) : zero4;
      } else {
        const int k = q / (BM / 8), mc = (q % (BM / 8)) * 8;
        const int gk = k0 + k, gm = m0 + mc;
        // gm < M (not < lda): a caller may offset A to a column window
        // (row chunks of a weight gradient); 8-wide loads stay inside the row
        ra[i] = (gk < kend && gm < M)
                    ? *reinterpret_cast<const u32x4*>(A + (size_t)gk * D.lda + gm) : zero4;
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = t + 256 * i;
      if (!TN) {
        const int row = q / CPR, kc = (q % CPR) * 8;
        const int gn = n0 + row, gk = k0 + kc;
        rb[i] = (gn < N && gk < kend)
                    ? *reinterpret_cast<const u32x4*>(Bm + (size_t)gn * D.ldb + gk) : zero4;
      } else {
        const int k = q / (BN / 8), nc = (q % (BN / 8)) * 8;
        const int gk = k0 + k, gn = n0 + nc;
        rb[i] = (gk < kend && gn < D.ldb)
                    ? *reinterpret_cast<const u32x4*>(Bm + (size_t)gk * D.ldb + gn) : zero4;
      }
    }
  };
  auto store_tiles = [&](int stage) {
    __bf16* As = lds + stage * STAGE;
    __bf16* Bs = As + A_ELEMS;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int q = t + 256 * i;
      if (!TN) {
        const int row = q / CPR, kc = (q % CPR) * 8;
        *reinterpret_cast<u32x4*>(&As[row * (BKK + 8) + kc]) = ra[i];
      } else {
        const int k = q / (BM / 8), mc = (q % (BM / 8)) * 8;
        *reinterpret_cast<u32x4*>(&As[k * (BM + 8) + mc]) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = t + 256 * i;
      if (!TN) {
        const int row = q / CPR, kc = (q % CPR) * 8;
        *reinterpret_cast<u32x4*>(&Bs[row * (BKK + 8) + kc]) = rb[i];
      } else {
        const int k = q / (BN / 8), nc = (q % (BN / 8)) * 8;
        *reinterpret_cast<u32x4*>(&Bs[k * (BN + 8) + nc]) = rb[i];
      }
    }
  };

  const int g = lane >> 4, li = lane & 15;
  // transpose-read lane roles: lane 4q+p of a 16-lane group -> row q, cols 4p..4p+3
  const int tq = li >> 2, tp = li & 3;
  auto compute = [&](int stage) {
    const __bf16* As = lds + stage * STAGE;
    const __bf16* Bs = As + A_ELEMS;
#pragma unroll
    for (int kk = 0; kk < BKK / 32; ++kk) {
      bf16x8 a[MI], b[NI];
      if (!TN) {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
          a[mi] = *reinterpret_cast<const bf16x8*>(
              &As[(wm + mi * 16 + li) * (BKK + 8) + kk * 32 + 8 * g]);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          b[ni] = *reinterpret_cast<const bf16x8*>(
              &Bs[(wn + ni * 16 + li) * (BKK + 8) + kk * 32 + 8 * g]);
      } else {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
          const __bf16* p0 = &As[(kk * 32 + 8 * g + tq) * (BM + 8) + wm + mi * 16 + 4 * tp];
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)p0);
          const bf16x4 hi =
              __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p0 + 4 * (BM + 8)));
          a[mi] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const __bf16* p0 = &Bs[(kk * 32 + 8 * g + tq) * (BN + 8) + wn + ni * 16 + 4 * tp];
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)p0);
          const bf16x4 hi =
              __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p0 + 4 * (BN + 8)));
          b[ni] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
    }
    if (do_cs) {
      if (TN) {
#pragma unroll 8
        for (int k = 0; k < BKK; ++k) cs += bf2f(Bs[k * (BN + 8) + t]);
      } else {
#pragma unroll 8
        for (int k = 0; k < BKK; ++k) cs += bf2f(Bs[t * (BKK + 8) + k]);
      }
    }
  };

  const int nk = kbeg < kend ? (kend - kbeg + BKK - 1) / BKK : 0;
  if (nk > 0) {
    load_tiles(kbeg);
    store_tiles(0);
    if (nk > 1) load_tiles(kbeg + BKK);
    __syncthreads();
    for (int it = 0; it < nk; ++it) {
      const int cur = it & 1;
      compute(cur);
      if (it + 1 < nk) {
        store_tiles(cur ^ 1);
        if (it + 2 < nk) load_tiles(kbeg + (it + 2) * BKK);
      }
      __syncthreads();
    }
  }
  if (do_cs && n0 + t < N) atomicAdd(colsum + n0 + t, cs);

  void* Cv = P.C[z];
  const float* bias = P.bias[z];
  const void* aux = P.aux[z];
  // bias and aux operands of the lane loaded up front from clamped indices,
  // unconditionally (see the Cin loads above)
  float bq[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
    bq[ni] = bias != nullptr ? bias[min(n0 + wn + ni * 16 + (lane & 15), N - 1)] : 0.0f;
  float xq[MI][NI][4];
  if constexpr (EPI == B_SOFTPLUS_BWD || EPI == B_SIGMOID_NOISE) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const size_t ao = (size_t)min(m0 + wm + mi * 16 + (lane >> 4) * 4 + r, M - 1) * D.ldaux +
                            min(n0 + wn + ni * 16 + (lane & 15), N - 1);
          xq[mi][ni][r] = EPI == B_SOFTPLUS_BWD ? bf2f(reinterpret_cast<const __bf16*>(aux)[ao])
                                                : reinterpret_cast<const float*>(aux)[ao];
        }
  }
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
        if (EPI == B_ATOMIC) {
          atomicAdd(reinterpret_cast<float*>(Cv) + o, v);
          continue;
        }
        // bf16 configuration: hardware transcendentals (v_exp/v_log, ~1 ulp);
        // the bit-exact spec functions are reserved for the fp32 parity path
        if (EPI == B_SOFTPLUS_BWD) {
          const float post = xq[mi][ni][r];
          // sigmoid(pre) = 1 - exp(-softplus(pre)); series for small post
          const float sg = post < 1e-3f ? post * (1.0f - 0.5f * post) : 1.0f - __expf(-post);
          v = v * sg;
        } else {
          if (bias != nullptr) v = v + bq[ni];
          if (EPI == B_SOFTPLUS) v = mog_softplus_hw(v);
          if (EPI == B_SIGMOID_NOISE) {
            const float y = __builtin_fmaf(xq[mi][ni][r], D.aux_scale, v);
            v = mog_sigmoid_hw(y);
          }
        }
        if (D.out_bf16) reinterpret_cast<__bf16*>(Cv)[o] = (__bf16)v;
        else reinterpret_cast<float*>(Cv)[o] = v;
      }
}

template <int BM, int BN, bool TN>
void launch(int epi, dim3 g, hipStream_t s, const BPtrs& P, const BDims& D) {
  switch (epi) {
    case B_STORE: gemm_bf16_kernel<BM, BN, TN, B_STORE><<<g, 256, 0, s>>>(P, D); break;
    case B_SOFTPLUS: gemm_bf16_kernel<BM, BN, TN, B_SOFTPLUS><<<g, 256, 0, s>>>(P, D); break;
    case B_SIGMOID_NOISE:
      gemm_bf16_kernel<BM, BN, TN, B_SIGMOID_NOISE><<<g, 256, 0, s>>>(P, D); break;
    case B_SOFTPLUS_BWD:
      gemm_bf16_kernel<BM, BN, TN, B_SOFTPLUS_BWD><<<g, 256, 0, s>>>(P, D); break;
    case B_ATOMIC: gemm_bf16_kernel<BM, BN, TN, B_ATOMIC><<<g, 256, 0, s>>>(P, D); break;
  }
}

template <int BM, int BN>
void launch_tile(bool tn, int epi, hipStream_t s, const BPtrs& P, BDims D, int batch) {
  int kchunk = (D.K + D.splitk - 1) / D.splitk;
  kchunk = ((kchunk + BKK - 1) / BKK) * BKK;
  if (kchunk == 0) kchunk = BKK;
  D.kchunk = kchunk;
  D.splitk = (D.K + kchunk - 1) / kchunk;
  if (D.splitk < 1) D.splitk = 1;
  D.nx = mog_cdiv(D.N, BN);
  D.ny = mog_cdiv(D.M, BM);
  dim3 g(D.nx, D.ny, batch * D.splitk);
  if (tn) launch<BM, BN, true>(epi, g, s, P, D);
  else launch<BM, BN, false>(epi, g, s, P, D);
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int mog_gemm_bf16(int batch, const void* const* A, const void* const* B,
                             void* const* C, const float* const* bias, const float* const* Cin,
                             const void* const* aux, float* const* colsum, int M, int N, int K,
                             int lda, int ldb, int ldc, int ldaux, int tn, int epi, int out_bf16,
                             float aux_scale, int splitk, void* stream) {
  MOG_CHECK_ARG(batch >= 1 && batch <= MAXB);
  MOG_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && splitk >= 1);
  MOG_CHECK_ARG(epi >= B_STORE && epi <= B_ATOMIC);
  MOG_CHECK_ARG(splitk == 1 || epi == B_ATOMIC);
  MOG_CHECK_ARG(colsum == nullptr || epi == B_ATOMIC);
  MOG_CHECK_ARG(epi != B_ATOMIC || !out_bf16);
  MOG_CHECK_ARG(lda % 8 == 0 && ldb % 8 == 0);  // 16-byte rows (zero-padded buffers)
  MOG_CHECK_ARG(tn || K % 8 == 0);
  MOG_CHECK_ARG(C && A && B);
  if (M == 0 || N == 0) return 0;
  BPtrs P;
  for (int i = 0; i < MAXB; ++i) {
    const bool on = i < batch;
    P.A[i] = on ? reinterpret_cast<const __bf16*>(A[i]) : nullptr;
    P.B[i] = on ? reinterpret_cast<const __bf16*>(B[i]) : nullptr;
    P.C[i] = on ? C[i] : nullptr;
    P.bias[i] = (on && bias) ? bias[i] : nullptr;
    P.Cin[i] = (on && Cin) ? Cin[i] : nullptr;
    P.aux[i] = (on && aux) ? aux[i] : nullptr;
    P.colsum[i] = (on && colsum) ? colsum[i] : nullptr;
    if (on) {
      MOG_CHECK_ARG(P.A[i] && P.B[i] && P.C[i] && al16(P.A[i]) && al16(P.B[i]));
      if (epi == B_SIGMOID_NOISE || epi == B_SOFTPLUS_BWD) MOG_CHECK_ARG(P.aux[i] != nullptr);
    }
  }
  BDims D;
  D.M = M; D.N = N; D.K = K; D.lda = lda; D.ldb = ldb; D.ldc = ldc; D.ldaux = ldaux;
  D.splitk = splitk; D.kchunk = 0; D.out_bf16 = out_bf16; D.aux_scale = aux_scale;
  D.nx = D.ny = 1;
  hipStream_t s = mog_stream(stream);
  // 128x128 only when it still gives >= 2 workgroups per CU (2 x 256 CUs);
  // MOG_BF16_BIG_NT / MOG_BF16_BIG_TN (profiling build) override the threshold
  const long big = (long)mog_cdiv(M, 128) * mog_cdiv(N, 128) * batch * splitk;
  long thr = 512;
  if (const char* e = mog_prof_env(tn ? "MOG_BF16_BIG_TN" : "MOG_BF16_BIG_NT")) thr = atol(e);
  if (M >= 128 && N >= 128 && big >= thr)
    launch_tile<128, 128>(tn != 0, epi, s, P, D, batch);
  else
    launch_tile<64, 64>(tn != 0, epi, s, P, D, batch);
  MOG_LAUNCH_RET();
}

// ---------------------------------------------------------------------------
// fp32 -> bf16 conversion with optional transpose and zero padding:
// dst[r][c] (ld_dst) = src[c][r] (transpose) or src[r][c]; rows x cols is the
// destination extent, (src_rows, src_cols) the valid source extent.
namespace {
__global__ __launch_bounds__(256) void cvt_bf16_kernel(const float* src, int src_rows,
                                                       int src_cols, int ld_src, __bf16* dst,
                                                       int rows, int cols, int ld_dst,
                                                       int transpose) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)rows * cols) return;
  const int r = i / cols, c = i - (long)r * cols;
  const int sr = transpose ? c : r, sc = transpose ? r : c;
  const float v = (sr < src_rows && sc < src_cols) ? src[(size_t)sr * ld_src + sc] : 0.0f;
  dst[(size_t)r * ld_dst + c] = (__bf16)v;
}

// Up to 16 conversions in one launch (the bf16 weight packs of all VAE
// layers after an optimizer step): job j covers elements [start[j], start[j+1]).
constexpr int CVT_MAX = 16;
struct CvtBatch {
  const float* src[CVT_MAX];
  __bf16* dst[CVT_MAX];
  int d[CVT_MAX][7];  // src_rows, src_cols, ld_src, rows, cols, ld_dst, transpose
  int count[CVT_MAX];  // rows * cols of each job (< 2^31)
  int n;
};

// One grid row (blockIdx.y) per job, 32-bit index arithmetic throughout (every
// pack is far below 2^31 elements; 64-bit divisions per element cost more than
// the copy itself).
__global__ __launch_bounds__(256) void cvt_bf16_batch_kernel(CvtBatch b) {
  const int j = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= b.count[j]) return;
  const int* d = b.d[j];
  const float* src = b.src[j];
  if (d[6] == 2) {
    // MFMA B-fragment order of W^T (vae_step.hip), k-step major: element
    // e = ((ks * NCT + ct) * 64 + lane) * 8 + q holds
    // W^T[ct*16 + lane%16][ks*32 + 8*(lane/16) + q], so one 16-B-per-lane wave
    // load is 1 KiB contiguous and the column tiles of one k-step are adjacent
    const int q = e & 7, l = (e >> 3) & 63;
    const int f = e >> 9;                        // ks * NCT + ct
    const int NCT = d[3] >> 4;
    const int ks = f / NCT, ct = f - ks * NCT;
    const int n = ct * 16 + (l & 15), k = ks * 32 + 8 * (l >> 4) + q;
    const float v = (k < d[0] && n < d[1]) ? src[k * d[2] + n] : 0.0f;
    b.dst[j][e] = (__bf16)v;
    return;
  }
  if (d[6] == 0 && (d[4] & 7) == 0 && (d[5] & 7) == 0) {
    // plain copy, 8 consecutive destination columns per thread (one 16-byte
    // store; two 16-byte loads where the source row is aligned and in range)
    const int e8 = e * 8;
    if (e8 >= b.count[j]) return;
    const int r = e8 / d[4], c = e8 - r * d[4];
    typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
    bf16x8_t o;
    const float* sp = src + r * d[2] + c;
    if (r < d[0] && c + 8 <= d[1] && ((d[2] & 3) == 0) && ((reinterpret_cast<size_t>(src) & 15) == 0)) {
      const float4 a0 = reinterpret_cast<const float4*>(sp)[0];
      const float4 a1 = reinterpret_cast<const float4*>(sp)[1];
      o[0] = (__bf16)a0.x; o[1] = (__bf16)a0.y; o[2] = (__bf16)a0.z; o[3] = (__bf16)a0.w;
      o[4] = (__bf16)a1.x; o[5] = (__bf16)a1.y; o[6] = (__bf16)a1.z; o[7] = (__bf16)a1.w;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = (__bf16)((r < d[0] && c + q < d[1]) ? sp[q] : 0.0f);
    }
    *reinterpret_cast<bf16x8_t*>(b.dst[j] + r * d[5] + c) = o;
    return;
  }
  const int r = e / d[4], c = e - r * d[4];
  const int sr = d[6] ? c : r, sc = d[6] ? r : c;
  const float v = (sr < d[0] && sc < d[1]) ? src[sr * d[2] + sc] : 0.0f;
  b.dst[j][r * d[5] + c] = (__bf16)v;
}
}  // namespace

extern "C" int mog_cvt_bf16_batch(int njobs, const float* const* src, void* const* dst,
                                  const int* dims, void* stream) {
  MOG_CHECK_ARG(njobs >= 0 && njobs <= CVT_MAX && (njobs == 0 || (src && dst && dims)));
  CvtBatch b;
  b.n = njobs;
  long mx = 0;
  for (int j = 0; j < njobs; ++j) {
    MOG_CHECK_ARG(src[j] && dst[j] && dims[7 * j + 3] >= 0 && dims[7 * j + 4] >= 0);
    const long cnt = (long)dims[7 * j + 3] * dims[7 * j + 4];
    const long lds = (long)dims[7 * j + 5] * (dims[7 * j + 6] == 2 ? 1 : dims[7 * j + 3]);
    const long lsrc = (long)dims[7 * j + 0] * dims[7 * j + 2];
    MOG_CHECK_ARG(cnt < (1L << 31) && lds < (1L << 31) && lsrc < (1L << 31));
    b.src[j] = src[j];
    b.dst[j] = reinterpret_cast<__bf16*>(dst[j]);
    for (int k = 0; k < 7; ++k) b.d[j][k] = dims[7 * j + k];
    b.count[j] = (int)cnt;
    // threads: one per element, or one per 8 for the vectorized plain copy
    const bool v8 = dims[7 * j + 6] == 0 && (dims[7 * j + 4] & 7) == 0 && (dims[7 * j + 5] & 7) == 0;
    const long thr = v8 ? (cnt + 7) / 8 : cnt;
    mx = thr > mx ? thr : mx;
  }
  if (njobs == 0 || mx == 0) return 0;
  cvt_bf16_batch_kernel<<<dim3(mog_cdiv(mx, 256), njobs), 256, 0, mog_stream(stream)>>>(b);
  MOG_LAUNCH_RET();
}

extern "C" int mog_cvt_bf16(const float* src, int src_rows, int src_cols, int ld_src, void* dst,
                            int rows, int cols, int ld_dst, int transpose, void* stream) {
  MOG_CHECK_ARG(src && dst && rows >= 0 && cols >= 0);
  if (rows == 0 || cols == 0) return 0;
  cvt_bf16_kernel<<<mog_cdiv((long)rows * cols, 256), 256, 0, mog_stream(stream)>>>(
      src, src_rows, src_cols, ld_src, reinterpret_cast<__bf16*>(dst), rows, cols, ld_dst,
      transpose);
  MOG_LAUNCH_RET();
}
