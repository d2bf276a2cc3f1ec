// Weight gradients of the narrow layers: C_b[M][N] += sum_k A_b[k][m] B_b[k][n]
// over the T*B rows, colsum_b[n] += sum_k B_b[k][n] (the bias gradient), for
// N <= 16 and long K -- the heads' 1- / 2-wide output layers (air_model.py:
// 462-499 backward).  mog_gemm_f32 routes its transA + EPI_ATOMIC launches of
// those shapes here (gemm_f32.hip's 64 x 64 LDS tiles spent 111 / 79 us on
// them at 24,576 rows: 64 x 1 outputs; this kernel 57 / 51 us with 512-row
// chunks, scripts/dw_small_bench.py).  Wider outputs stay on gemm_f32.hip:
// without LDS staging the per-lane 4-byte loads leave each chunk a chain of
// load latencies (M = 256 x N = 64: 302 us here against 66 us there).
//
// No LDS: v_mfma_f32_16x16x4_f32 takes one fp32 of A (row li, k g) and one of
// B (k g, column li) per lane, so each lane loads its operands straight from
// the k-major rows (16 consecutive floats per k-row and lane group: 64-byte
// segments).  Workgroup = 4 waves over a 64 x 64 output tile, wave w owns rows
// 16w .. 16w+15 and up to four 16-column tiles; the K range is cut into chunks
// (grid.y) whose partial sums meet in fp32 atomics -- a single chunk (K < 256,
// e.g. the reference's batch of 64) adds each output once to the zeroed
// gradient, so that case is deterministic.
#include <algorithm>

#include "mog_common.h"

namespace {

constexpr int MAXB = 8;

struct TnSmallArgs {
  const float* A[MAXB];
  const float* B[MAXB];
  float* C[MAXB];
  float* cs[MAXB];
  int M, N, K, lda, ldb, ldc, kchunk, mtiles;
};

__global__ __launch_bounds__(256) void gemm_tn_small_kernel(TnSmallArgs D) {
  const int tile = blockIdx.x, b = blockIdx.z;
  const int mt = tile % D.mtiles, nt0 = tile / D.mtiles;
  const int m0 = mt * 64, n0 = nt0 * 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int k0 = blockIdx.y * D.kchunk, k1 = min(D.K, k0 + D.kchunk);
  const float* __restrict__ A = D.A[b];
  const float* __restrict__ B = D.B[b];
  const int M = D.M, N = D.N, lda = D.lda, ldb = D.ldb;
  const int m = m0 + 16 * w + li;
  const int mc = m < M ? m : M - 1;  // clamped: loads stay in range, the row is masked
  const bool mv = m < M;
  const int nact = min(4, (N - n0 + 15) / 16);  // live column tiles (uniform)
  int nc[4];
  bool nv[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n = n0 + 16 * t + li;
    nv[t] = n < N;
    nc[t] = nv[t] ? n : N - 1;
  }
  const bool do_cs = D.cs[b] != nullptr && mt == 0 && w == 0;
  floatx4 acc[4];
  float cs[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    cs[t] = 0.f;
  }
  // 16 k-rows per iteration: four MFMA k-steps, every load issued first
  constexpr int KU = 4;
  for (int kb = k0; kb < k1; kb += 4 * KU) {
    float a[KU], bv[KU][4];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int k = kb + 4 * u + g;
      const bool kv = k < k1;
      const int kc = kv ? k : k1 - 1;
      const float av = A[(size_t)kc * lda + mc];
      a[u] = (kv && mv) ? av : 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < nact) {
          const float x = B[(size_t)kc * ldb + nc[t]];
          bv[u][t] = (kv && nv[t]) ? x : 0.f;
        } else {
          bv[u][t] = 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < KU; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < nact) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], bv[u][t], acc[t], 0, 0, 0);
    if (do_cs) {
#pragma unroll
      for (int u = 0; u < KU; ++u)
#pragma unroll
        for (int t = 0; t < 4; ++t) cs[t] += bv[u][t];
    }
  }
  // acc[t][r]: row 4g + r of the wave's 16, column li of tile t
  float* __restrict__ C = D.C[b];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t >= nact) break;
    const int col = n0 + 16 * t + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + 16 * w + 4 * g + r;
      if (row < M && col < N) atomicAdd(C + (size_t)row * D.ldc + col, acc[t][r]);
    }
  }
  if (do_cs) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float v = cs[t];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int col = n0 + 16 * t + li;
      if (g == 0 && t < nact && col < N) atomicAdd(D.cs[b] + col, v);
    }
  }
}

}  // namespace

// C_b += A_b^T B_b (k-major operands), colsum_b += column sums of B_b; see the
// header comment.  Called by mog_gemm_f32 (gemm_f32.hip).
int mog_internal_gemm_tn_small(int batch, const float* const* A, const float* const* B,
                               float* const* C, float* const* colsum, int M, int N, int K,
                               int lda, int ldb, int ldc, hipStream_t stream) {
  if (batch < 1 || batch > MAXB || M <= 0 || N <= 0 || K <= 0) return MOG_ERR_INVALID;
  TnSmallArgs D{};
  for (int i = 0; i < batch; ++i) {
    D.A[i] = A[i];
    D.B[i] = B[i];
    D.C[i] = C[i];
    D.cs[i] = colsum ? colsum[i] : nullptr;
  }
  D.M = M; D.N = N; D.K = K; D.lda = lda; D.ldb = ldb; D.ldc = ldc;
  D.mtiles = mog_cdiv(M, 64);
  const int tiles = D.mtiles * mog_cdiv(N, 64);
  // about 1024 workgroups (four per CU; each chunk is a chain of dependent
  // load rounds, so many short chunks), chunks of >= 128 rows; one chunk below
  // K = 256 (deterministic)
  int nsplit = mog_cdiv(1024, tiles * batch);
  nsplit = std::max(1, std::min(nsplit, K / 128));
  D.kchunk = ((mog_cdiv(K, nsplit) + 15) / 16) * 16;
  nsplit = mog_cdiv(K, D.kchunk);
  gemm_tn_small_kernel<<<dim3((unsigned)tiles, (unsigned)nsplit, (unsigned)batch), 256, 0, stream>>>(D);
  return (int)hipGetLastError();
}
