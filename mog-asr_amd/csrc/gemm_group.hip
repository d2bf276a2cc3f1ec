// Grouped fp32 weight gradients: C_p[M_p][N_p] += A_p^T B_p over K_p rows for
// every problem p of a host table, ONE launch (the weight gradients of a
// small-batch train step: at the reference's batch of 64 each of them is a
// K = 64..192 product, so each separate launch was a few k-steps of work
// behind a launch latency).  Optional column sums of B_p (the
// bias gradients).  Every output element has one writer (no split-K), so the
// result is deterministic and C += acc is a plain read-add-write.
//
// The problems travel BY VALUE in the kernel argument (up to WG_MAX per launch:
// no device table to upload, so a captured graph holds the launch as one node
// with its arguments); problem p owns workgroups base[p] .. base[p+1] - 1,
// ceil(M/64) x ceil(N/64) output tiles.
//
// 64 x 64 x 16 tiles, four waves of 32 x 32 on v_mfma_f32_16x16x4_f32 (k of
// MFMA kk from lane group g: k0 + 4 kk + g, the k-ordered chain of
// gemm_f32.hip), operand k-tiles register-prefetched one ahead and staged in
// LDS rows padded to 80 floats (the four k-rows one MFMA operand read touches
// start 16 banks apart).
#include "mog_common.h"

namespace {

constexpr int WG_MAX = 24;
constexpr int GB = 64, GK = 16, GLD = 80;

struct WgProblem {
  const float* A;
  const float* B;
  float* C;
  float* colsum;
  int M, N, K, lda, ldb, ldc;
};
struct WgGroup {
  WgProblem p[WG_MAX];
  int base[WG_MAX + 1];
  int n;
};

__global__ __launch_bounds__(256) void wgrad_group_kernel(const WgGroup G) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float sA[2][GK * GLD];
  __shared__ __attribute__((aligned(16))) float sB[2][GK * GLD];
  const int wg = blockIdx.x;
  int p = 0;
  for (int q = 1; q < G.n; ++q) {
    if (G.base[q] <= wg) p = q;
    else break;
  }
  const WgProblem& e = G.p[p];
  const float* A = e.A;
  const float* B = e.B;
  float* C = e.C;
  float* colsum = e.colsum;
  const int M = e.M, N = e.N, K = e.K, lda = e.lda, ldb = e.ldb, ldc = e.ldc;
  const int tn = (N + GB - 1) / GB, local = wg - G.base[p];
  const int m0 = (local / tn) * GB, n0 = (local % tn) * GB;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
  const int li = lane & 15, g = lane >> 4;
  // staging: thread t holds k-row t / 16, columns 4 (t % 16) .. + 3 of each operand
  const int sr = t >> 4, sc = (t & 15) * 4;
  float ra[4], rb[4];
  auto load = [&](int k0) {
    const int k = k0 + sr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + sc + i, n = n0 + sc + i;
      ra[i] = (k < K && m < M) ? A[(size_t)k * lda + m] : 0.0f;
      rb[i] = (k < K && n < N) ? B[(size_t)k * ldb + n] : 0.0f;
    }
  };
  auto store = [&](int s) {
    *reinterpret_cast<float4*>(&sA[s][sr * GLD + sc]) = make_float4(ra[0], ra[1], ra[2], ra[3]);
    *reinterpret_cast<float4*>(&sB[s][sr * GLD + sc]) = make_float4(rb[0], rb[1], rb[2], rb[3]);
  };
  floatx4 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = floatx4{0.f, 0.f, 0.f, 0.f};
  const bool do_cs = colsum != nullptr && m0 == 0 && t < GB;
  float cs = 0.0f;
  const int nk = (K + GK - 1) / GK;
  if (nk > 0) {
    load(0);
    store(0);
  }
  for (int it = 0; it < nk; ++it) {
    const int s = it & 1;
    if (it + 1 < nk) load((it + 1) * GK);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK / 4; ++kk) {
      const float* a = &sA[s][(4 * kk + g) * GLD];
      const float* b = &sB[s][(4 * kk + g) * GLD];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[wm + 16 * mi + li], b[wn + 16 * ni + li],
                                                             acc[mi][ni], 0, 0, 0);
    }
    if (do_cs) {
#pragma unroll
      for (int k = 0; k < GK; ++k) cs += sB[s][k * GLD + t];
    }
    if (it + 1 < nk) store(s ^ 1);
  }
  if (do_cs && n0 + t < N) colsum[n0 + t] += cs;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * mi + 4 * g + r, n = n0 + wn + 16 * ni + li;
        if (m < M && n < N) C[(size_t)m * ldc + n] += acc[mi][ni][r];
      }
}

}  // namespace

extern "C" int mog_gemm_f32_wgrad_group(const long long* table, int nprob, void* stream) {
  MOG_CHECK_ARG(nprob >= 0 && (nprob == 0 || table));
  for (int i = 0; i < nprob; ++i) {
    const long long* r = table + 10 * i;
    MOG_CHECK_ARG(r[0] && r[1] && r[2] && r[4] >= 0 && r[5] >= 0 && r[6] >= 0);
    MOG_CHECK_ARG(r[4] < (1 << 24) && r[5] < (1 << 24) && r[6] < (1 << 24));
    MOG_CHECK_ARG(r[7] >= r[4] && r[8] >= r[5] && r[9] >= r[5]);
  }
  for (int i0 = 0; i0 < nprob; i0 += WG_MAX) {
    WgGroup G{};
    int tiles = 0;
    G.n = 0;
    for (int i = i0; i < nprob && i < i0 + WG_MAX; ++i) {
      const long long* r = table + 10 * i;
      if (r[4] == 0 || r[5] == 0) continue;
      WgProblem& q = G.p[G.n];
      q.A = reinterpret_cast<const float*>(r[0]);
      q.B = reinterpret_cast<const float*>(r[1]);
      q.C = reinterpret_cast<float*>(r[2]);
      q.colsum = reinterpret_cast<float*>(r[3]);
      q.M = (int)r[4]; q.N = (int)r[5]; q.K = (int)r[6];
      q.lda = (int)r[7]; q.ldb = (int)r[8]; q.ldc = (int)r[9];
      G.base[G.n] = tiles;
      tiles += (int)(mog_cdiv(q.M, GB) * mog_cdiv(q.N, GB));
      ++G.n;
    }
    G.base[G.n] = tiles;
    if (tiles == 0) continue;
    wgrad_group_kernel<<<dim3((unsigned)tiles), 256, 0, mog_stream(stream)>>>(G);
    const hipError_t rc = hipGetLastError();
    if (rc != hipSuccess) return (int)rc;
  }
  return 0;
}
