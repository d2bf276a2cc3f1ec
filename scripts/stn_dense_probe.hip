// Measurement probe (not product code): the STN write backward's input gradient
// in DENSE form on the fp32 matrix cores, dU = W_y^T (s G) W_x per image, with
// W_x [50 x 28] / W_y [50 x 28] the banded bilinear weight matrices of the
// axis-aligned transform (transformer.py:102-116's gradient; the degenerate
// columns / rows of the product kernel are zero rows here).  One wave per
// image: G (the canvas gradient, 50 x 50) staged in LDS, T = (s G) W_x as
// 4 x 2 blocks of v_mfma_f32_16x16x4_f32 over K = 52 (104 MFMAs), T through
// LDS, dU = W_y^T T as 2 x 2 blocks (52 MFMAs); the W operands are formed in
// registers from the per-column / per-row geometry tables.  Measures what the
// dense form costs at the step's 24,576 images against the product kernel's
// whole write backward (dU + dtheta + dot), scripts/stn_dense_probe.py.
#include "../mog-asr_amd/csrc/stn_geom.h"

namespace {

constexpr int C = 50, W = 28, KP = 52, GP = 52;  // canvas, glimpse, padded K, G pitch
constexpr int WAVE_F = C * GP + KP * 32;          // floats per wave: G | T

__global__ __launch_bounds__(256, 2) void dense_du_kernel(const float* __restrict__ G,
                                                          int g_period,
                                                          const float* __restrict__ theta,
                                                          const float* __restrict__ gscale,
                                                          float* __restrict__ dU, int N) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float smem[4 * WAVE_F];
  __shared__ float4 geo[4][2][64];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n = blockIdx.x * 4 + wv;
  if (n >= N) return;
  float th[6];
#pragma unroll
  for (int k = 0; k < 6; ++k)
    th[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(theta[n * 6 + k])));
  const float sc = gscale[n];
  float* sg = smem + wv * WAVE_F;
  float* sT = sg + C * GP;
  const float* Gn = G + (size_t)(n % g_period) * C * C;
  for (int e = lane; e < C * C; e += 64) sg[(e / C) * GP + e % C] = Gn[e] * sc;
  if (lane < C) {
    geo[wv][0][lane] = axis4(axis_col(th, W, W, C, C, lane), 1);
    geo[wv][1][lane] = axis4(axis_row(th, W, W, C, C, lane), 1);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int li = lane & 15, g = lane >> 4;
  // weight of source index s in the bilinear pair of entry e (0 when degenerate)
  auto wsel = [](float4 e, int s) {
    const int lo = __float_as_int(e.x), hi = __float_as_int(e.y);
    if (lo == hi) return 0.0f;
    return (s == lo ? e.z : 0.0f) + (s == hi ? e.w : 0.0f);
  };
  floatx4 t[4][2];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) t[mi][ni] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < KP / 4; ++ks) {
    const int j = 4 * ks + g;  // canvas column = k
    const float4 cg = geo[wv][0][min(j, C - 1)];
    float b[2];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) b[ni] = j < C ? wsel(cg, 16 * ni + li) : 0.0f;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int i = 16 * mi + li;
      const float a = (i < C && j < C) ? sg[i * GP + j] : 0.0f;
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        t[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[ni], t[mi][ni], 0, 0, 0);
    }
  }
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * mi + 4 * g + r;
        if (i < KP) sT[i * 32 + 16 * ni + li] = t[mi][ni][r];
      }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  floatx4 d[2][2];
#pragma unroll
  for (int vi = 0; vi < 2; ++vi)
#pragma unroll
    for (int ui = 0; ui < 2; ++ui) d[vi][ui] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < KP / 4; ++ks) {
    const int i = 4 * ks + g;  // canvas row = k
    const float4 rg = geo[wv][1][min(i, C - 1)];
    float bt[2];
#pragma unroll
    for (int ui = 0; ui < 2; ++ui) bt[ui] = sT[i * 32 + 16 * ui + li];
#pragma unroll
    for (int vi = 0; vi < 2; ++vi) {
      const float a = i < C ? wsel(rg, 16 * vi + li) : 0.0f;
#pragma unroll
      for (int ui = 0; ui < 2; ++ui)
        d[vi][ui] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bt[ui], d[vi][ui], 0, 0, 0);
    }
  }
  float* out = dU + (size_t)n * W * W;
#pragma unroll
  for (int vi = 0; vi < 2; ++vi)
#pragma unroll
    for (int ui = 0; ui < 2; ++ui)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int v = 16 * vi + 4 * g + r, u = 16 * ui + li;
        if (v < W && u < W) out[v * W + u] = d[vi][ui][r];
      }
}

}  // namespace

extern "C" int stn_dense_du(const float* G, int g_period, const float* theta, const float* gscale,
                            float* dU, int N, void* stream) {
  if (N <= 0) return 0;
  dense_du_kernel<<<dim3((unsigned)((N + 3) / 4)), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      G, g_period, theta, gscale, dU, N);
  return (int)hipGetLastError();
}
