// Fused multi-tensor gradient processing + TF-1.12 Adam (air/air_model.py:941-999).
//
// Per tensor (the reference loops over variables, :963-972):
//   g = where(isinf(g), 0, g); g = where(isnan(g), 0, g)
//   g = clip_by_norm(g, clip) = (g * clip) / max(||g||_2, clip)
// then ApplyAdam (epsilon outside the bias correction, TF training_ops):
//   m += (g - m) * (1 - b1);  v += (g*g - v) * (1 - b2)
//   var -= (m * lr_t) / (sqrt(v) + eps),  lr_t = lr sqrt(1 - b2^t) / (1 - b1^t)
// Two launches: (1) sanitize + each block's sum of squares of its chunk,
// (2) clip + Adam, every block forming its tensor's squared norm from the
// tensor's chunk sums in chunk order -- no atomics, so the norm, the clip and
// the update are the same bits on every run (and in a replayed graph).
// The tensor table maps a block to (tensor, chunk) so one launch covers all
// ~36 parameter tensors of the flat parameter buffer.
#include "mog_common.h"

namespace {

constexpr int CHUNK = 4096;  // elements per block

__global__ __launch_bounds__(256) void sanitize_sumsq_kernel(float* g, const long* off,
                                                            const long* len,
                                                            const int* block_tensor,
                                                            const long* block_start,
                                                            float* part) {
  __shared__ float red[4];
  const int ti = block_tensor[blockIdx.x];
  const long base = off[ti], n = len[ti];
  const long c0 = block_start[blockIdx.x];
  const long c1 = min(n, c0 + CHUNK);
  // 16-byte accesses (tensors start 256-B aligned, chunks at multiples of
  // CHUNK elements); the ragged end of a tensor element by element
  const long v1 = c0 + ((c1 - c0) & ~3L);
  float s = 0.0f;
  for (long i = c0 + 4 * threadIdx.x; i < v1; i += 1024) {
    float4 v = *reinterpret_cast<const float4*>(g + base + i);
    float e[4] = {v.x, v.y, v.z, v.w};
    bool bad = false;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (isinf(e[k]) || isnan(e[k])) {
        e[k] = 0.0f;
        bad = true;
      }
    if (bad) *reinterpret_cast<float4*>(g + base + i) = make_float4(e[0], e[1], e[2], e[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k) s += e[k] * e[k];
  }
  for (long i = v1 + threadIdx.x; i < c1; i += 256) {
    float v = g[base + i];
    if (isinf(v) || isnan(v)) {
      v = 0.0f;
      g[base + i] = 0.0f;
    }
    s += v * v;
  }
  s = mog_block_sum256(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void clip_adam_kernel(float* p, const float* g, float* m,
                                                       float* v, const long* off, const long* len,
                                                       const int* block_tensor,
                                                       const long* block_start,
                                                       const float* part, float clip,
                                                       float lr_t, float b1, float b2,
                                                       float eps) {
#pragma clang fp contract(off)
  __shared__ float red[4];
  const int ti = block_tensor[blockIdx.x];
  const long base = off[ti], n = len[ti];
  const long c0 = block_start[blockIdx.x];
  const long c1 = min(n, c0 + CHUNK);
  // part == nullptr: gradient_clipping_norm=None -- no sanitize, no clip
  // (air_model.py:948 skips both), plain ApplyAdam
  const bool clipped = part != nullptr;
  float l2 = 0.0f;
  if (clipped) {
    // the tensor's chunk sums: blocks first .. first + nc - 1, summed in a
    // fixed order (per thread strided, then the block tree)
    const int first = blockIdx.x - (int)(c0 / CHUNK);
    const int nc = (int)((n + CHUNK - 1) / CHUNK);
    float s = 0.0f;
    for (int j = threadIdx.x; j < nc; j += 256) s += part[first + j];
    l2 = mog_block_sum256(s, red);
  }
  const float norm = l2 > 0.0f ? sqrtf(l2) : l2;
  const float denom = fmaxf(norm, clip);
  auto upd = [&](float gk, float& mm, float& vv, float& pp) {
    const float gc = clipped ? (gk * clip) / denom : gk;
    mm = mm + (gc - mm) * (1.0f - b1);
    vv = vv + (gc * gc - vv) * (1.0f - b2);
    pp = pp - (mm * lr_t) / (sqrtf(vv) + eps);
  };
  const long v1 = c0 + ((c1 - c0) & ~3L);
  for (long i = c0 + 4 * threadIdx.x; i < v1; i += 1024) {  // 16-byte accesses
    const long k = base + i;
    const float4 g4 = *reinterpret_cast<const float4*>(g + k);
    float4 m4 = *reinterpret_cast<const float4*>(m + k);
    float4 v4 = *reinterpret_cast<const float4*>(v + k);
    float4 p4 = *reinterpret_cast<const float4*>(p + k);
    upd(g4.x, m4.x, v4.x, p4.x);
    upd(g4.y, m4.y, v4.y, p4.y);
    upd(g4.z, m4.z, v4.z, p4.z);
    upd(g4.w, m4.w, v4.w, p4.w);
    *reinterpret_cast<float4*>(m + k) = m4;
    *reinterpret_cast<float4*>(v + k) = v4;
    *reinterpret_cast<float4*>(p + k) = p4;
  }
  for (long i = v1 + threadIdx.x; i < c1; i += 256) {
    const long k = base + i;
    float mm = m[k], vv = v[k], pp = p[k];
    upd(g[k], mm, vv, pp);
    m[k] = mm;
    v[k] = vv;
    p[k] = pp;
  }
}

}  // namespace

extern "C" int mog_optim_chunk_elems(void) { return CHUNK; }

// `sumsq`: scratch of nblocks floats (per-chunk sums of squares); a null
// `sumsq` skips the NaN/Inf zeroing and the clip (gradient_clipping_norm=None).
extern "C" int mog_clip_adam(float* params, float* grads, float* m, float* v, const long* off,
                             const long* len, const int* block_tensor, const long* block_start,
                             int nblocks, float* sumsq, float clip, float lr_t, float beta1,
                             float beta2, float eps, void* stream) {
  MOG_CHECK_ARG(params && grads && m && v && off && len && block_tensor && block_start);
  MOG_CHECK_ARG(nblocks >= 0);
  // 16-byte vector accesses: the flat buffers 16-byte aligned (and every
  // tensor offset a multiple of 4 elements: the parameter store aligns them to 64)
  for (const void* q : {(const void*)params, (const void*)grads, (const void*)m, (const void*)v})
    MOG_CHECK_ARG((reinterpret_cast<uintptr_t>(q) & 15) == 0);
  if (nblocks == 0) return 0;
  hipStream_t s = mog_stream(stream);
  if (sumsq != nullptr)
    sanitize_sumsq_kernel<<<nblocks, 256, 0, s>>>(grads, off, len, block_tensor, block_start,
                                                  sumsq);
  clip_adam_kernel<<<nblocks, 256, 0, s>>>(params, grads, m, v, off, len, block_tensor,
                                           block_start, sumsq, clip, lr_t, beta1, beta2, eps);
  MOG_LAUNCH_RET();
}
