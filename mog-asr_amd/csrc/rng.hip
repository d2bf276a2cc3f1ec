// Counter-based noise for perf mode (replaces the reference's tf.random_normal /
// tf.random_uniform sites: air_model.py:191, vae.py:29,44, concrete.py:23).
// Philox4x32-10; each thread emits 4 values.  Parity tests inject noise
// tensors instead (TF's RNG stream is not reproducible; SURVEY.md §7 'RNG').
#include "philox.h"

namespace {

__global__ __launch_bounds__(256) void rng_kernel(float* out, long n, uint64_t seed,
                                                  uint64_t offset, int normal) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;  // quad index
  const long i0 = q * 4;
  if (i0 >= n) return;
  float v[4];
  mog_philox_quad(seed, offset + (uint64_t)q, normal != 0, v);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (i0 + k < n) out[i0 + k] = v[k];
}

// Up to 8 noise buffers in one launch (grid row j: buffer j, its own counter
// offset and normal / uniform choice): element i of buffer j is lane i % 4 of
// quad offset[j] + i / 4 -- bit-identical to mog_rng_fill per buffer.
constexpr int RNG_MAX = 8;
struct RngBatch {
  float* out[RNG_MAX];
  long n[RNG_MAX];
  uint64_t offset[RNG_MAX];
  int normal[RNG_MAX];
};
__global__ __launch_bounds__(256) void rng_batch_kernel(RngBatch b, uint64_t seed) {
  const int j = blockIdx.y;
  const long n = b.n[j];
  for (long q = (long)blockIdx.x * 256 + threadIdx.x; q * 4 < n; q += (long)gridDim.x * 256) {
    float v[4];
    mog_philox_quad(seed, b.offset[j] + (uint64_t)q, b.normal[j] != 0, v);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (q * 4 + k < n) b.out[j][q * 4 + k] = v[k];
  }
}

}  // namespace

extern "C" int mog_rng_fill_batch(int nbuf, float* const* out, const long* n, unsigned long long seed,
                                  const unsigned long long* offset, const int* normal, void* stream) {
  MOG_CHECK_ARG(nbuf >= 0 && nbuf <= RNG_MAX && (nbuf == 0 || (out && n && offset && normal)));
  RngBatch b;
  long mx = 0;
  for (int j = 0; j < RNG_MAX; ++j) {
    const bool on = j < nbuf;
    b.out[j] = on ? out[j] : nullptr;
    b.n[j] = on ? n[j] : 0;
    b.offset[j] = on ? offset[j] : 0;
    b.normal[j] = on ? normal[j] : 0;
    if (on) {
      MOG_CHECK_ARG(out[j] != nullptr && n[j] >= 0);
      mx = n[j] > mx ? n[j] : mx;
    }
  }
  if (nbuf == 0 || mx == 0) return 0;
  const long quads = (mx + 3) / 4;
  const long blocks = quads < 256L * 4096 ? (long)mog_cdiv(quads, 256) : 4096L;
  rng_batch_kernel<<<dim3((unsigned)blocks, nbuf), 256, 0, mog_stream(stream)>>>(b, seed);
  MOG_LAUNCH_RET();
}

extern "C" int mog_rng_fill(float* out, long n, unsigned long long seed,
                            unsigned long long offset, int normal, void* stream) {
  MOG_CHECK_ARG(out && n >= 0);
  if (n == 0) return 0;
  rng_kernel<<<mog_cdiv((n + 3) / 4, 256), 256, 0, mog_stream(stream)>>>(out, n, seed, offset,
                                                                        normal);
  MOG_LAUNCH_RET();
}
