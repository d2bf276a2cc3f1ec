// Weight-stream microbenchmark for the fused step kernel's dense layers: how
// fast can one CU pull a 2.2 MB bf16 weight set (the VAE's, L2-resident,
// re-read by every CU) into its waves?  Each wave streams 1-KiB MFMA
// B-fragments (buffer_load_b128 per lane, the vae_step.hip pattern) through a
// register ring of depth D, consuming each with MFMAs on LDS-resident A.
// Variants: waves per CU (8 / 16), ring depth, and an LDS-DMA ring filled by
// loader waves.  Prints GB/s per CU (bytes of fragments consumed / kernel time).
// Build: hipcc -O3 --offload-arch=gfx950 -o wstream scripts/wstream_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int NFRAG = 2240;  // 2.24 MB of 1-KiB fragments

// each wave: fragments f = (w + nw * i + rot) % NFRAG, i < PER (PER fragments per wave)
template <int D, int MT>
__global__ void stream_regs(const __bf16* W, float* out, int per, int passes, int lock = 0) {
  __shared__ __bf16 A[MT * 16 * 40];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  for (int i = threadIdx.x; i < MT * 16 * 40; i += blockDim.x) A[i] = (__bf16)(0.001f * (i & 7));
  __syncthreads();
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(W), 0, NFRAG * 1024, 0x00020000);
  // lock: every CU streams the same fragment sequence at the same time (the
  // fused step kernel's lockstep layers: fragment i*nw + w at step i)
  const int rot = lock ? 0 : (blockIdx.x * 37) % NFRAG;
  floatx4 acc[MT];
  for (int m = 0; m < MT; ++m) acc[m] = floatx4{0, 0, 0, 0};
  bf16x8 a[MT];
  for (int m = 0; m < MT; ++m) a[m] = *reinterpret_cast<const bf16x8*>(&A[(m * 16 + li) * 40 + 8 * g]);
  for (int ps = 0; ps < passes; ++ps) {
    auto off = [&](int i) {
      return (((w + nw * i + rot + (lock ? 0 : ps * 97)) % NFRAG) * 64 + lane) * 16;
    };
    bf16x8 q[D];
#pragma unroll
    for (int d = 0; d < D; ++d)
      q[d] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off(d), 0, 0));
#pragma unroll 1
    for (int i = 0; i < per; i += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], q[d], acc[m], 0, 0, 0);
        q[d] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off(i + d + D), 0, 0));
      }
    }
  }
  float s = 0;
  for (int m = 0; m < MT; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3];
  if (s == 12345.0f) out[blockIdx.x] = s;
}

// LDS-DMA ring: loader waves (the first NL) fill slots of SLOT fragments,
// consumer waves read B-fragments from LDS; slot hand-off by s_barrier.
template <int NL, int SLOTS, int SLOT, int MT>
__global__ void stream_lds(const __bf16* W, float* out, int nslab, int passes) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char ring[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(W), 0, NFRAG * 1024, 0x00020000);
  const int rot = (blockIdx.x * 37) % NFRAG;
  floatx4 acc[MT];
  for (int m = 0; m < MT; ++m) acc[m] = floatx4{0, 0, 0, 0};
  bf16x8 a[MT];
  for (int m = 0; m < MT; ++m) a[m] = bf16x8{};
  const int nc = nw;  // every wave consumes its share of each slot
  auto issue = [&](int s) {
    // SLOT fragments per slab, loader wave l issues fragments l, l+NL, ...
    if (w < NL)
      for (int f = w; f < SLOT; f += NL) {
        const int fr = (s * SLOT + f + rot) % NFRAG;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)(ring + ((s % SLOTS) * SLOT + f) * 1024), 16,
            (fr * 64 + lane) * 16, 0, 0, 0);
      }
  };
  for (int ps = 0; ps < passes; ++ps) {
    for (int s = 0; s < SLOTS - 1; ++s) issue(s);
    for (int s = 0; s < nslab; ++s) {
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((SLOT / NL) * (SLOTS - 2)) : "memory");
      if (s + SLOTS - 1 < nslab) issue(s + SLOTS - 1);
      const unsigned char* sl = ring + (s % SLOTS) * SLOT * 1024;
      for (int f = w; f < SLOT; f += nc) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(sl + f * 1024 + lane * 16);
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], b, acc[m], 0, 0, 0);
      }
    }
  }
  float s = 0;
  for (int m = 0; m < MT; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3];
  if (s == 12345.0f) out[blockIdx.x] = s;
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  f();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  int ncu = 256;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  __bf16* W;
  float* out;
  hipMalloc(&W, NFRAG * 1024);
  hipMalloc(&out, 4096 * 4);
  hipMemset(W, 0, NFRAG * 1024);
  // a 256 MB buffer streamed by a copy between reps would model the other
  // traffic; here: the weights alone (upper bound)
  const int grid = ncu;
  const int passes = 4;
  auto report = [&](const char* name, int waves, double frags_per_cu, float ms) {
    const double gbs = frags_per_cu * 1024.0 / (ms * 1e-3) / 1e9;
    printf("%-34s waves/CU %2d: %7.1f us  %6.1f GB/s per CU  (%.2f TB/s chip)\n", name, waves,
           ms * 1e3, gbs, gbs * ncu / 1000.0);
    fflush(stdout);
  };
#define RUN_REGS(D, MT, NW)                                                                  \
  {                                                                                          \
    const int per = NFRAG / NW;                                                              \
    float ms = timeit([&] { stream_regs<D, MT><<<grid, NW * 64>>>(W, out, per, passes); }, 10); \
    report("regs D=" #D " MT=" #MT, NW, (double)per * NW * passes, ms);                      \
  }
  RUN_REGS(2, 4, 8);
  RUN_REGS(4, 4, 8);
  RUN_REGS(8, 4, 8);
  RUN_REGS(16, 4, 8);
  RUN_REGS(2, 4, 16);
  RUN_REGS(4, 4, 16);
  RUN_REGS(8, 4, 16);
  RUN_REGS(16, 4, 16);
  RUN_REGS(8, 1, 16);
  RUN_REGS(8, 4, 4);
  RUN_REGS(16, 4, 4);
  {  // lockstep: every CU the same fragments in the same order
    const int per = NFRAG / 16;
    for (int D4 = 0; D4 < 2; ++D4) {
      float ms = timeit([&] {
        if (D4) stream_regs<4, 4><<<grid, 1024>>>(W, out, per, passes, 1);
        else stream_regs<4, 1><<<grid, 1024>>>(W, out, per, passes, 1);
      }, 10);
      report(D4 ? "regs D=4 MT=4 LOCKSTEP" : "regs D=4 MT=1 LOCKSTEP", 16, (double)per * 16 * passes, ms);
    }
  }
#define RUN_LDS(NL, SLOTS, SLOT, NW)                                                              \
  {                                                                                               \
    const int nslab = NFRAG / SLOT;                                                               \
    const size_t lds = (size_t)SLOTS * SLOT * 1024;                                               \
    float ms = timeit([&] { stream_lds<NL, SLOTS, SLOT, 4><<<grid, NW * 64, lds>>>(W, out, nslab, passes); }, 10); \
    report("ldsdma NL=" #NL " slots=" #SLOTS "x" #SLOT, NW, (double)nslab * SLOT * passes, ms); \
  }
  RUN_LDS(16, 4, 16, 16);
  RUN_LDS(16, 4, 32, 16);
  RUN_LDS(16, 3, 32, 16);
  RUN_LDS(8, 4, 32, 8);
  RUN_LDS(16, 6, 16, 16);
  RUN_LDS(4, 4, 32, 16);
  return 0;
}
