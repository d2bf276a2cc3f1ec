// Grouped tall-K weight gradients on the gfx950 bf16 matrix cores:
//   out_i[M_i][N_i] += X_i^T dY_i  over K batch rows,  colsum_i[N_i] += sum_k dY_i[k][:]
// for up to eight problems in ONE launch (the seven VAE layers of the bf16
// configuration: the MatMul / BiasAdd gradients of air/vae.py:18-46 over all
// T*B rows).  Shapes: K = T*B = 24,576, M, N = 50..784 -- a few hundred
// output tiles against a K that is 100x the output edge, so the kernel is
// built around K:
//   * the K rows are cut into nsplit splits; split s runs on XCD s % 8 (the
//     hardware deals workgroup b to XCD b % 8), so every tile of a k-range
//     streams the same X / dY rows through ONE XCD's L2 (each row of X is
//     read by N/128 tiles, each row of dY by M/128);
//   * each split's 128 x 128 partial tile goes to a workspace and a second
//     launch adds the splits into out in split order: deterministic, no
//     float atomics (round 5's split-K atomics wrote 30x the output);
//   * operand k-tiles go global -> LDS by buffer_load_dwordx4 ... lds (LDS-DMA),
//     NS stages deep, so 2 k-tiles per workgroup stay in flight without
//     registers; three workgroups per CU;
//   * fragments come out of the k-major images with the transpose read
//     ds_read_b64_tr_b16; rows of the image are XOR-swizzled in 16-byte
//     chunks (cdna_hip_programming.md T10 (b)) so the reads are conflict-free;
//   * the bias gradient (column sums of dY) is one more MFMA per column block
//     with a ones A-fragment, on the workgroups of the first row of tiles:
//     exact products, fp32 sums, and deterministic like the rest.
// Columns past M / N load neighbouring data (rows past the k-range load 0
// through the buffer range check); they reach only tile rows / columns that
// the reduction never stores.
//
// The fp32 form (wgrad_tn_x3_kernel: the fp32 configuration's VAE weight
// gradients at fp32-level accuracy) is the same grouped, XCD-split,
// workspace-reduced GEMM with gemm_x3.hip's exact three-piece operand splits:
// fp32 k-tiles staged through registers, split as they are written into six
// bf16 images (A0 A1 A2 B0 B1 B2, the same swizzled layout), six MFMA
// products per 16x16x32 block; the column sums take the ones-MFMA of each B
// piece (b = b0 + b1 + b2 exactly).
#include "mog_common.h"
#include "x3_split.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int WT = 128;               // output tile edge
constexpr int BK = 32;                // k-rows per LDS stage
constexpr int IMG = BK * WT;          // bf16 elements of one operand image (8 KB)
constexpr int STAGE = 2 * IMG;        // A then B
constexpr int NS = 3;                 // LDS stages (48 KB: three workgroups per CU)
constexpr int MAXP = 8;
constexpr int TILE_F = WT * WT;       // floats of one partial tile
constexpr int OOB = (int)0x80000000u; // a buffer offset past every range

struct WgProblem {
  const void* X;     // [K][lda] bf16 (wgrad_tn_bf16_kernel) or fp32 (wgrad_tn_x3_kernel)
  const void* dY;    // [K][ldb]
  float* out;        // [M][ldc]
  float* colsum;     // [N] or null
  int M, N, lda, ldb, ldc;
  int tx, tile0;     // column tiles; first tile of the problem in the group
};

struct WgArgs {
  WgProblem p[MAXP];
  int np, T, K, kchunk, nsplit, xcd_map;
  float* work;       // [nsplit][T][WT][WT] partial tiles, then [nsplit][T][WT] column sums
};

// Loader forms: 0 LDS-DMA (the product form: 104 vs 115 us for the seven
// VAE layers at 24,576 rows, scripts/wgmodes.sh); 2 register staging
// (buffer_load_dwordx4 -> ds_write_b128, two LDS stages; profiling build,
// MOG_WG_MODE=2).  Both fill the same XOR-swizzled image.
// 16-byte chunk swizzle of k-row r of a 256-byte-row image (guide T10 (b))
template <int MODE>
__device__ __forceinline__ int swz(int r) {
  return ((r & 3) << 2) | ((r >> 2) & 3);
}
// bf16 index of (k-row r, column c), c a multiple of 4
template <int MODE>
__device__ __forceinline__ int tpos(int r, int c) {
  return r * WT + ((((c >> 3) ^ swz<MODE>(r)) << 3) | (c & 4));
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// the problem owning `tile`: a select chain over constant indices (a
// dynamically indexed kernel-argument array is copied to scratch first)
__device__ __forceinline__ WgProblem find_problem(const WgArgs& D, int tile) {
  WgProblem P = D.p[0];
#pragma unroll
  for (int i = 1; i < MAXP; ++i)
    if (i < D.np && tile >= D.p[i].tile0) P = D.p[i];
  return P;
}

__device__ __forceinline__ float wt_dpp1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float wt_dpp2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}
// 4 x 4 transpose inside lane quads: row g*4 + r of column li in, row
// g*4 + (li & 3) at columns (li & ~3) + r out (as gemm_x3.hip)
__device__ __forceinline__ floatx4 quad_transpose(const floatx4& a, int lane) {
  const int e = lane & 3;
  float r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3];
  {
    const bool hi = (e & 2) != 0;
    const float t0 = wt_dpp2(hi ? r0 : r2), t1 = wt_dpp2(hi ? r1 : r3);
    if (hi) { r0 = t0; r1 = t1; } else { r2 = t0; r3 = t1; }
  }
  {
    const bool od = (e & 1) != 0;
    const float t0 = wt_dpp1(od ? r0 : r1), t1 = wt_dpp1(od ? r2 : r3);
    if (od) { r0 = t0; r2 = t1; } else { r1 = t0; r3 = t1; }
  }
  return floatx4{r0, r1, r2, r3};
}

// workgroup b -> split s (on XCD s % 8 when nsplit is a multiple of 8) and tile
__device__ __forceinline__ void block_job(const WgArgs& D, int b, int& s, int& tile) {
  if ((D.nsplit & 7) == 0 && D.xcd_map) {
    const int x = b & 7, j = b >> 3;
    s = x + 8 * (j / D.T);
    tile = j % D.T;
  } else {
    s = b / D.T;
    tile = b % D.T;
  }
}

// this split's 128 x 128 partial tile into the workspace: lane quads
// transposed so a lane stores four consecutive columns of one row (16-byte
// stores); the column-sum partials (first row of tiles) after the tiles
__device__ __forceinline__ void store_partial(const WgArgs& D, const floatx4 (&acc)[4][4],
                                              const floatx4 (&csa)[2], bool do_cs, int s,
                                              int tile, int wm, int wn, int cni, int lane) {
  const int g = lane >> 4, li = lane & 15;
  float* W = D.work + ((size_t)s * D.T + tile) * TILE_F;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const floatx4 v = quad_transpose(acc[mi][ni], lane);
      const int row = wm + mi * 16 + 4 * g + (li & 3);
      const int col = wn + ni * 16 + (li & ~3);
      *reinterpret_cast<floatx4*>(W + row * WT + col) = v;
    }
  if (do_cs && g == 0) {
    float* Wc = D.work + (size_t)D.nsplit * D.T * TILE_F + ((size_t)s * D.T + tile) * WT;
    Wc[wn + cni * 16 + li] = csa[0][0];
    Wc[wn + (cni + 1) * 16 + li] = csa[1][0];
  }
}

template <int MODE>
__global__ __launch_bounds__(256, 3) void wgrad_tn_bf16_kernel(WgArgs D) {
  __shared__ __attribute__((aligned(1024))) __bf16 lds[NS * STAGE];
  int s, tile;
  block_job(D, blockIdx.x, s, tile);
  const WgProblem P = find_problem(D, tile);
  const int lt = tile - P.tile0;
  const int by = lt / P.tx, bx = lt - by * P.tx;
  const int m0 = by * WT, n0 = bx * WT;
  const int kbeg = s * D.kchunk;
  const int kend = min(D.K, kbeg + D.kchunk);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const bool do_cs = P.colsum != nullptr && by == 0;

  // operand descriptors over whole rows: [K][ld] bf16
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(P.X), 0, (int)((long)D.K * P.lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(P.dY), 0, (int)((long)D.K * P.ldb * 2), 0x00020000);
  // DMA roles: wave w fills 1-KiB blocks q = w and w + 4 of each image (k-rows
  // 4q .. 4q+3); lane l -> k-row 4q + l/16, LDS chunk l%16 = global chunk
  // (l%16) ^ swz(row)
  int aoff[2], boff[2], krow[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = w + 4 * j;
    const int r = 4 * q + (lane >> 4);
    const int c = (lane & 15) ^ swz<MODE>(r);
    krow[j] = r;
    aoff[j] = (r * P.lda + m0 + 8 * c) * 2;
    boff[j] = (r * P.ldb + n0 + 8 * c) * 2;
  }
  const int nk = kbeg < kend ? (kend - kbeg + BK - 1) / BK : 0;
  // byte advance of one k-tile in each operand, and this lane's offsets at
  // the workgroup's first k-row (scalars / registers fixed before the loop)
  const int astep = BK * P.lda * 2, bstep = BK * P.ldb * 2;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    aoff[j] += kbeg * P.lda * 2;
    boff[j] += kbeg * P.ldb * 2;
    krow[j] += kbeg;
  }
  auto issue = [&](int it, int stage) {
    __bf16* img = lds + stage * STAGE;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = w + 4 * j;
      const bool in = krow[j] + it * BK < kend;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ra, (__attribute__((address_space(3))) void*)(img + q * 512), 16,
          in ? aoff[j] + it * astep : OOB, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (__attribute__((address_space(3))) void*)(img + IMG + q * 512), 16,
          in ? boff[j] + it * bstep : OOB, 0, 0, 0);
    }
  };
  constexpr int DPT = 4;  // DMA instructions per wave per stage

  floatx4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = floatx4{0.f, 0.f, 0.f, 0.f};
  floatx4 csa[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
  const int cni = 2 * (w >> 1);  // the two column blocks whose sums this wave takes
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

  // transposed-read roles: lane 4q+p of a 16-lane group -> k-row 8g + q (+4),
  // columns 4p .. 4p+3 of the block
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  int ao[4][2], bo[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ao[i][0] = tpos<MODE>(8 * g + tq, wm + 16 * i + 4 * tp);
    ao[i][1] = tpos<MODE>(8 * g + tq + 4, wm + 16 * i + 4 * tp);
    bo[i][0] = tpos<MODE>(8 * g + tq, wn + 16 * i + 4 * tp);
    bo[i][1] = tpos<MODE>(8 * g + tq + 4, wn + 16 * i + 4 * tp);
  }
  // fragment reads in inline asm: the compiler's wait insertion does not
  // see them, so it does not drain the LDS-DMAs in flight before every read
  // (it cannot tell the stages of the one LDS array apart); the lgkmcnt wait
  // below ties the fragments to the MFMAs that use them
  auto frag = [&](unsigned base, const int (&o)[2]) -> bf16x8 {
    bf16x4 lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(base + 2u * o[0]));
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(base + 2u * o[1]));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  const unsigned lds_base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds;

  bf16x8 bf[4], af[4];
  auto frags = [&](int stage) {
    const unsigned A = lds_base + 2u * (unsigned)(stage * STAGE), B = A + 2u * IMG;
#pragma unroll
    for (int i = 0; i < 4; ++i) bf[i] = frag(B, bo[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(A, ao[i]);
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(bf[0]), "+v"(bf[1]), "+v"(bf[2]), "+v"(bf[3]), "+v"(af[0]), "+v"(af[1]),
                   "+v"(af[2]), "+v"(af[3]));
  };
  auto mfmas = [&]() {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
    if (do_cs) {
      // whole-vector selects on the wave-uniform half (an array index would
      // be lowered as a select over every 16-bit element)
      const bool hi = cni != 0;
      csa[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, hi ? bf[2] : bf[0], csa[0], 0, 0, 0);
      csa[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, hi ? bf[3] : bf[1], csa[1], 0, 0, 0);
    }
  };

  if constexpr (MODE == 2) {
    // register staging: chunk i of thread t is the DMA lane's chunk (block
    // q = w + 4 i, lane l), stored lane-linearly, so the image is the same
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 ra4[2], rb4[2];
    auto load = [&](int it) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool in = krow[j] + it * BK < kend;
        ra4[j] = __builtin_amdgcn_raw_buffer_load_b128(ra, in ? aoff[j] + it * astep : OOB, 0, 0);
        rb4[j] = __builtin_amdgcn_raw_buffer_load_b128(rb, in ? boff[j] + it * bstep : OOB, 0, 0);
      }
    };
    auto store = [&](int stage) {
      __bf16* img = lds + stage * STAGE;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q = w + 4 * j;
        *reinterpret_cast<u32x4*>(img + q * 512 + lane * 8) = ra4[j];
        *reinterpret_cast<u32x4*>(img + IMG + q * 512 + lane * 8) = rb4[j];
      }
    };
    if (nk > 0) {
      load(0);
      store(0);
      if (nk > 1) load(1);
      __syncthreads();
    }
    for (int it = 0; it < nk; ++it) {
      const int cur = it & 1;
      frags(cur);
      if (it + 1 < nk) {
        store(cur ^ 1);
        if (it + 2 < nk) load(it + 2);
      }
      mfmas();
      __syncthreads();
    }
  } else {
#pragma unroll
    for (int j = 0; j < NS - 1; ++j)
      if (j < nk) issue(j, j);
    int st = 0;
    for (int it = 0; it < nk; ++it) {
      // this wave's DMAs of tile it have landed (NS-2 later tiles stay in
      // flight), then every wave's; every wave is done reading the stage the
      // next DMA overwrites (tile it-1's)
      if (it + NS - 2 < nk) wait_vm<DPT * (NS - 2)>();
      else wait_vm<0>();
      asm volatile("s_barrier" ::: "memory");
      frags(st);
      // the next DMA after this wave's fragment reads have landed
      if (it + NS - 1 < nk) issue(it + NS - 1, st == 0 ? NS - 1 : st - 1);
      mfmas();
      st = st == NS - 1 ? 0 : st + 1;
    }
  }

  store_partial(D, acc, csa, do_cs, s, tile, wm, wn, cni, lane);
}

__global__ __launch_bounds__(256, 2) void wgrad_tn_x3_kernel(WgArgs D) {
  // one stage of six images (48 KB: two workgroups per CU overlap each
  // other's split and MFMA phases, as gemm_x3.hip's TN form)
  __shared__ __attribute__((aligned(1024))) __bf16 lds[6 * IMG];
  int s, tile;
  block_job(D, blockIdx.x, s, tile);
  const WgProblem P = find_problem(D, tile);
  const int lt = tile - P.tile0;
  const int by = lt / P.tx, bx = lt - by * P.tx;
  const int m0 = by * WT, n0 = bx * WT;
  const int kbeg = s * D.kchunk;
  const int kend = min(D.K, kbeg + D.kchunk);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const bool do_cs = P.colsum != nullptr && by == 0;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(P.X), 0, (int)((long)D.K * P.lda * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(P.dY), 0, (int)((long)D.K * P.ldb * 4), 0x00020000);
  // staging roles: float4 i of this thread is k-row t/32 + 8 i, columns
  // 4 (t % 32) .. + 3 of the tile
  const int sr = t >> 5, sc = (t & 31) * 4;
  int aoff[4], boff[4], krow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    krow[i] = kbeg + sr + 8 * i;
    aoff[i] = (krow[i] * P.lda + m0 + sc) * 4;
    boff[i] = (krow[i] * P.ldb + n0 + sc) * 4;
  }
  const int astep = BK * P.lda * 4, bstep = BK * P.ldb * 4;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 ra4[4], rb4[4];
  // operands whose row pitch is not a multiple of 4 floats (the 50-wide
  // latent layers) load each 16-byte chunk as two 8-byte halves
  const bool pitch8 = ((P.lda | P.ldb) & 3) != 0;
  auto ld16 = [&](__amdgpu_buffer_rsrc_t r, int off) -> u32x4 {
    if (!pitch8) return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    const u32x2 lo = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    const u32x2 hi = __builtin_amdgcn_raw_buffer_load_b64(r, off == OOB ? OOB : off + 8, 0, 0);
    return u32x4{lo[0], lo[1], hi[0], hi[1]};
  };
  auto load = [&](int it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool in = krow[i] + it * BK < kend;
      ra4[i] = ld16(ra, in ? aoff[i] + it * astep : OOB);
      rb4[i] = ld16(rb, in ? boff[i] + it * bstep : OOB);
    }
  };
  auto f4 = [](const u32x4& v) {
    return float4{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                  __uint_as_float(v[3])};
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = tpos<0>(sr + 8 * i, sc);
      u32x2 p0, p1, p2;
      split4(f4(ra4[i]), p0, p1, p2);
      *reinterpret_cast<u32x2*>(lds + 0 * IMG + o) = p0;
      *reinterpret_cast<u32x2*>(lds + 1 * IMG + o) = p1;
      *reinterpret_cast<u32x2*>(lds + 2 * IMG + o) = p2;
      split4(f4(rb4[i]), p0, p1, p2);
      *reinterpret_cast<u32x2*>(lds + 3 * IMG + o) = p0;
      *reinterpret_cast<u32x2*>(lds + 4 * IMG + o) = p1;
      *reinterpret_cast<u32x2*>(lds + 5 * IMG + o) = p2;
    }
  };

  floatx4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = floatx4{0.f, 0.f, 0.f, 0.f};
  floatx4 csa[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
  const int cni = 2 * (w >> 1);
  const bool chi = cni != 0;
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  int ao[4][2], bo[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ao[i][0] = tpos<0>(8 * g + tq, wm + 16 * i + 4 * tp);
    ao[i][1] = tpos<0>(8 * g + tq + 4, wm + 16 * i + 4 * tp);
    bo[i][0] = tpos<0>(8 * g + tq, wn + 16 * i + 4 * tp);
    bo[i][1] = tpos<0>(8 * g + tq + 4, wn + 16 * i + 4 * tp);
  }
  auto frag = [&](int img, const int (&o)[2]) -> bf16x8 {
    const __bf16* base = lds + img * IMG;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base + o[0]));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(base + o[1]));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto compute = [&]() {
    // the B pieces held for the k-tile, the A pieces one at a time, smallest
    // products first (a2 b0; a1 b1, a1 b0; a0 b2, a0 b1, a0 b0)
    bf16x8 b[3][4];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i) b[p][i] = frag(3 + p, bo[i]);
#pragma unroll
    for (int pa = 2; pa >= 0; --pa) {
      bf16x8 a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag(pa, ao[i]);
#pragma unroll
      for (int pb = 2 - pa; pb >= 0; --pb)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            acc[mi][ni] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mi], b[pb][ni], acc[mi][ni], 0, 0, 0);
    }
    if (do_cs) {
#pragma unroll
      for (int p = 2; p >= 0; --p) {
        csa[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, chi ? b[p][2] : b[p][0], csa[0], 0, 0, 0);
        csa[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, chi ? b[p][3] : b[p][1], csa[1], 0, 0, 0);
      }
    }
  };
  const int nk = kbeg < kend ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) load(0);
  for (int it = 0; it < nk; ++it) {
    store();
    if (it + 1 < nk) load(it + 1);
    __syncthreads();
    compute();
    __syncthreads();
  }
  store_partial(D, acc, csa, do_cs, s, tile, wm, wn, cni, lane);
}

// out += sum over splits s = 0 .. nsplit-1 of the partial tiles, in that order;
// thread q: tile q / 4096, row (q / 32) % 128, columns 4 (q % 32) ..; then one
// thread per (tile, column) for the column sums (first row of tiles only)
__global__ __launch_bounds__(256) void wgrad_tn_reduce_kernel(WgArgs D) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  const long nq = (long)D.T * (TILE_F / 4);
  if (q < nq) {
    const int tile = (int)(q >> 12), r = (int)(q >> 5) & 127, c = (int)(q & 31) * 4;
    const WgProblem P = find_problem(D, tile);
    const int lt = tile - P.tile0;
    const int by = lt / P.tx, bx = lt - by * P.tx;
    const int m = by * WT + r, n = bx * WT + c;
    if (m >= P.M || n >= P.N) return;
    const float* W = D.work + (size_t)tile * TILE_F + r * WT + c;
    floatx4 v = *reinterpret_cast<const floatx4*>(W);
    for (int s = 1; s < D.nsplit; ++s) {
      const floatx4 u = __builtin_nontemporal_load(
          reinterpret_cast<const floatx4*>(W + (size_t)s * D.T * TILE_F));
      v += u;
    }
    float* o = P.out + (size_t)m * P.ldc + n;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (n + e < P.N) o[e] += v[e];
    return;
  }
  const long qc = q - nq;
  if (qc >= (long)D.T * WT) return;
  const int tile = (int)(qc >> 7), c = (int)(qc & 127);
  const WgProblem P = find_problem(D, tile);
  const int lt = tile - P.tile0;
  const int by = lt / P.tx, bx = lt - by * P.tx;
  const int n = bx * WT + c;
  if (P.colsum == nullptr || by != 0 || n >= P.N) return;
  const float* Wc = D.work + (size_t)D.nsplit * D.T * TILE_F + (size_t)tile * WT + c;
  float v = Wc[0];
  for (int s = 1; s < D.nsplit; ++s) v += Wc[(size_t)s * D.T * WT];
  P.colsum[n] += v;
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int group_tiles(int nprob, const int* dims) {
  int T = 0;
  for (int i = 0; i < nprob; ++i) T += (int)mog_cdiv(dims[5 * i], WT) * (int)mog_cdiv(dims[5 * i + 1], WT);
  return T;
}

}  // namespace

extern "C" long mog_wgrad_tn_work_elems(int nprob, const int* dims, int nsplit) {
  if (nprob < 1 || nprob > MAXP || !dims || nsplit < 1) return -1;
  return (long)nsplit * group_tiles(nprob, dims) * (TILE_F + WT);
}

namespace {

// the launch of either form: elem = 2 (bf16 operands) or 4 (fp32, the x3
// form); whole rows inside the 32-bit buffer range
int wgrad_tn_launch(int elem, int nprob, const void* const* X, const void* const* dY,
                    float* const* out, float* const* colsum, const int* dims, int K, int nsplit,
                    float* work, long work_elems, void* stream) {
  MOG_CHECK_ARG(nprob >= 1 && nprob <= MAXP && X && dY && out && dims && K >= 0 && nsplit >= 1);
  MOG_CHECK_ARG(work != nullptr && al16(work) &&
                work_elems >= mog_wgrad_tn_work_elems(nprob, dims, nsplit));
  // bf16: 16-byte rows (pitches multiples of 8); fp32: 8-byte rows
  // (pitches even: the x3 kernel loads 16-byte chunks as two halves when a
  // pitch is not a multiple of 4)
  const int vec = elem == 2 ? 8 : 2;
  WgArgs D{};
  D.np = nprob;
  D.K = K;
  int T = 0;
  for (int i = 0; i < nprob; ++i) {
    const int M = dims[5 * i], N = dims[5 * i + 1], lda = dims[5 * i + 2], ldb = dims[5 * i + 3],
              ldc = dims[5 * i + 4];
    MOG_CHECK_ARG(M >= 1 && N >= 1 && lda >= M && ldb >= N && ldc >= N && lda % vec == 0 &&
                  ldb % vec == 0);
    MOG_CHECK_ARG((long)K * lda * elem < (1L << 31) && (long)K * ldb * elem < (1L << 31));
    MOG_CHECK_ARG(X[i] && dY[i] && out[i] && al16(X[i]) && al16(dY[i]));
    WgProblem& P = D.p[i];
    P.X = X[i];
    P.dY = dY[i];
    P.out = out[i];
    P.colsum = colsum ? colsum[i] : nullptr;
    P.M = M; P.N = N; P.lda = lda; P.ldb = ldb; P.ldc = ldc;
    P.tx = (int)mog_cdiv(N, WT);
    P.tile0 = T;
    T += P.tx * (int)mog_cdiv(M, WT);
  }
  D.T = T;
  int kchunk = (K + nsplit - 1) / nsplit;
  kchunk = ((kchunk + BK - 1) / BK) * BK;
  if (kchunk == 0) kchunk = BK;
  D.kchunk = kchunk;
  D.nsplit = nsplit;
  D.work = work;
  D.xcd_map = 1;
  if (const char* e = mog_prof_env("MOG_WG_MAP")) D.xcd_map = atoi(e);
  if (K == 0) return 0;
  hipStream_t s = mog_stream(stream);
  const dim3 grid((unsigned)(T * nsplit));
  if (elem == 4) {
    wgrad_tn_x3_kernel<<<grid, 256, 0, s>>>(D);
  } else {
    int mode = 0;
    if (const char* e = mog_prof_env("MOG_WG_MODE")) mode = atoi(e);
    if (mode == 2) wgrad_tn_bf16_kernel<2><<<grid, 256, 0, s>>>(D);
    else wgrad_tn_bf16_kernel<0><<<grid, 256, 0, s>>>(D);
  }
  const long nthr = (long)T * (TILE_F / 4) + (long)T * WT;
  wgrad_tn_reduce_kernel<<<dim3((unsigned)((nthr + 255) / 256)), 256, 0, s>>>(D);
  MOG_LAUNCH_RET();
}

}  // namespace

extern "C" int mog_wgrad_tn_bf16(int nprob, const void* const* X, const void* const* dY,
                                 float* const* out, float* const* colsum, const int* dims, int K,
                                 int nsplit, float* work, long work_elems, void* stream) {
  return wgrad_tn_launch(2, nprob, X, dY, out, colsum, dims, K, nsplit, work, work_elems, stream);
}

extern "C" int mog_wgrad_tn_x3(int nprob, const float* const* X, const float* const* dY,
                               float* const* out, float* const* colsum, const int* dims, int K,
                               int nsplit, float* work, long work_elems, void* stream) {
  return wgrad_tn_launch(4, nprob, reinterpret_cast<const void* const*>(X),
                         reinterpret_cast<const void* const*>(dY), out, colsum, dims, K, nsplit,
                         work, work_elems, stream);
}
