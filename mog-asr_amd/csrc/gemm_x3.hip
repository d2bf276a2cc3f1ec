// fp32 weight gradient on the bf16 matrix cores: C[M][N] += sum_k A[k][m] B[k][n]
// (both operands fp32, k-major: dW = X^T dY over the batch rows), split-K, optional
// column sums of B (the bias gradient).  Split-K partials (and the column sums'
// per-split partials) go to a workspace and a second launch adds them into C
// (and the column sums) in split order (deterministic; the float
// atomics it replaces measured equal at 3 splits and 71.6 vs 87.7 us at 8 on
// the bf16 x-rows gradient, scripts/x1_sweep.py); one split adds C += acc with
// plain loads and stores.
//
// Every fp32 operand is split EXACTLY into three bf16 pieces by truncation,
// x = x0 + x1 + x2 (x0 = the top 8 significand bits, x1 the next 8 of x - x0,
// x2 = the rest, which has at most 8 significant bits), so
//   a b = sum_{i+j<=2} a_i b_j  +  (a1 b2 + a2 b1 + a2 b2)
// and the six kept products carry every term down to 2^-16 of a b; the dropped
// three are below 2^-23 of it -- the size of the rounding of one fp32 product.
// bf16 x bf16 products are exact in the MFMA's fp32 accumulator, so the result
// differs from an fp32 fma chain by summation order only (a gradient, gated by
// tolerance like every split-K/atomic gradient; the forward layers keep the
// bit-exact fp32 kernels of gemm_f32.hip).  Six v_mfma_f32_16x16x32_bf16 per
// 16x16x32 block against eight v_mfma_f32_16x16x4_f32: 96 vs 256 MFMA cycles.
//
// Tile 128 x 128 x 32, four waves of 64 x 64.  Each k-tile is loaded as fp32
// float4 rows (k-major, coalesced), split in registers and stored as three
// k-major bf16 LDS images per operand; fragments come out with the gfx950
// transpose read ds_read_b64_tr_b16 (as the TN form of gemm_bf16.hip).  One
// LDS stage, register prefetch of the next k-tile, two workgroups per CU.
//
// Three forms (measured on MI355X, scripts/x3_lib_bench.py, us; fp32-level
// accuracy gated in tests/test_gpu_x3.py):
//   * gemm_x3_tn_kernel<false>: the split inside the GEMM (7 VALU per
//     element, every workgroup of a row panel re-splits its A tile) -- the
//     fp32 VAE weight gradients (AIRModel._dw_x3): 239 us at 784 x 512 x 24,576
//     rows against 166 us pre-split;
//   * gemm_x3_tn_kernel<true>: operands split once by mog_split3_bf16 -- the
//     LSTM x-rows gradient X^T dG (AIR and ASR, the default MOG_X_GRAD_X3=2):
//     251 us at 2500 x 1024 x 8192 (343 us split in-kernel);
//   * gemm_x3_nt_kernel (below): dX = dY W^T, dY split in-kernel, W split once
//     per optimizer step -- the fp32 VAE input-gradient chain: 161 / 184 us at
//     24,576 x 512 x 784 / 24,576 x 784 x 512 (hipBLASLt fp32 176 / 222 us).
// MFMA is under half busy in every form (0.26-0.45 of the bf16 peak).  The
// kernel moves ~9 TB/s of operand tiles from L2 / Infinity Cache into LDS in
// both the one- and three-piece forms (663 MB / 72 us, 1.99 GB / 224 us at
// 2500 x 1024 x 8192: 128 x 128 tiles re-read A 8x and B 20x), so its time
// follows the bytes its tiles re-read, not the MFMA count.  An LDS-DMA
// multi-stage form of the pre-split kernel (buffer_load ... lds, 2-4 stages,
// 128 x 128 and 256 x 128 tiles, bank-swizzled transposed reads) measured no
// faster: 70-95 us one-piece, 237-340 us three-piece (round 5, git history).
#include <cstdlib>
#include <type_traits>

#include "mog_common.h"
#include "x3_split.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 32;
constexpr int LDR = BM;                     // LDS row (k) pitch in bf16 (BM == BN), unpadded:
// the 8-byte units (4 bf16) of k-row r sit at unit u ^ tsw(r), so the 16 rows x
// 32 B that one ds_read_b64_tr_b16 touches (rows 8g + tq [+ 4], four units per
// row) cover the 64 banks once (a padded pitch of 136 left them 2-way
// conflicted: SQ_LDS_BANK_CONFLICT a third of the LDS cycles)
constexpr int PIECE = BK * LDR;             // one bf16 image
constexpr int STAGE = 6 * PIECE;            // A0 A1 A2 B0 B1 B2
constexpr int NL = (BM * BK / 4) / 256;     // float4 loads per thread per operand (4)

// bijective XCD-grouping remap of the linear workgroup id (as gemm_bf16.hip)
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

__device__ __forceinline__ int tsw(int r) { return ((r & 3) << 2) | (((r >> 3) & 1) << 4); }
// bf16 offset of (k-row r, column c), c a multiple of 4, in a TN operand image
__device__ __forceinline__ int tpos(int r, int c) { return r * LDR + (((c >> 2) ^ tsw(r)) << 2); }

struct X3Args {
  const float* A;
  const float* B;
  const __bf16* A3;  // PRE: the pieces split beforehand (mog_split3_bf16), piece p
  const __bf16* B3;  // at A3 + p * sa (B3 + p * sb)
  long sa, sb;
  float* C;
  float* colsum;
  float* work;  // split-K partials [nsplit][M][N] (summed into C by splitk_reduce_kernel), or null
  int M, N, K, lda, ldb, ldc, kchunk, nx, ny, nsplit;
};

// the accumulator tile of one wave (4 x 4 blocks of 16 x 16, lane (g, li) holds
// rows 4 g .. 4 g + 3 of column li of each) into C: one split -> C += acc (a
// plain read-add-write: no other workgroup touches these elements); split-K
// with a workspace -> stored as this split's partial; else float atomics
__device__ __forceinline__ void x3_epilogue(const X3Args& D, const floatx4 (&acc)[4][4], int r0,
                                            int c0, int ks, int lane) {
  const int g = lane >> 4, li = lane & 15;
  const int mode = D.nsplit == 1 ? 0 : D.work != nullptr ? 1 : 2;
  float* W = D.work + (size_t)ks * D.M * D.N;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + mi * 16 + g * 4 + r;
        const int col = c0 + ni * 16 + li;
        if (row < D.M && col < D.N) {
          if (mode == 0) D.C[(size_t)row * D.ldc + col] += acc[mi][ni][r];
          else if (mode == 1) W[(size_t)row * D.N + col] = acc[mi][ni][r];
          else atomicAdd(D.C + (size_t)row * D.ldc + col, acc[mi][ni][r]);
        }
      }
}

constexpr int NP = (BM * BK / 8) / 256;  // 16-byte bf16 chunks per thread per piece (2)

__device__ __forceinline__ float bf_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

// NPC: pieces per operand (3; 1 = plain bf16 operands, one product)
template <bool PRE, int NPC = 3>
__global__ __launch_bounds__(256, 2) void gemm_x3_tn_kernel(X3Args D) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[STAGE];

  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int bx = wg % D.nx, by = (wg / D.nx) % D.ny, ks = wg / (D.nx * D.ny);
  const int m0 = by * BM, n0 = bx * BN;
  const int kbeg = ks * D.kchunk;
  const int kend = min(D.K, kbeg + D.kchunk);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const int M = D.M, N = D.N;
  // staging roles: float4 i of this thread covers k-row t/32 + 8 i, columns 4 (t % 32) ..
  const int sk = t >> 5, sc = (t & 31) * 4;
  const bool do_cs = D.colsum != nullptr && by == 0;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  // PRE staging roles: 16-byte chunk i covers k-row t/16 + 16 i, columns 8 (t % 16) ..
  const int pk = t >> 4, pc = (t & 15) * 8;
  float cs8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  u32x4 pa[3][NP], pb[3][NP];

  floatx4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = floatx4{0.f, 0.f, 0.f, 0.f};

  // Operand loads through buffer descriptors, unconditional: rows past the
  // K chunk get an offset past every range (they load 0; a predicated load
  // compiled to a branch per load, and the generic-pointer form to FLAT loads,
  // which also count in lgkmcnt -- so the barrier's lgkmcnt(0) waited for the
  // next k-tile's prefetch every iteration).  Columns >= M / N load a
  // neighbour's data (or 0 past the buffer): they reach only rows / columns of
  // C that are not stored, and column sums that are not stored.  Kept as raw
  // dwords until the split (a conversion at the load makes the compiler copy
  // the registers there, which waits for the load).
  u32x4 ra[NL], rb[NL];
  constexpr int OOB = (int)0x80000000u;
  // record ranges = the operands' validated extents (each piece's last k-row
  // ends at column round8(M) / round8(N)): nothing past them is read.  PRE:
  // one descriptor per piece, so the range check (which covers the per-lane
  // offset only, not the scalar one) holds every piece to its own extent.
  __amdgpu_buffer_rsrc_t arsc[PRE ? NPC : 1], brsc[PRE ? NPC : 1];
#pragma unroll
  for (int p = 0; p < (PRE ? NPC : 1); ++p) {
    arsc[p] = __builtin_amdgcn_make_buffer_rsrc(
        PRE ? (void*)(D.A3 + p * D.sa) : (void*)D.A, 0,
        PRE ? (int)(((long)(D.K - 1) * D.lda + ((M + 7) & ~7)) * 2)
            : (int)(((long)(D.K - 1) * D.lda + M) * 4),
        0x00020000);
    brsc[p] = __builtin_amdgcn_make_buffer_rsrc(
        PRE ? (void*)(D.B3 + p * D.sb) : (void*)D.B, 0,
        PRE ? (int)(((long)(D.K - 1) * D.ldb + ((N + 7) & ~7)) * 2)
            : (int)(((long)(D.K - 1) * D.ldb + N) * 4),
        0x00020000);
  }
  auto load_tiles = [&](int k0) {
    if constexpr (PRE) {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int gk = k0 + pk + 16 * i;
        // gm < lda, multiples of 8: a chunk starting in the row stays in it
        const int ao = gk < kend ? (gk * D.lda + m0 + pc) * 2 : OOB;
        const int bo = gk < kend ? (gk * D.ldb + n0 + pc) * 2 : OOB;
#pragma unroll
        for (int p = 0; p < NPC; ++p) {
          pa[p][i] = __builtin_amdgcn_raw_buffer_load_b128(arsc[p], ao, 0, 0);
          pb[p][i] = __builtin_amdgcn_raw_buffer_load_b128(brsc[p], bo, 0, 0);
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int gk = k0 + sk + 8 * i;
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(
          arsc[0], gk < kend ? (gk * D.lda + m0 + sc) * 4 : OOB, 0, 0);
      rb[i] = __builtin_amdgcn_raw_buffer_load_b128(
          brsc[0], gk < kend ? (gk * D.ldb + n0 + sc) * 4 : OOB, 0, 0);
    }
  };
  auto f4 = [](const u32x4& v) {
    return float4{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                  __uint_as_float(v[3])};
  };
  auto store_tiles = [&](int stage) {
    __bf16* S = lds + stage * STAGE;
    if constexpr (PRE) {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int o = tpos(pk + 16 * i, pc);
#pragma unroll
        for (int p = 0; p < NPC; ++p) {
          *reinterpret_cast<u32x4*>(S + p * PIECE + o) = pa[p][i];
          *reinterpret_cast<u32x4*>(S + (3 + p) * PIECE + o) = pb[p][i];
        }
        if (do_cs && NPC == 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            cs8[2 * j] += bf_lo(pb[0][i][j]);
            cs8[2 * j + 1] += bf_hi(pb[0][i][j]);
          }
        } else if (do_cs) {  // x = x0 + x1 + x2 exactly
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            cs8[2 * j] += (bf_lo(pb[0][i][j]) + bf_lo(pb[1][i][j])) + bf_lo(pb[2][i][j]);
            cs8[2 * j + 1] += (bf_hi(pb[0][i][j]) + bf_hi(pb[1][i][j])) + bf_hi(pb[2][i][j]);
          }
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int o = tpos(sk + 8 * i, sc);
      u32x2 p0, p1, p2;
      split4(f4(ra[i]), p0, p1, p2);
      *reinterpret_cast<u32x2*>(S + 0 * PIECE + o) = p0;
      *reinterpret_cast<u32x2*>(S + 1 * PIECE + o) = p1;
      *reinterpret_cast<u32x2*>(S + 2 * PIECE + o) = p2;
      const float4 bf = f4(rb[i]);
      split4(bf, p0, p1, p2);
      *reinterpret_cast<u32x2*>(S + 3 * PIECE + o) = p0;
      *reinterpret_cast<u32x2*>(S + 4 * PIECE + o) = p1;
      *reinterpret_cast<u32x2*>(S + 5 * PIECE + o) = p2;
      if (do_cs) {
        cs[0] += bf.x;
        cs[1] += bf.y;
        cs[2] += bf.z;
        cs[3] += bf.w;
      }
    }
  };

  const int g = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;  // transpose-read roles (gemm_bf16.hip TN form)
  auto frag = [&](const __bf16* P, int col) -> bf16x8 {
    // (tsw(r + 4) == tsw(r) for r = 8g + tq: the hi rows keep the lo rows' units)
    const __bf16* p0 = P + tpos(8 * g + tq, col + 4 * tp);
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)p0);
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p0 + 4 * LDR));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto compute = [&](int stage) {
    const __bf16* S = lds + stage * STAGE;
    auto pass = [&](const bf16x8 (&x)[4], const bf16x8 (&y)[4]) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[mi], y[ni], acc[mi][ni], 0, 0, 0);
    };
    // the B pieces held for the k-tile, the A pieces one at a time (smallest
    // terms first: a2 b0; a1 b1, a1 b0; a0 b2, a0 b1, a0 b0): 64 fragment
    // registers live instead of 96
    bf16x8 b[NPC][4];
#pragma unroll
    for (int p = 0; p < NPC; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i) b[p][i] = frag(S + (3 + p) * PIECE, wn + 16 * i);
#pragma unroll
    for (int pa = NPC - 1; pa >= 0; --pa) {
      bf16x8 a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag(S + pa * PIECE, wm + 16 * i);
#pragma unroll
      for (int pb = NPC - 1 - pa; pb >= 0; --pb) pass(a, b[pb]);
    }
  };

  const int nk = kbeg < kend ? (kend - kbeg + BK - 1) / BK : 0;
  {
    // one LDS stage (52 KB: two workgroups per CU overlap each other's split
    // and MFMA phases; two stages at one workgroup per CU measured 417 vs
    // 318 us); the next k-tile's loads are in flight under the MFMAs
    if (nk > 0) load_tiles(kbeg);
    for (int it = 0; it < nk; ++it) {
      store_tiles(0);
      if (it + 1 < nk) load_tiles(kbeg + (it + 1) * BK);
      __syncthreads();
      compute(0);
      __syncthreads();
    }
  }
  if (do_cs) {
    // the per-thread column partials summed in a fixed order through LDS (free
    // after the loop's last barrier): one atomic per column and workgroup, so
    // the bias gradient is deterministic whenever split-K is 1
    float* red = reinterpret_cast<float*>(lds);  // [16 row groups][BN]
    constexpr int RG = PRE ? 16 : 8;
    if (PRE) {
#pragma unroll
      for (int c = 0; c < 8; ++c) red[pk * BN + pc + c] = cs8[c];
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) red[sk * BN + sc + c] = cs[c];
    }
    __syncthreads();
    if (t < BN && n0 + t < N) {
      float v = 0.f;
#pragma unroll
      for (int r = 0; r < RG; ++r) v += red[r * BN + t];
      // split-K through the workspace: this split's column partial goes to
      // work[nsplit][M][N] + [ks][N] and splitk_reduce_kernel adds the splits
      // in split order (deterministic); one split: the only writer of these
      // columns; float atomics otherwise
      if (D.nsplit > 1 && D.work != nullptr)
        D.work[(size_t)D.nsplit * M * N + (size_t)ks * N + n0 + t] = v;
      else
        atomicAdd(D.colsum + n0 + t, v);
    }
  }
  x3_epilogue(D, acc, m0 + wm, n0 + wn, ks, lane);
}


bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

void splitk_reduce(const X3Args& D, hipStream_t s);

void launch_x3(bool pre, X3Args D, int splitk, hipStream_t s, int npieces = 3) {
  int kchunk = (D.K + splitk - 1) / splitk;
  kchunk = ((kchunk + BK - 1) / BK) * BK;
  D.kchunk = kchunk;
  const int nsplit = (D.K + kchunk - 1) / kchunk;
  D.nsplit = nsplit;
  D.nx = mog_cdiv(D.N, BN);
  D.ny = mog_cdiv(D.M, BM);
  const long nwg = (long)D.nx * D.ny * nsplit;
  if (pre && npieces == 1) gemm_x3_tn_kernel<true, 1><<<dim3((unsigned)nwg), 256, 0, s>>>(D);
  else if (pre) gemm_x3_tn_kernel<true><<<dim3((unsigned)nwg), 256, 0, s>>>(D);
  else gemm_x3_tn_kernel<false><<<dim3((unsigned)nwg), 256, 0, s>>>(D);
  if (nsplit > 1 && D.work != nullptr) splitk_reduce(D, s);
}

// the three exact truncated bf16 pieces of an fp32 [rows][cols] matrix: piece p
// at dst + p * pstride, element (r, c) at r * ld_dst + c; columns cols..ld_dst-1
// are written as zeros
__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ src, int rows,
                                                     int cols, int ld_src, __bf16* dst, int ld_dst,
                                                     long pstride) {
  const int q4 = ld_dst / 4;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)rows * q4) return;
  const int r = (int)(i / q4), c = (int)(i % q4) * 4;
  const float4 v = c < cols ? *reinterpret_cast<const float4*>(src + (size_t)r * ld_src + c)
                            : float4{0.f, 0.f, 0.f, 0.f};
  u32x2 p0, p1, p2;
  split4(v, p0, p1, p2);
  __bf16* d = dst + (size_t)r * ld_dst + c;
  *reinterpret_cast<u32x2*>(d) = p0;
  *reinterpret_cast<u32x2*>(d + pstride) = p1;
  *reinterpret_cast<u32x2*>(d + 2 * pstride) = p2;
}

// The same pieces of a sum of nsum fp32 matrices src + j * sum_stride, added
// from the LAST to the first starting from +0 (((0 + s[n-1]) + s[n-2]) + ...
// + s[0]: the order in which the LSTM chain's reversed loop accumulated the
// gate gradients' step sum, bit for bit), so the sum never goes to HBM
__global__ __launch_bounds__(256) void split3_sum_kernel(const float* __restrict__ src, int nsum,
                                                         long sum_stride, int rows, int cols,
                                                         int ld_src, __bf16* dst, int ld_dst,
                                                         long pstride) {
#pragma clang fp contract(off)
  const int q4 = ld_dst / 4;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)rows * q4) return;
  const int r = (int)(i / q4), c = (int)(i % q4) * 4;
  float4 v = float4{0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    const float* p = src + (size_t)r * ld_src + c;
    float4 t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < nsum) t[j] = *reinterpret_cast<const float4*>(p + (size_t)j * sum_stride);
#pragma unroll
    for (int j = 7; j >= 0; --j)
      if (j < nsum) {
        v.x = v.x + t[j].x; v.y = v.y + t[j].y; v.z = v.z + t[j].z; v.w = v.w + t[j].w;
      }
  }
  u32x2 p0, p1, p2;
  split4(v, p0, p1, p2);
  __bf16* d = dst + (size_t)r * ld_dst + c;
  *reinterpret_cast<u32x2*>(d) = p0;
  *reinterpret_cast<u32x2*>(d + pstride) = p1;
  *reinterpret_cast<u32x2*>(d + 2 * pstride) = p2;
}

// C[m][n] += sum over s = 0 .. nsplit-1 of work[s][m][n], in that order (the
// split-K partials of the TN forms: deterministic, plain loads and stores);
// with a column sum, colsum[n] += the splits' column partials (stored after
// the [nsplit][M][N] partials, [nsplit][N]) likewise in split order -- thread
// q handles column q (the grid covers max(M*N/4, N) threads)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ W, int nsplit,
                                                            float* C, int M, int N, int ldc,
                                                            bool vec, float* colsum) {
  const long MN = (long)M * N;
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  if (colsum != nullptr && q < N) {
    const float* P = W + (size_t)nsplit * MN;
    float v = P[q];
    for (int s = 1; s < nsplit; ++s) v += P[(size_t)s * N + q];
    colsum[q] += v;
  }
  const long i = q * 4;
  if (i >= MN) return;
  if (vec) {
    float4 v = *reinterpret_cast<const float4*>(W + i);
    for (int s = 1; s < nsplit; ++s) {
      const floatx4 u = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(W + s * MN + i));
      v.x += u[0]; v.y += u[1]; v.z += u[2]; v.w += u[3];
    }
    const int m = (int)(i / N), n = (int)(i % N);
    float4* c = reinterpret_cast<float4*>(C + (size_t)m * ldc + n);
    float4 o = *c;
    o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
    *c = o;
    return;
  }
  for (long e = i; e < min(i + 4, MN); ++e) {
    float v = W[e];
    for (int s = 1; s < nsplit; ++s) v += W[s * MN + e];
    C[(size_t)(e / N) * ldc + e % N] += v;
  }
}

void splitk_reduce(const X3Args& D, hipStream_t s) {
  const long n4 = ((long)D.M * D.N + 3) / 4;
  const long nt = n4 > D.N ? n4 : (long)D.N;
  const bool vec = D.N % 4 == 0 && D.ldc % 4 == 0 && (reinterpret_cast<uintptr_t>(D.C) & 15) == 0;
  splitk_reduce_kernel<<<dim3((unsigned)((nt + 255) / 256)), 256, 0, s>>>(
      D.work, D.nsplit, D.C, D.M, D.N, D.ldc, vec, D.colsum);
}

// ---- NT form: C[M][N] = epi(sum_k A[m][k] B[n][k]) ------------------------
// The input gradients of the VAE (dX = dY W^T: A = dY [M][lda] fp32,
// k-contiguous rows; B = W [N][K] given as its three bf16 pieces, split once
// per optimizer step, k-contiguous rows of ldb) at fp32-level accuracy on the
// bf16 matrix cores: A is split in registers as it is staged, both operands
// live in LDS as k-contiguous rows, so every MFMA fragment (row li, k 8g ..
// 8g+7) is one ds_read_b128; six products per 16x16x32 block, smallest first.
// Epilogue: the accumulator quads transposed across lanes (a lane owns four
// consecutive columns), then store or softplus backward (C = v * sigmoid(aux),
// gemm_f32.hip's EPI_SOFTPLUS_BWD), 16-byte stores.  No split-K: the sums
// over K (<= 784) stay inside one workgroup, so the result is deterministic.
constexpr int NT_LDK = BK + 16;  // LDS row pitch (bf16): 96 B -- the fragment reads (ds_read_b128,
                                 // lane groups of MI355X_MICROARCH §LDS) hit distinct banks; 80 B
                                 // left them 2-way conflicted (half the LDS cycles, SQ_LDS_BANK_CONFLICT)
constexpr int NT_PIECE = BM * NT_LDK;
constexpr int NT_STAGE = 6 * NT_PIECE;         // A0 A1 A2 B0 B1 B2 (73,728 B)
constexpr int NT_NLA = (BM * BK / 4) / 256;    // float4 loads of A per thread (4)
constexpr int NT_NLB = (BN * BK / 8) / 256;    // 16-byte chunks of a B piece per thread (2)

struct X3NtArgs {
  const float* A;
  const __bf16* B3;
  long sb;
  float* C;
  const float* aux;
  int M, N, K, lda, ldb, ldc, ldaux, nx, ny, epi;
};

__device__ __forceinline__ float xt_dpp1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float xt_dpp2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}
// 4 x 4 transpose inside lane quads: row g*4 + r of column li in, row
// g*4 + (li & 3) at columns (li & ~3) + r out
__device__ __forceinline__ floatx4 xt_quad_transpose(const floatx4& a, int lane) {
  const int e = lane & 3;
  float r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3];
  {
    const bool hi = (e & 2) != 0;
    const float t0 = xt_dpp2(hi ? r0 : r2), t1 = xt_dpp2(hi ? r1 : r3);
    if (hi) { r0 = t0; r1 = t1; } else { r2 = t0; r3 = t1; }
  }
  {
    const bool od = (e & 1) != 0;
    const float t0 = xt_dpp1(od ? r0 : r1), t1 = xt_dpp1(od ? r2 : r3);
    if (od) { r0 = t0; r2 = t1; } else { r1 = t0; r3 = t1; }
  }
  return floatx4{r0, r1, r2, r3};
}

// EPI: 0 store, 1 softplus backward (aux = the softplus output p:
// sigmoid(x) = 1 - exp(-p) = -expm1(-p)).  The next k-tile's loads are in flight
// under the MFMAs (one register set: a second, loads two MFMA phases ahead,
// measured no faster; neither was a double-buffered 8-wave form with the
// split woven between the MFMA passes, 158 -> 162 us)
template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_x3_nt_kernel(X3NtArgs D) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[NT_STAGE];
  const int nwg = gridDim.x;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int bx = wg % D.nx, by = wg / D.nx;
  const int m0 = by * BM, n0 = bx * BN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const int M = D.M, N = D.N, K = D.K;
  // staging roles: A float4 i covers row t/8 + 32 i, k 4 (t % 8) ..; B chunk i
  // of a piece covers row t/4 + 64 i, k 8 (t % 4) ..
  const int ar = t >> 3, ak = (t & 7) * 4;
  const int br = t >> 2, bk = (t & 3) * 8;
  floatx4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = floatx4{0.f, 0.f, 0.f, 0.f};
  // loaded as raw dwords and reinterpreted only at the split: a conversion at
  // the load makes the compiler copy the registers right after it, which
  // waits for the load there and serialises the prefetch
  u32x4 ra[NT_NLA];
  u32x4 rb[3][NT_NLB];
  // Buffer loads: the workgroup's A rows behind one descriptor and each B
  // piece behind its own, the row offsets in the per-thread (range-checked)
  // offset, only the uniform k-tile step in the scalar offset, which the
  // range check does not cover (it stays inside a row: k0 + 8 <= K <= ld).
  // Every load is issued unconditionally -- a predicated load (`cond ? load
  // : 0`) becomes a branch around it with a vmcnt(0) wait inside, one full
  // memory latency per load -- and what must read as zero is pushed out of
  // the descriptor's range instead: A rows >= M and B rows >= N fall outside
  // their operand's record range; k >= K (the last k-tile, K % 32 != 0; with
  // lda == K those addresses hold the next row) gets an offset past every
  // range, on both operands.
  // record ranges: the rows, ending at column K of the operand's last row --
  // its validated extent
  const int arows = min(M - m0, BM);
  const __amdgpu_buffer_rsrc_t arsc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(D.A) + (size_t)m0 * D.lda, 0,
      (M - m0 > BM ? BM * D.lda : (arows - 1) * D.lda + K) * 4, 0x00020000);
  __amdgpu_buffer_rsrc_t brsc[3];
#pragma unroll
  for (int p = 0; p < 3; ++p)
    brsc[p] = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(D.B3) + (size_t)p * D.sb, 0,
                                                ((N - 1) * D.ldb + K) * 2, 0x00020000);
  int avo[NT_NLA], bvo[NT_NLB];
#pragma unroll
  for (int i = 0; i < NT_NLA; ++i) avo[i] = ((ar + 32 * i) * D.lda + ak) * 4;
#pragma unroll
  for (int i = 0; i < NT_NLB; ++i) bvo[i] = ((n0 + br + 64 * i) * D.ldb + bk) * 2;
  constexpr int OOB = (int)0x80000000u;  // past every range
  auto load_tiles = [&](int k0) {
    const bool ak_in = k0 + ak < K, bk_in = k0 + bk < K;
#pragma unroll
    for (int i = 0; i < NT_NLA; ++i)
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(arsc, ak_in ? avo[i] : OOB, k0 * 4, 0);
#pragma unroll
    for (int i = 0; i < NT_NLB; ++i)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        rb[p][i] = __builtin_amdgcn_raw_buffer_load_b128(brsc[p], bk_in ? bvo[i] : OOB, k0 * 2, 0);
  };
  auto store_tiles = [&]() {
#pragma unroll
    for (int i = 0; i < NT_NLA; ++i) {
      const int o = (ar + 32 * i) * NT_LDK + ak;
      u32x2 p0, p1, p2;
      split4(float4{__uint_as_float(ra[i][0]), __uint_as_float(ra[i][1]),
                    __uint_as_float(ra[i][2]), __uint_as_float(ra[i][3])},
             p0, p1, p2);
      *reinterpret_cast<u32x2*>(lds + 0 * NT_PIECE + o) = p0;
      *reinterpret_cast<u32x2*>(lds + 1 * NT_PIECE + o) = p1;
      *reinterpret_cast<u32x2*>(lds + 2 * NT_PIECE + o) = p2;
    }
#pragma unroll
    for (int i = 0; i < NT_NLB; ++i) {
      const int o = (br + 64 * i) * NT_LDK + bk;
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<u32x4*>(lds + (3 + p) * NT_PIECE + o) = rb[p][i];
    }
  };
  const int g = lane >> 4, li = lane & 15;
  auto frag = [&](int piece, int row) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(lds + piece * NT_PIECE + (row + li) * NT_LDK + 8 * g);
  };
  // the B pieces held for the whole k-tile, the A pieces one at a time
  // (smallest first: a2 b0; a1 b1, a1 b0; a0 b2, a0 b1, a0 b0): 64 fragment
  // registers live instead of 96
  auto compute = [&]() {
    bf16x8 b[3][4];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i) b[p][i] = frag(3 + p, wn + 16 * i);
    auto pass = [&](const bf16x8 (&x)[4], const bf16x8 (&y)[4]) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[mi], y[ni], acc[mi][ni], 0, 0, 0);
    };
#pragma unroll
    for (int pa = 2; pa >= 0; --pa) {
      bf16x8 a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag(pa, wm + 16 * i);
#pragma unroll
      for (int pb = 2 - pa; pb >= 0; --pb) pass(a, b[pb]);
    }
  };
  const int nk = (K + BK - 1) / BK;
  load_tiles(0);
  for (int it = 0; it < nk; ++it) {
    store_tiles();
    if (it + 1 < nk) load_tiles((it + 1) * BK);
    __syncthreads();
    compute();
    __syncthreads();
  }
  // softplus backward: every aux quad of the lane loaded up front,
  // unconditionally (rows >= M fall outside the descriptor; columns >= N are
  // loaded but not stored), so the sixteen loads share one latency
  u32x4 xq[4][4];
  if constexpr (EPI == 1) {
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(D.aux) + (size_t)m0 * D.ldaux, 0,
        (M - m0 > BM ? BM * D.ldaux : (arows - 1) * D.ldaux + N) * 4, 0x00020000);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        xq[mi][ni] = __builtin_amdgcn_raw_buffer_load_b128(
            xr, ((wm + mi * 16 + g * 4 + (li & 3)) * D.ldaux + n0 + wn + ni * 16 + (li & ~3)) * 4,
            0, 0);
  }
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const floatx4 v = xt_quad_transpose(acc[mi][ni], lane);
      const int row = m0 + wm + mi * 16 + g * 4 + (li & 3);
      const int col = n0 + wn + ni * 16 + (li & ~3);
      float o[4] = {v[0], v[1], v[2], v[3]};
      if (EPI == 1) {
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = v[q] * -mog_expm1f(-__uint_as_float(xq[mi][ni][q]));
      }
      if (row < M && col < N)
        *reinterpret_cast<float4*>(D.C + (size_t)row * D.ldc + col) = make_float4(o[0], o[1], o[2], o[3]);
    }
}

}  // namespace

extern "C" int mog_split3_bf16(const float* src, int rows, int cols, int ld_src, void* dst,
                               int ld_dst, long piece_stride, void* stream) {
  MOG_CHECK_ARG(src && dst && rows >= 0 && cols >= 0 && cols % 4 == 0 && ld_src % 4 == 0 &&
                ld_dst % 4 == 0 && ld_dst >= cols && ld_src >= cols && piece_stride % 4 == 0 &&
                piece_stride >= (long)rows * ld_dst && al16(src) && al16(dst));
  const long n = (long)rows * (ld_dst / 4);
  if (n == 0) return 0;
  split3_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, mog_stream(stream)>>>(
      src, rows, cols, ld_src, reinterpret_cast<__bf16*>(dst), ld_dst, piece_stride);
  MOG_LAUNCH_RET();
}

extern "C" int mog_split3_sum_bf16(const float* src, int nsum, long sum_stride, int rows,
                                   int cols, int ld_src, void* dst, int ld_dst, long piece_stride,
                                   void* stream) {
  MOG_CHECK_ARG(src && dst && nsum >= 1 && nsum <= 8 && sum_stride % 4 == 0 &&
                (nsum == 1 || sum_stride >= (long)(rows - 1) * ld_src + cols));
  MOG_CHECK_ARG(rows >= 0 && cols >= 0 && cols % 4 == 0 && ld_src % 4 == 0 &&
                ld_dst % 4 == 0 && ld_dst >= cols && ld_src >= cols && piece_stride % 4 == 0 &&
                piece_stride >= (long)rows * ld_dst && al16(src) && al16(dst));
  const long n = (long)rows * (ld_dst / 4);
  if (n == 0) return 0;
  split3_sum_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, mog_stream(stream)>>>(
      src, nsum, sum_stride, rows, cols, ld_src, reinterpret_cast<__bf16*>(dst), ld_dst,
      piece_stride);
  MOG_LAUNCH_RET();
}

extern "C" int mog_gemm_x3p_tn(const void* A3, long sa, const void* B3, long sb, float* C,
                               float* colsum, int M, int N, int K, int lda, int ldb, int ldc,
                               int splitk, int npieces, float* work, long work_elems,
                               void* stream) {
  MOG_CHECK_ARG(A3 && B3 && C && M >= 0 && N >= 0 && K >= 0 && splitk >= 1);
  MOG_CHECK_ARG(work == nullptr ||
                work_elems >= (long)splitk * M * N + (colsum ? (long)splitk * N : 0));
  MOG_CHECK_ARG(npieces == 3 || npieces == 1);
  // 16-byte chunks of 8 bf16: strides and piece strides multiples of 8 (a chunk
  // that starts below M ends inside the row; its columns >= M are not stored)
  MOG_CHECK_ARG(al16(A3) && al16(B3) && lda % 8 == 0 && ldb % 8 == 0 && sa % 8 == 0 &&
                sb % 8 == 0 && lda >= M && ldb >= N && ldc >= N);
  // 32-bit buffer offsets over the pieces
  MOG_CHECK_ARG((2 * sa + (long)K * lda) * 2 < (1L << 31) && (2 * sb + (long)K * ldb) * 2 < (1L << 31));
  if (M == 0 || N == 0 || K == 0) return 0;
  X3Args D{};
  D.A3 = reinterpret_cast<const __bf16*>(A3);
  D.B3 = reinterpret_cast<const __bf16*>(B3);
  D.sa = sa; D.sb = sb; D.C = C; D.colsum = colsum; D.work = work;
  D.M = M; D.N = N; D.K = K; D.lda = lda; D.ldb = ldb; D.ldc = ldc;
  launch_x3(true, D, splitk, mog_stream(stream), npieces);
  MOG_LAUNCH_RET();
}

extern "C" int mog_gemm_f32_x3_tn(const float* A, const float* B, float* C, float* colsum,
                                  int M, int N, int K, int lda, int ldb, int ldc, int splitk,
                                  float* work, long work_elems, void* stream) {
  MOG_CHECK_ARG(A && B && C && M >= 0 && N >= 0 && K >= 0 && splitk >= 1);
  MOG_CHECK_ARG(work == nullptr ||
                work_elems >= (long)splitk * M * N + (colsum ? (long)splitk * N : 0));
  // float4 rows: 16-byte operands, widths and strides multiples of 4
  MOG_CHECK_ARG(al16(A) && al16(B) && M % 4 == 0 && N % 4 == 0 && lda % 4 == 0 &&
                ldb % 4 == 0 && lda >= M && ldb >= N && ldc >= N);
  MOG_CHECK_ARG((long)K * lda * 4 < (1L << 31) && (long)K * ldb * 4 < (1L << 31));
  if (M == 0 || N == 0 || K == 0) return 0;
  X3Args D{};
  D.A = A; D.B = B; D.C = C; D.colsum = colsum; D.work = work;
  D.M = M; D.N = N; D.K = K; D.lda = lda; D.ldb = ldb; D.ldc = ldc;
  launch_x3(false, D, splitk, mog_stream(stream));
  MOG_LAUNCH_RET();
}

extern "C" int mog_gemm_x3_nt(const float* A, const void* B3, long sb, float* C, const float* aux,
                              int M, int N, int K, int lda, int ldb, int ldc, int ldaux, int epi,
                              void* stream) {
  MOG_CHECK_ARG(A && B3 && C && M >= 0 && N >= 0 && K >= 0 && (epi == 0 || epi == 1));
  MOG_CHECK_ARG(epi == 0 || (aux && ldaux % 4 == 0 && ldaux >= N && al16(aux)));
  // 16-byte accesses: float4 rows of A and C (K, N, lda, ldc multiples of 4),
  // 8-bf16 chunks of the B pieces (K, ldb, sb multiples of 8: a chunk never
  // straddles the end of a row, so no pad element of W is read)
  MOG_CHECK_ARG(al16(A) && al16(B3) && al16(C) && K % 8 == 0 && N % 4 == 0 && lda % 4 == 0 &&
                ldc % 4 == 0 && ldb % 8 == 0 && sb % 8 == 0 && lda >= K && ldb >= K && ldc >= N);
  // 32-bit buffer offsets: the pieces and one 128-row panel of A
  MOG_CHECK_ARG((long)N * ldb * 2 < (1L << 31) && (long)BM * lda * 4 < (1L << 31) &&
                (long)BM * ldaux * 4 < (1L << 31));
  if (M == 0 || N == 0) return 0;
  X3NtArgs D{};
  D.A = A; D.B3 = reinterpret_cast<const __bf16*>(B3); D.sb = sb; D.C = C; D.aux = aux;
  D.M = M; D.N = N; D.K = K; D.lda = lda; D.ldb = ldb; D.ldc = ldc; D.ldaux = ldaux;
  D.nx = mog_cdiv(N, BN);
  D.ny = mog_cdiv(M, BM);
  D.epi = epi;
  const unsigned nwg = (unsigned)D.nx * D.ny;
  hipStream_t s = mog_stream(stream);
  if (epi == 1) gemm_x3_nt_kernel<1><<<nwg, 256, 0, s>>>(D);
  else gemm_x3_nt_kernel<0><<<nwg, 256, 0, s>>>(D);
  MOG_LAUNCH_RET();
}
