// Exact three-piece bf16 splits of fp32 operands (the x3 GEMMs of
// gemm_x3.hip and wgrad_tn.hip): x = x0 + x1 + x2 by truncation, x0 the top 8
// significand bits, x1 the next 8 of x - x0, x2 the rest (at most 8
// significant bits), so sum_{i+j<=2} a_i b_j carries a b down to 2^-16 of it.
#pragma once
#include "mog_common.h"

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// the three truncated bf16 pieces of one float (as fp32 bit patterns whose low
// halves are zero, except lo's, which the packing drops)
static __device__ __forceinline__ void split1(float f, unsigned& hi, unsigned& mid, unsigned& lo) {
  hi = __float_as_uint(f) & 0xffff0000u;
  const float r1 = f - __uint_as_float(hi);  // exact
  mid = __float_as_uint(r1) & 0xffff0000u;
  lo = __float_as_uint(r1 - __uint_as_float(mid));  // exact, <= 8 significant bits
}

static __device__ __forceinline__ unsigned pack2(unsigned a, unsigned b) {
  return (a >> 16) | (b & 0xffff0000u);
}

// the pieces of four floats, packed two bf16 per dword
static __device__ __forceinline__ void split4(const float4 v, u32x2& p0, u32x2& p1, u32x2& p2) {
  unsigned h0, m0, l0, h1, m1, l1, h2, m2, l2, h3, m3, l3;
  split1(v.x, h0, m0, l0);
  split1(v.y, h1, m1, l1);
  split1(v.z, h2, m2, l2);
  split1(v.w, h3, m3, l3);
  p0.x = pack2(h0, h1);
  p0.y = pack2(h2, h3);
  p1.x = pack2(m0, m1);
  p1.y = pack2(m2, m3);
  p2.x = pack2(l0, l1);
  p2.y = pack2(l2, l3);
}

