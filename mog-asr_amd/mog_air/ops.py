"""Typed wrappers of the HIP entry points over torch device tensors.

Every launch goes through the PyTorch-ROCm custom operators torch.ops.mog_air.*
(csrc/torch_ops.cpp, a TORCH_LIBRARY fragment over the C ABI of libmog_air.so)
on torch's current HIP stream.  Arguments are validated here (device, dtype,
contiguity, shape) before any launch, so a shape error never reaches a
kernel."""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from . import _lib

_lib.load_torch_ops()
_ops = torch.ops.mog_air

EPI_STORE, EPI_RELU, EPI_SOFTPLUS, EPI_SIGMOID_NOISE = 0, 1, 2, 3
EPI_SOFTPLUS_BWD, EPI_ATOMIC, EPI_RELU_BWD = 4, 5, 6


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def dp(t: Optional[torch.Tensor]):
    if t is None:
        return None
    return t.data_ptr()


def _chk(t: torch.Tensor, name: str, dtype=torch.float32):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a HIP device tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _opt_list(xs):
    return [] if xs is None else list(xs)


def gemm(A: Sequence[torch.Tensor], B: Sequence[torch.Tensor], C: Sequence[torch.Tensor],
         M: int, N: int, K: int, lda: int, ldb: int, ldc: int, transA=False, transB=False,
         epi=EPI_STORE, bias=None, Cin=None, Cpre=None, aux=None, ldaux=0,
         aux_scale=0.0, splitk=1, colsum=None) -> None:
    """Batched fp32 MFMA GEMM (see mog_gemm_f32).  A/B/C are sequences of
    tensors (or views) whose data_ptr is the matrix origin."""
    nb = len(C)
    assert len(A) == nb and len(B) == nb and 1 <= nb <= 8
    _ops.gemm_f32_(list(A), list(B), list(C), _opt_list(bias), _opt_list(Cin), _opt_list(Cpre),
                   _opt_list(aux), _opt_list(colsum), M, N, K, lda, ldb, ldc, ldaux,
                   bool(transA), bool(transB), epi, float(aux_scale), int(splitk))


def gemm_x3_tn(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, M: int, N: int, K: int,
               lda: int, ldb: int, ldc: int, splitk: int = 8, colsum=None,
               reduce: bool = True) -> None:
    """C[M,N] += A^T B over K rows on the bf16 matrix cores with exact
    three-piece operand splits (fp32-level accuracy; mog_gemm_f32_x3_tn);
    colsum += column sums of B.  reduce: split-K partials summed through a
    workspace in a fixed order (deterministic); False: float atomics."""
    _ops.gemm_f32_x3_tn_(A, B, C, colsum, M, N, K, lda, ldb, ldc, int(splitk), int(reduce))


def split3_bf16(src: torch.Tensor, dst: torch.Tensor, rows: int, cols: int, ld_src: int,
                ld_dst: int, piece_stride: int) -> None:
    """The three exact truncated bf16 pieces of an fp32 matrix
    (mog_split3_bf16)."""
    _ops.split3_bf16_(src, dst, rows, cols, ld_src, ld_dst, int(piece_stride))


def gemm_x3p_tn(A3: torch.Tensor, sa: int, B3: torch.Tensor, sb: int, C: torch.Tensor, M: int,
                N: int, K: int, lda: int, ldb: int, ldc: int, splitk: int = 8,
                colsum=None, npieces: int = 3, reduce: bool = True) -> None:
    """gemm_x3_tn from operands split beforehand by split3_bf16
    (mog_gemm_x3p_tn); npieces=1: plain bf16 operands, one product."""
    _ops.gemm_x3p_tn_(A3, int(sa), B3, int(sb), C, colsum, M, N, K, lda, ldb, ldc, int(splitk),
                      int(npieces), int(reduce))


def gemm_x3_nt(A: torch.Tensor, B3: torch.Tensor, sb: int, C: torch.Tensor, M: int, N: int,
               K: int, lda: int, ldb: int, ldc: int, aux=None, ldaux: int = 0) -> None:
    """C[M,N] = A B^T at fp32-level accuracy (A split into three bf16 pieces
    in the kernel, B given as split3_bf16's pieces of W [N][K]); with aux:
    C = (A B^T) * sigmoid(aux) (the softplus backward) -- mog_gemm_x3_nt."""
    _ops.gemm_x3_nt_(A, B3, int(sb), C, aux, M, N, K, lda, ldb, ldc, int(ldaux),
                     1 if aux is not None else 0)


def wgrad_tn_bf16(X: Sequence[torch.Tensor], dY: Sequence[torch.Tensor],
                  out: Sequence[torch.Tensor], colsum: Sequence[Optional[torch.Tensor]],
                  dims: Sequence[Sequence[int]], K: int, nsplit: int = 8) -> None:
    """out[i] += X[i]^T dY[i] over K rows on bf16 operands, colsum[i] += the
    column sums of dY[i], every problem in one launch (dims[i] = (M, N, lda,
    ldb, ldc)); K split nsplit ways, the splits added in order by a second
    launch: deterministic (mog_wgrad_tn_bf16)."""
    _ops.wgrad_tn_bf16_(list(X), list(dY), list(out), list(colsum),
                        [int(d) for ds in dims for d in ds], int(K), int(nsplit))


def wgrad_tn_x3(X: Sequence[torch.Tensor], dY: Sequence[torch.Tensor],
                out: Sequence[torch.Tensor], colsum: Sequence[Optional[torch.Tensor]],
                dims: Sequence[Sequence[int]], K: int, nsplit: int = 8) -> None:
    """wgrad_tn_bf16 on fp32 operands at fp32-level accuracy (exact
    three-piece bf16 splits in the kernel; mog_wgrad_tn_x3)."""
    _ops.wgrad_tn_x3_(list(X), list(dY), list(out), list(colsum),
                      [int(d) for ds in dims for d in ds], int(K), int(nsplit))


class WgradGroup:
    """Weight gradients collected over a backward pass and run as ONE grouped
    launch (mog_gemm_f32_wgrad_group): each problem is out[M,N] += X^T dY
    over K rows (+ bias_out += column sums of dY); the problems travel in the
    kernel argument (graph-capturable).  Problems that share output elements
    go to successive launches (one writer per element within a launch)."""

    def __init__(self):
        self.probs = []

    @staticmethod
    def _check(t, extent, what):
        if t.dtype != torch.float32 or not t.is_cuda:
            raise RuntimeError(f"WgradGroup: {what} must be a float32 device tensor")
        avail = t.untyped_storage().nbytes() // 4 - t.storage_offset()
        if extent > avail:
            raise RuntimeError(f"WgradGroup: {what} holds {avail} elements, needs {extent}")

    def add(self, X, dY, out, M, N, K, lda, ldb, ldc, bias_out=None):
        if min(M, N) <= 0:
            return
        span = lambda r, c, ld: 0 if r <= 0 else (r - 1) * ld + c  # noqa: E731
        self._check(X, span(K, M, lda), "X")
        self._check(dY, span(K, N, ldb), "dY")
        self._check(out, span(M, N, ldc), "out")
        if bias_out is not None:
            self._check(bias_out, N, "bias_out")
        self.probs.append((X, dY, out, bias_out, M, N, K, lda, ldb, ldc))

    def launch(self):
        """In collection order; a problem whose output or bias range overlaps
        one already in the current launch starts the next launch (same
        stream, so the two accumulate in order)."""
        batch, ranges = [], []

        def flush():
            if batch:
                X, dY, out, bias, dims = zip(*batch)
                _ops.gemm_f32_wgrad_group_(list(X), list(dY), list(out), list(bias),
                                           [d for ds in dims for d in ds])
            batch.clear()
            ranges.clear()

        for X, dY, out, b, M, N, K, lda, ldb, ldc in self.probs:
            mine = [(out.data_ptr(), out.data_ptr() + 4 * ((M - 1) * ldc + N))]
            if b is not None:
                mine.append((b.data_ptr(), b.data_ptr() + 4 * N))
            if any(lo < h and l2 < hi for lo, hi in mine for l2, h in ranges):
                flush()
            ranges.extend(mine)
            batch.append((X, dY, out, b, (M, N, K, lda, ldb, ldc)))
        flush()
        self.probs = []


def gemm_sigmoid_philox(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, bias, M: int, N: int,
                        K: int, lda: int, ldb: int, ldc: int, scale: float, seed: int,
                        offset: int) -> None:
    """C = sigmoid((A B + bias) + scale * eps), eps generated in the epilogue
    exactly as rng_fill(seed, offset) of an [M, N] buffer would hold it
    (mog_gemm_f32_sigmoid_philox)."""
    _ops.gemm_f32_sigmoid_philox_(A, B, C, bias, M, N, K, lda, ldb, ldc, float(scale),
                                  _i64(seed), _i64(offset))


def gemm_kseg(A: Sequence[torch.Tensor], B: Sequence[torch.Tensor], C: torch.Tensor, M: int,
              N: int, kseg: int, lda: int, ldb: int, ldc: int, transB=False, Cin=None,
              epi=EPI_STORE) -> None:
    """C = sum_s A_s op(B_s) as ONE k-ordered chain (mog_gemm_f32_kseg)."""
    _ops.gemm_f32_kseg_(list(A), list(B), C, None, Cin, M, N, kseg, lda, ldb, ldc, False,
                        bool(transB), epi)


def gemm_kseg_group(probs, M: int, N: int, kseg: int, lda: int, ldb: int, ldc: int,
                    transB=False) -> None:
    """Independent k-segment chains of one shape in ONE launch
    (mog_gemm_f32_kseg_group): ``probs`` = [(A_list, B_list, C, Cin), ...],
    C_z = Cin_z + sum_s A_s op(B_s) -- the same bits as one gemm_kseg each."""
    A = [a for p in probs for a in p[0]]
    B = [b for p in probs for b in p[1]]
    _ops.gemm_f32_kseg_group_(A, B, [p[2] for p in probs], [p[3] for p in probs],
                              [len(p[0]) for p in probs], M, N, kseg, lda, ldb, ldc,
                              bool(transB))


def dense(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], out: torch.Tensor,
          epi=EPI_STORE, pre: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = act(x @ w + b), one k-ordered fp32 chain per output."""
    M, K = x.shape
    K2, N = w.shape
    assert K == K2 and out.shape == (M, N)
    gemm([x], [w], [out], M, N, K, K, N, N, epi=epi, bias=None if b is None else [b],
         Cpre=None if pre is None else [pre])
    return out


def stn_forward(U: torch.Tensor, theta: torch.Tensor, out_hw, out: Optional[torch.Tensor] = None,
                z: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None,
                accumulate: bool = False, n: Optional[int] = None) -> torch.Tensor:
    """transformer() of air/transformer.py:18 for U [N,Hin,Win] (or [N,Hin*Win] with
    Hin=Win) and theta [N,6].  A bf16 ``out`` receives the bf16 image.  n > N:
    n images, image i reading U[i % N] (every loop step's read of one canvas)."""
    _chk(U, "U")
    _chk(theta, "theta")
    period = U.shape[0] if n is not None and n != U.shape[0] else 0
    N = U.shape[0] if n is None else n
    if U.dim() == 3:
        Hin, Win = U.shape[1], U.shape[2]
    else:
        Hin = Win = int(round(U.shape[1] ** 0.5))
        assert Hin * Win == U.shape[1]
    Ho, Wo = out_hw
    assert theta.shape == (N, 6)
    if out is None:
        out = torch.empty((N, Ho * Wo), device=U.device, dtype=torch.float32)
    assert out.numel() == N * Ho * Wo and out.is_contiguous()
    if accumulate:
        assert z is not None and mask is not None and z.shape == (N,) and mask.shape == (N,)
        assert out.dtype == torch.float32
        mode = 1
    else:
        mode = 2 if out.dtype == torch.bfloat16 else 0
    _ops.stn_forward_(U, N, Hin, Win, theta, Ho, Wo, out, z, mask, mode, period)
    return out


BF_STORE, BF_SOFTPLUS, BF_SIGMOID_NOISE, BF_SOFTPLUS_BWD, BF_ATOMIC = 0, 1, 2, 3, 4


def gemm_bf16(A, B, C, M: int, N: int, K: int, lda: int, ldb: int, ldc: int, tn=False,
              epi=BF_STORE, bias=None, Cin=None, aux=None, ldaux=0, aux_scale=0.0, splitk=1,
              colsum=None) -> None:
    """Batched bf16-operand MFMA GEMM (see mog_gemm_bf16); output dtype is C's."""
    nb = len(C)
    assert len(A) == nb and len(B) == nb and 1 <= nb <= 8
    _ops.gemm_bf16_(list(A), list(B), list(C), _opt_list(bias), _opt_list(Cin), _opt_list(aux),
                    _opt_list(colsum), M, N, K, lda, ldb, ldc, ldaux, bool(tn), epi,
                    float(aux_scale), int(splitk))


def stn_backward(U: torch.Tensor, theta: torch.Tensor, out_hw, G: torch.Tensor,
                 gscale: Optional[torch.Tensor] = None, want_dU=True, want_dtheta=True,
                 want_dot=False, dU=None, dtheta=None, dot=None, n: Optional[int] = None,
                 dm: Optional[torch.Tensor] = None, dm_bf16: Optional[torch.Tensor] = None):
    """Gradient of transformer().  ``n`` images (default U's); when U or G
    holds fewer rows than ``n``, image i reads row i % rows (several loop
    steps of one batch against the shared canvas or canvas gradient).

    ``dm`` (bf16 or fp32 [N, Hin*Win], U = the VAE output sigmoid r): the
    input gradient is taken on through the sigmoid (vae.py:44-46) and stored
    there instead of dU -- bit-identical to dU followed by
    mog_sigmoid_backward.  (``dm_bf16``: the same, kept as an alias.)"""
    _chk(U, "U")
    _chk(G, "G")
    if dm is None:
        dm = dm_bf16
    if U.dim() == 3:
        Hin, Win = U.shape[1], U.shape[2]
    else:
        Hin = Win = int(round(U.shape[1] ** 0.5))
    Ho, Wo = out_hw
    NU, NG = U.numel() // (Hin * Win), G.numel() // (Ho * Wo)
    N = NU if n is None else int(n)
    assert N % NU == 0 and N % NG == 0 and theta.numel() == 6 * N
    dev = U.device
    if dm is not None:
        assert want_dU and dU is None and NU == N
        assert dm.numel() >= N * Hin * Win
        _chk(dm, "dm", dm.dtype if dm.dtype in (torch.bfloat16, torch.float32) else None)
        if want_dtheta and dtheta is None:
            dtheta = torch.empty((N, 6), device=dev, dtype=torch.float32)
        if want_dot and dot is None:
            dot = torch.empty((N,), device=dev, dtype=torch.float32)
        _ops.stn_backward_sigmoid_(U, N, Hin, Win, theta, Ho, Wo, G, gscale, dm,
                                   dtheta if want_dtheta else None, dot if want_dot else None,
                                   NG if NG < N else 0)
        return dm, dtheta, dot
    if want_dU and dU is None:
        dU = torch.empty((N, Hin * Win), device=dev, dtype=torch.float32)
    if want_dtheta and dtheta is None:
        dtheta = torch.empty((N, 6), device=dev, dtype=torch.float32)
    if want_dot and dot is None:
        dot = torch.empty((N,), device=dev, dtype=torch.float32)
    _ops.stn_backward_(U, N, Hin, Win, theta, Ho, Wo, G, gscale, dU if want_dU else None,
                       dtheta if want_dtheta else None, dot if want_dot else None,
                       NU if NU < N else 0, NG if NG < N else 0)
    return dU, dtheta, dot


def _i64(v: int) -> int:
    """a 64-bit counter / seed as the signed int64 of an op schema's `int`"""
    v &= 2 ** 64 - 1
    return v - 2 ** 64 if v >= 2 ** 63 else v


def rng_fill(out: torch.Tensor, seed: int, offset: int, normal: bool) -> None:
    _chk(out, "out")
    _ops.rng_fill_(out, _i64(seed), _i64(offset), bool(normal))


def spin(ticks: int, device=None) -> None:
    """Hold the current stream for `ticks` of the 100 MHz wall clock (test
    instrument mog_spin of libmog_air_test.so)."""
    if ticks == 0:
        return
    rc = _lib.load_test().mog_spin(int(ticks), stream_ptr())
    if rc != 0:
        raise _lib.MogError(f"mog_spin failed ({rc})")


def lds_poison(bits: int = 0x7FC00000) -> None:
    """Fill every CU's LDS with a 32-bit pattern on the current stream (test
    instrument mog_lds_poison of libmog_air_test.so; default a quiet NaN)."""
    rc = _lib.load_test().mog_lds_poison(int(bits) & 0xFFFFFFFF, stream_ptr())
    if rc != 0:
        raise _lib.MogError(f"mog_lds_poison failed ({rc})")
