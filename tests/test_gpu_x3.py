"""The fp32 weight-gradient GEMM on the bf16 matrix cores (csrc/gemm_x3.hip,
mog_gemm_f32_x3_tn): C += A^T B with every operand split exactly into three
bf16 pieces.  Bar: fp32-level accuracy -- the error against a float64 product,
normalised by |A|^T |B|, within 1e-6 everywhere and no larger than 2x the
error of the fp32 MFMA chain (mog_gemm_f32, the form it replaces for the
LSTM x-part gradient, air_model.py:454-456) on the same operands; column sums
of B within the same bound.  Ragged shapes, split-K counts, a column window of
a wider operand (the data-parallel row chunks) and a wide exponent range (the
exact split must hold for every binade)."""
import numpy as np
import pytest
import torch

from mog_air import ops

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _case(M, N, K, lda, ldb, spread, seed):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(K, lda, generator=g, dtype=torch.float64)
    B = torch.randn(K, ldb, generator=g, dtype=torch.float64)
    if spread:
        A *= torch.exp2(torch.randint(-spread, spread + 1, A.shape, generator=g).double())
        B *= torch.exp2(torch.randint(-spread, spread + 1, B.shape, generator=g).double())
    return A.float(), B.float()


def _err(got, ref, scale):
    return float(((got.double() - ref).abs() / (scale + 1e-300)).max())


@pytest.mark.parametrize("M,N,K,lda,ldb,m0,splitk,spread", [
    (2500, 1024, 8192, 2500, 1024, 0, 8, 0),     # the x-part gradient of the bench step
    (640, 1024, 4096, 2500, 1024, 1280, 4, 0),   # a data-parallel row chunk (column window)
    (132, 36, 77, 136, 36, 0, 1, 0),             # ragged tiles, K not a multiple of 32
    (260, 200, 999, 260, 200, 0, 3, 12),         # exponent spread 2^-12 .. 2^12
    (128, 128, 32, 128, 128, 0, 16, 0),          # more splits than k-tiles
    (4, 4, 1, 4, 4, 0, 1, 0),
])
def test_x3_accuracy(M, N, K, lda, ldb, m0, splitk, spread):
    A, B = _case(M, N, K, lda, ldb, spread, seed=M + N + K)
    Ad, Bd = A.to(DEV), B.to(DEV)
    ref = A[:, m0:m0 + M].double().T @ B[:, :N].double()
    scale = A[:, m0:m0 + M].double().abs().T @ B[:, :N].double().abs()
    C0 = torch.randn(M, N, generator=torch.Generator().manual_seed(1)).float()
    C = C0.to(DEV)
    cs0 = torch.randn(N, generator=torch.Generator().manual_seed(2)).float()
    cs = cs0.to(DEV)
    ops.gemm_x3_tn(Ad[:, m0:], Bd, C, M, N, K, lda, ldb, N, splitk=splitk, colsum=cs)
    torch.cuda.synchronize()
    e_x3 = _err(C.cpu() - C0, ref, scale + C0.double().abs())
    # the pre-split form: pieces in HBM (row pitch padded to 8), same product
    p8 = lambda n: (n + 7) // 8 * 8  # noqa: E731
    A3 = torch.empty(3, K, p8(lda), device=DEV, dtype=torch.bfloat16)
    B3 = torch.empty(3, K, p8(ldb), device=DEV, dtype=torch.bfloat16)
    ops.split3_bf16(Ad, A3, K, lda, lda, p8(lda), K * p8(lda))
    ops.split3_bf16(Bd, B3, K, ldb, ldb, p8(ldb), K * p8(ldb))
    # the split is exact: the pieces sum back to the operand
    assert torch.equal(((A3[0].float() + A3[1].float()) + A3[2].float())[:, :lda].cpu(), A)
    assert bool((A3[:, :, lda:] == 0).all())
    Cp = C0.to(DEV)
    csp = cs0.to(DEV)
    if m0 % 8 == 0:
        ops.gemm_x3p_tn(A3.view(-1)[m0:], K * p8(lda), B3, K * p8(ldb), Cp, M, N, K, p8(lda),
                        p8(ldb), N, splitk=splitk, colsum=csp)
        torch.cuda.synchronize()
        e_p = _err(Cp.cpu() - C0, ref, scale + C0.double().abs())
        assert e_p <= 1e-6, e_p
        cref_p = B[:, :N].double().sum(0)
        assert _err(csp.cpu() - cs0, cref_p, B[:, :N].double().abs().sum(0) + cs0.double().abs()) \
            <= 1e-6
    # the fp32 MFMA chain (split-K atomics) on the same operands
    C32 = C0.to(DEV)
    ops.gemm([Ad[:, m0:]], [Bd], [C32], M, N, K, lda, ldb, N, transA=True, epi=ops.EPI_ATOMIC,
             splitk=max(1, min(K // 256, 4)))
    torch.cuda.synchronize()
    e_32 = _err(C32.cpu() - C0, ref, scale + C0.double().abs())
    assert e_x3 <= 1e-6, (e_x3, e_32)
    assert e_x3 <= 2 * e_32 + 1e-7, (e_x3, e_32)
    cref = B[:, :N].double().sum(0)
    cscale = B[:, :N].double().abs().sum(0)
    assert _err(cs.cpu() - cs0, cref, cscale + cs0.double().abs()) <= 1e-6


def test_x3_zero_extents_and_checks():
    A = torch.zeros(8, 8, device=DEV)
    C = torch.ones(8, 8, device=DEV)
    ops.gemm_x3_tn(A, A, C, 8, 8, 0, 8, 8, 8)     # K = 0: no launch, C unchanged
    torch.cuda.synchronize()
    assert bool((C == 1).all())
    with pytest.raises(RuntimeError):
        ops.gemm_x3_tn(A, A, C, 6, 8, 8, 8, 8, 8)  # M not a multiple of 4
    with pytest.raises(RuntimeError):
        ops.gemm_x3_tn(A[:, 1:], A, C, 4, 8, 8, 8, 8, 8)  # A not 16-byte aligned


def test_x3_fp32_step_gradients_match_chain():
    """The whole fp32 train step's gradients with the x3 x-part gradient (in-
    kernel split and pre-split) and the x3 VAE weight gradients, and with the
    fp32 chain, agree to fp32 level (every gradient)."""
    from mog_air.air_model import AIRModel
    rng = np.random.default_rng(5)
    # 1024 images: 3072 rows, past AIRModel.X3_MIN_ROWS, so the VAE's x3
    # weight gradients run too; the input gradients' NT form is let in from
    # 2048 rows here (the model gates it at X3_DX_MIN_ROWS)
    x = (rng.uniform(size=(1024, 2500)) * (rng.uniform(size=(1024, 2500)) < 0.3)).astype(np.float32)
    grads = []
    for x3 in (1, 2, 0, 0):
        m = AIRModel(max_steps=3, max_digits=3, canvas_size=50, scale_prior_variance=0.05,
                     z_pres_prior_log_odds=-0.01, cnn=False, train=True, scope="x3",
                     device=DEV, precision="fp32", seed=3, noise_seed=4)
        m.X_GRAD_X3 = x3
        # (the VAE gradients' and the recurrent rows' x3 forms ride along)
        m.VAE_WGRAD_X3 = m.VAE_DX_X3 = m.REC_WGRAD_X3 = x3 != 0
        m.X3_DX_MIN_ROWS = 2048
        # one k pass per weight gradient: no split-K atomics, so each form is
        # reproducible and the forms differ by their products' summation only
        m.ONE_PASS_WGRADS = True
        assert 3 * 1024 >= m.X3_MIN_ROWS
        grads.append({k: torch.as_tensor(np.asarray(v), dtype=torch.float64)
                      for k, v in m.compute_gradients(x).items()})
    for k in grads[2]:  # the chain against itself: bit for bit
        assert torch.equal(grads[3][k], grads[2][k]), k
    # fp32-level agreement per tensor, in the 2-norm (the x3 forms' products
    # are summed in another order than the fp32 chain's, and the differences
    # travel the whole backward chain, where gradients that are sums with
    # heavy cancellation, e.g. the heads' bias column sums, move most), and
    # elementwise within 1e-5 of the tensor's largest entry
    for g in (grads[0], grads[1]):
        for k in g:
            a, b = g[k], grads[2][k]
            nb = b.norm().item() + 1e-30
            # (tensors of a few entries: each entry one long column sum)
            tol = 2e-5 if b.numel() > 64 else 2e-4
            assert (a - b).norm().item() <= tol * nb, k
            assert (a - b).abs().max().item() <= 1e-5 * (b.abs().max().item() + 1e-30), k


@pytest.mark.parametrize("M,N,K,m0,splitk", [(2500, 1024, 4096, 0, 8), (580, 1024, 777, 1920, 1),
                                             (132, 40, 300, 0, 2)])
def test_x1_plain_bf16_operands(M, N, K, m0, splitk):
    """npieces = 1 (the bf16 configuration's x-rows gradient): plain bf16
    operands, one product; exact bf16 products accumulated in fp32, so within
    1e-6 of |A|^T |B| of the float64 product of the same bf16 values, and the
    column sums of the bf16 B likewise."""
    lda = (m0 + M + 7) // 8 * 8
    g = torch.Generator().manual_seed(K)
    A = torch.randn(K, lda, generator=g).bfloat16()
    B = torch.randn(K, N, generator=g).bfloat16()
    C = torch.zeros(M, N, device=DEV)
    cs = torch.zeros(N, device=DEV)
    ops.gemm_x3p_tn(A.to(DEV).view(-1)[m0:], 0, B.to(DEV), 0, C, M, N, K, lda, N, N,
                    splitk=splitk, colsum=cs, npieces=1)
    torch.cuda.synchronize()
    Ad, Bd = A[:, m0:m0 + M].double(), B.double()
    assert _err(C.cpu(), Ad.T @ Bd, Ad.abs().T @ Bd.abs()) <= 1e-6
    assert _err(cs.cpu(), Bd.sum(0), Bd.abs().sum(0)) <= 1e-6


def test_x3_asr_step_gradients_match_chain():
    """AIR-ASR (configs[2]) from B = 1024: the inference LSTM's x-rows
    gradient on the three-piece bf16 form (X split on the side stream under the
    x-projection) and the per-step VAE input gradients on the NT x3 form (let
    in from 1024 rows here; the model gates it at X3_DX_MIN_ROWS = the bench's
    8,192 per step) against the fp32 chain: every gradient to fp32 level."""
    import bench
    rng = np.random.default_rng(6)
    B = 1024
    x = (rng.uniform(size=(B, 2500)) * (rng.uniform(size=(B, 2500)) < 0.3)).astype(np.float32)
    X = torch.as_tensor(x).to(DEV)
    grads = []
    for x3 in (2, 0):
        m = bench.make_asr_model("fp32", torch.device(DEV), "x3asr%d" % x3)
        m.X_GRAD_X3 = x3
        m.VAE_DX_X3 = m.REC_WGRAD_X3 = x3 != 0
        m.X3_DX_MIN_ROWS = 1024
        assert m._x3_asr(B) == (x3 == 2)
        grads.append({k: torch.as_tensor(np.asarray(v), dtype=torch.float64)
                      for k, v in m.compute_gradients(X).items()})
    for k in grads[0]:  # (the 2-norm bound of test_x3_fp32_step_gradients_match_chain)
        a, b = grads[0][k], grads[1][k]
        tol = 2e-5 if b.numel() > 64 else 2e-4
        assert (a - b).norm().item() <= tol * (b.norm().item() + 1e-30), k
        assert (a - b).abs().max().item() <= 1e-4 * (b.abs().max().item() + 1e-30), k


@pytest.mark.parametrize("M,N,K,epi", [(777, 512, 784, 1), (300, 784, 512, 0), (129, 256, 512, 1),
                                       (64, 512, 256, 1), (5, 4, 8, 0)])
def test_x3_nt_accuracy(M, N, K, epi):
    """mog_gemm_x3_nt (the VAE input gradients dY W^T, optional softplus
    backward from the softplus output) against float64: error <= 1e-6 of |A||B|^T (the fp32 chain's
    level; test_x3_accuracy's gate) with ragged M / N tiles."""
    from mog_air import ops
    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((M, K)).astype(np.float32)
    W = (rng.standard_normal((N, K)) * np.exp2(rng.integers(-6, 6, (N, 1)))).astype(np.float32)
    # aux = the softplus output of the layer (epi 1 takes sigmoid(x) as
    # 1 - exp(-softplus(x))): pre-activations over a wide range
    pre = (rng.standard_normal((M, N)) * 4).astype(np.float32)
    aux = np.log1p(np.exp(pre.astype(np.float64))).astype(np.float32)
    At, Wt = torch.as_tensor(A).to(DEV), torch.as_tensor(W).to(DEV)
    W3 = torch.empty((3, N, K), device=DEV, dtype=torch.bfloat16)
    ops.split3_bf16(Wt, W3, N, K, K, K, N * K)
    C = torch.full((M, N), float("nan"), device=DEV)
    ops.gemm_x3_nt(At, W3, N * K, C, M, N, K, K, K, N,
                   aux=torch.as_tensor(aux).to(DEV) if epi else None, ldaux=N if epi else 0)
    ref = A.astype(np.float64) @ W.astype(np.float64).T
    bound = np.abs(A).astype(np.float64) @ np.abs(W).astype(np.float64).T
    if epi:
        sig = -np.expm1(-aux.astype(np.float64))
        ref, bound = ref * sig, bound * sig
    err = np.abs(C.cpu().numpy().astype(np.float64) - ref)
    assert np.isfinite(C.cpu().numpy()).all()
    assert (err <= 1e-6 * bound + 1e-30).all(), float((err / (bound + 1e-30)).max())


@pytest.mark.parametrize("npieces", [1, 3])
def test_x3p_splitk_reduce_deterministic(npieces):
    """Split-K through the workspace (reduce=True, the default): the partials
    are added in split order, so two launches give the same bits, and they
    agree with the float-atomic form (reduce=False) to fp32 level."""
    M, N, K = 300, 260, 3000
    g = torch.Generator().manual_seed(7)
    A = torch.randn(K, 304, generator=g).to(DEV)
    B = torch.randn(K, N, generator=g).to(DEV)
    A3 = torch.empty(3, K, 304, device=DEV, dtype=torch.bfloat16)
    B3 = torch.empty(3, K, 264, device=DEV, dtype=torch.bfloat16)
    ops.split3_bf16(A, A3, K, 304, 304, 304, K * 304)
    ops.split3_bf16(B, B3, K, N, N, 264, K * 264)
    outs, sums = [], []
    for red in (True, True, False):
        C = torch.ones(M, N, device=DEV)
        cs = torch.ones(N, device=DEV)
        ops.gemm_x3p_tn(A3.view(-1), K * 304, B3, K * 264, C, M, N, K, 304, 264, N, splitk=7,
                        colsum=cs, npieces=npieces, reduce=red)
        torch.cuda.synchronize()
        outs.append(C.cpu())
        sums.append(cs.cpu())
    assert torch.equal(outs[0], outs[1])
    # the column sums (the bias gradient) too: per-split partials added in
    # split order by the reduce launch, no float atomics
    assert torch.equal(sums[0], sums[1])
    assert float((outs[0] - outs[2]).abs().max()) <= 1e-5 * float(outs[2].abs().max())
    Bd = (B3[0].double() + B3[1].double() + B3[2].double())[:, :N] if npieces == 3 else \
        B3[0].double()[:, :N]
    ref = 1.0 + Bd.sum(0).cpu()
    assert float((sums[0].double() - ref).abs().max()) <= 1e-6 * float(Bd.abs().sum(0).max())


def test_x3_tn_splitk_reduce_deterministic_colsum():
    """The in-kernel-split TN form through the workspace: C and the column
    sums bit-identical over two launches, and against float64."""
    M, N, K = 260, 300, 5000
    g = torch.Generator().manual_seed(8)
    A = torch.randn(K, M, generator=g).to(DEV)
    B = torch.randn(K, N, generator=g).to(DEV)
    res = []
    for _ in range(2):
        C = torch.zeros(M, N, device=DEV)
        cs = torch.zeros(N, device=DEV)
        ops.gemm_x3_tn(A, B, C, M, N, K, M, N, N, splitk=9, colsum=cs, reduce=True)
        torch.cuda.synchronize()
        res.append((C.cpu(), cs.cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    Ad, Bd = A.double().cpu(), B.double().cpu()
    assert _err(res[0][0], Ad.T @ Bd, Ad.abs().T @ Bd.abs()) <= 1e-6
    assert _err(res[0][1], Bd.sum(0), Bd.abs().sum(0)) <= 1e-6
