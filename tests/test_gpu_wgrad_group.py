"""The grouped fp32 weight-gradient launch (csrc/gemm_group.hip,
mog_gemm_f32_wgrad_group; mog_air.ops.WgradGroup): every problem's C += A^T B
and column sums of B against float64, fp32-level (the gate of
test_gpu_x3.py), on ragged shapes (M, N not multiples of the 64 x 64 tile or of
4, K not a multiple of 16), column windows of wider operands, and problems
sharing operands; and the batch-64 train step with the group against the same
step with one launch per gradient (MOG_WGRAD_GROUP=0's path)."""
import numpy as np
import pytest
import torch

from mog_air import ops

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _err(got, ref, scale):
    return float(((got.double() - ref).abs() / (scale + 1e-300)).max())


def test_wgrad_group_matches_float64():
    g = torch.Generator().manual_seed(3)
    shapes = [  # M, N, K, lda, ldb, bias
        (784, 512, 192, 784, 512, True),
        (256, 50, 192, 256, 50, True),
        (50, 256, 192, 56, 256, False),
        (64, 1, 190, 64, 2, True),
        (2500, 1024, 64, 2500, 1024, True),
        (3, 5, 17, 7, 9, True),
        (130, 70, 1, 130, 70, False),
    ]
    grp = ops.WgradGroup()
    cases = []
    for M, N, K, lda, ldb, bias in shapes:
        A = torch.randn(K, lda, generator=g).to(DEV)
        B = torch.randn(K, ldb, generator=g).to(DEV)
        C0 = torch.randn(M, N, generator=g)
        C = C0.to(DEV)
        b0 = torch.randn(N, generator=g)
        b = b0.to(DEV) if bias else None
        grp.add(A, B, C, M, N, K, lda, ldb, N, b)
        cases.append((A, B, C, C0, b, b0, M, N))
    grp.launch()
    torch.cuda.synchronize()
    for A, B, C, C0, b, b0, M, N in cases:
        Ad, Bd = A.cpu().double()[:, :M], B.cpu().double()[:, :N]
        ref = C0.double() + Ad.T @ Bd
        assert _err(C.cpu(), ref, Ad.abs().T @ Bd.abs() + C0.double().abs()) <= 1e-6
        if b is not None:
            assert _err(b.cpu(), b0.double() + Bd.sum(0), Bd.abs().sum(0) + b0.double().abs()) <= 1e-6


def test_wgrad_group_is_deterministic_and_checks_extents():
    g = torch.Generator().manual_seed(4)
    A = torch.randn(192, 300, generator=g).to(DEV)
    B = torch.randn(192, 200, generator=g).to(DEV)
    grp = ops.WgradGroup()
    C1 = torch.zeros(300, 200, device=DEV)
    C2 = torch.zeros(300, 200, device=DEV)
    for C in (C1, C2):
        grp.add(A, B, C, 300, 200, 192, 300, 200, 200)
        grp.launch()
    torch.cuda.synchronize()
    assert torch.equal(C1, C2)
    with pytest.raises(RuntimeError):
        grp.add(A, B, torch.zeros(10, 10, device=DEV), 300, 200, 192, 300, 200, 200)


def test_batch64_step_grouped_matches_per_gradient_launches():
    """The reference's batch of 64: the step's gradients with the grouped
    launch and with one launch per gradient agree to fp32 level (one k pass
    each: the two differ by the products' summation order only)."""
    from mog_air.air_model import AIRModel
    rng = np.random.default_rng(9)
    x = (rng.uniform(size=(64, 2500)) * (rng.uniform(size=(64, 2500)) < 0.3)).astype(np.float32)
    grads = []
    for grouped in (True, False, True):
        m = AIRModel(max_steps=3, max_digits=3, canvas_size=50, scale_prior_variance=0.05,
                     z_pres_prior_log_odds=-0.01, cnn=False, train=True, scope="wg%d" % grouped,
                     device=DEV, precision="fp32", seed=3, noise_seed=4)
        m.WGRAD_GROUP = grouped
        m.ONE_PASS_WGRADS = True
        grads.append({k: torch.as_tensor(np.asarray(v), dtype=torch.float64)
                      for k, v in m.compute_gradients(x).items()})
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[2][k]), k  # the group is deterministic
        a, b = grads[0][k], grads[1][k]
        tol = 2e-5 if b.numel() > 64 else 2e-4
        assert (a - b).norm().item() <= tol * (b.norm().item() + 1e-30), k


def test_wgrad_group_shared_outputs_accumulate_in_order():
    """Two problems adding into the same output (and bias): they go to
    successive launches, so both products land."""
    g = torch.Generator().manual_seed(5)
    A1, A2 = (torch.randn(100, 70, generator=g).to(DEV) for _ in range(2))
    B1, B2 = (torch.randn(100, 40, generator=g).to(DEV) for _ in range(2))
    C = torch.zeros(70, 40, device=DEV)
    b = torch.zeros(40, device=DEV)
    grp = ops.WgradGroup()
    grp.add(A1, B1, C, 70, 40, 100, 70, 40, 40, b)
    grp.add(A2, B2, C[10:], 60, 40, 100, 70, 40, 40, b)  # rows 10.. of the same output
    grp.launch()
    torch.cuda.synchronize()
    ref = A1.cpu().double().T @ B1.cpu().double()
    ref[10:] += A2.cpu().double()[:, :60].T @ B2.cpu().double()
    scale = A1.cpu().double().abs().T @ B1.cpu().double().abs()
    scale[10:] += A2.cpu().double()[:, :60].abs().T @ B2.cpu().double().abs()
    assert _err(C.cpu(), ref, scale) <= 1e-6
    bref = B1.cpu().double().sum(0) + B2.cpu().double().sum(0)
    assert _err(b.cpu(), bref, B1.cpu().double().abs().sum(0) + B2.cpu().double().abs().sum(0)) <= 1e-6


def test_asr_batch64_step_grouped_matches_per_gradient_launches():
    """AIR-ASR (configs[2]) at the reference's batch of 64: grouped against
    one launch per gradient, every gradient to fp32 level."""
    import bench
    rng = np.random.default_rng(10)
    x = (rng.uniform(size=(64, 2500)) * (rng.uniform(size=(64, 2500)) < 0.3)).astype(np.float32)
    X = torch.as_tensor(x).to(DEV)
    grads = []
    for grouped in (True, False):
        m = bench.make_asr_model("fp32", torch.device(DEV), "wgasr%d" % grouped)
        m.WGRAD_GROUP = grouped
        m.ONE_PASS_WGRADS = True
        grads.append({k: torch.as_tensor(np.asarray(v), dtype=torch.float64)
                      for k, v in m.compute_gradients(X).items()})
    for k in grads[0]:
        a, b = grads[0][k], grads[1][k]
        tol = 2e-5 if b.numel() > 64 else 2e-4
        assert (a - b).norm().item() <= tol * (b.norm().item() + 1e-30), k


def test_wgrad_group_op_schema_and_extents():
    """torch.ops.mog_air.gemm_f32_wgrad_group_ takes tensors (out / bias
    alias-annotated as written, opcheck's schema test) and checks each
    problem's extents in C++: an output too small for its M x N is refused
    before anything launches."""
    from torch.library import opcheck
    op = torch.ops.mog_air.gemm_f32_wgrad_group_
    g = torch.Generator().manual_seed(6)
    A = torch.randn(64, 48, generator=g).to(DEV)
    B = torch.randn(64, 32, generator=g).to(DEV)
    C = torch.zeros(48, 32, device=DEV)
    b = torch.zeros(32, device=DEV)
    opcheck(op.default, ([A], [B], [C], [b], [48, 32, 64, 48, 32, 32]),
            test_utils=("test_schema",))
    with pytest.raises(RuntimeError, match="out"):
        op([A], [B], [torch.zeros(10, 32, device=DEV)], [None], [48, 32, 64, 48, 32, 32])
    with pytest.raises(RuntimeError, match="dY"):
        op([A], [B[:8].clone()], [C], [None], [48, 32, 64, 48, 32, 32])
