"""The grouped tall-K bf16 weight-gradient kernel (csrc/wgrad_tn.hip,
mog_wgrad_tn_bf16; the MatMul / BiasAdd gradients of air/vae.py:18-46 over
T*B rows in the bf16 configuration): every problem's out += X^T dY and
colsum += column sums of dY against a float64 product of the same bf16
values, ragged shapes (M, N off the 128 tile, the 50-wide latent layers with
their 56-element pitch, K off the 32-row k-tile), accumulation onto existing
values, bitwise determinism, and the XCD-split and plain split mappings."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

from mog_air import ops  # noqa: E402


def _problems(K, shapes, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for M, N, lda, ldb in shapes:
        X = torch.zeros(K, lda)
        X[:, :M] = torch.randn(K, M, generator=g)
        dY = torch.zeros(K, ldb)
        dY[:, :N] = torch.randn(K, N, generator=g) * 0.1
        out.append((X.to(torch.bfloat16).to(DEV), dY.to(torch.bfloat16).to(DEV), M, N, lda, ldb))
    return out


def _run(probs, K, nsplit, C0=None, b0=None):
    Cs = [torch.zeros(M, N, device=DEV) if C0 is None else C0[i].clone()
          for i, (_, _, M, N, _, _) in enumerate(probs)]
    bs = [torch.zeros(N, device=DEV) if b0 is None else b0[i].clone()
          for i, (_, _, _, N, _, _) in enumerate(probs)]
    ops.wgrad_tn_bf16([p[0] for p in probs], [p[1] for p in probs], Cs, bs,
                      [(M, N, lda, ldb, N) for _, _, M, N, lda, ldb in probs], K, nsplit)
    torch.cuda.synchronize()
    return Cs, bs


def _check(probs, Cs, bs, C0=None, b0=None):
    for i, (X, dY, M, N, _, _) in enumerate(probs):
        Xd, Yd = X.double().cpu()[:, :M], dY.double().cpu()[:, :N]
        ref = Xd.t() @ Yd + (0 if C0 is None else C0[i].double().cpu())
        scale = Xd.abs().t() @ Yd.abs() + 1e-30
        err = ((Cs[i].double().cpu() - ref).abs() / scale).max().item()
        assert err <= 1e-5, (i, err)
        bref = Yd.sum(0) + (0 if b0 is None else b0[i].double().cpu())
        berr = ((bs[i].double().cpu() - bref).abs() / (Yd.abs().sum(0) + 1e-30)).max().item()
        assert berr <= 1e-5, (i, berr)


# the bf16 VAE's seven layers (C = 50: 784 / 512 / 256 / 50 with the latent
# pitch 56) and ragged extras
VAE = [(784, 512, 784, 512), (512, 256, 512, 256), (256, 50, 256, 56), (256, 50, 256, 56),
       (50, 256, 56, 256), (256, 512, 256, 512), (512, 784, 512, 784)]


@pytest.mark.parametrize("K,nsplit", [(3000, 8), (1000, 3), (4099, 16)])
def test_wgrad_tn_matches_float64(K, nsplit):
    probs = _problems(K, VAE, seed=K)
    Cs, bs = _run(probs, K, nsplit)
    _check(probs, Cs, bs)


def test_wgrad_tn_ragged_accumulates_and_is_deterministic():
    K = 777
    shapes = [(130, 70, 136, 72), (8, 300, 8, 304), (200, 129, 200, 136)]
    probs = _problems(K, shapes, seed=3)
    g = torch.Generator().manual_seed(4)
    C0 = [torch.randn(M, N, generator=g).to(DEV) for _, _, M, N, _, _ in probs]
    b0 = [torch.randn(N, generator=g).to(DEV) for _, _, _, N, _, _ in probs]
    Cs, bs = _run(probs, K, 8, C0, b0)
    _check(probs, Cs, bs, C0, b0)
    Cs2, bs2 = _run(probs, K, 8, C0, b0)
    for a, b in zip(Cs + bs, Cs2 + bs2):
        assert torch.equal(a, b)


def test_wgrad_tn_checks_extents():
    probs = _problems(64, [(64, 64, 64, 64)], seed=5)
    X, dY = probs[0][0], probs[0][1]
    with pytest.raises(RuntimeError, match="dY"):
        ops.wgrad_tn_bf16([X], [dY[:32].clone()], [torch.zeros(64, 64, device=DEV)], [None],
                          [(64, 64, 64, 64, 64)], 64, 8)
    with pytest.raises(RuntimeError, match="out"):
        ops.wgrad_tn_bf16([X], [dY], [torch.zeros(10, 64, device=DEV)], [None],
                          [(64, 64, 64, 64, 64)], 64, 8)


@pytest.mark.parametrize("K,nsplit", [(2500, 8), (1001, 7)])
def test_wgrad_tn_x3_matches_float64(K, nsplit):
    """The fp32 form (mog_wgrad_tn_x3: exact three-piece splits, six
    products): fp32-level accuracy against a float64 product of the fp32
    operands -- the fp32 configuration's four large VAE layers plus ragged
    shapes -- accumulated onto existing values, and bitwise deterministic."""
    shapes = [(784, 512, 784, 512), (512, 256, 512, 256), (256, 512, 256, 512),
              (512, 784, 512, 784), (132, 68, 136, 72)]
    g = torch.Generator().manual_seed(K)
    Xs = [torch.randn(K, lda, generator=g).to(DEV) for _, _, lda, _ in shapes]
    Ys = [(torch.randn(K, ldb, generator=g) * 1e-2).to(DEV) for _, _, _, ldb in shapes]
    C0 = [torch.randn(M, N, generator=g).to(DEV) for M, N, _, _ in shapes]
    b0 = [torch.randn(N, generator=g).to(DEV) for _, N, _, _ in shapes]
    res = []
    for _ in range(2):
        Cs = [c.clone() for c in C0]
        bs = [b.clone() for b in b0]
        ops.wgrad_tn_x3(Xs, Ys, Cs, bs, [(M, N, lda, ldb, N) for M, N, lda, ldb in shapes], K,
                        nsplit)
        torch.cuda.synchronize()
        res.append((Cs, bs))
    for a, b in zip(res[0][0] + res[0][1], res[1][0] + res[1][1]):
        assert torch.equal(a, b)
    Cs, bs = res[0]
    for i, (M, N, _, _) in enumerate(shapes):
        Xd, Yd = Xs[i].double().cpu()[:, :M], Ys[i].double().cpu()[:, :N]
        ref = Xd.t() @ Yd + C0[i].double().cpu()
        scale = Xd.abs().t() @ Yd.abs() + C0[i].double().cpu().abs()
        assert ((Cs[i].double().cpu() - ref).abs() / scale).max().item() <= 1e-5, i
        bref = Yd.sum(0) + b0[i].double().cpu()
        bscale = Yd.abs().sum(0) + b0[i].double().cpu().abs()
        assert ((bs[i].double().cpu() - bref).abs() / bscale).max().item() <= 1e-5, i


def test_heads_output_wgrad_vs_float64_and_deterministic():
    """mog_heads_output_wgrad (the heads' 1- / 2-column output layers,
    air_model.py:462-499 backward): gw += hid^T dout[:, :k], gb += colsum,
    within 1e-5 of float64 (fp32 sums of 128-row chunks) and bitwise equal across launches; the
    unused column of a 1-column head is ignored; a ragged last chunk."""
    import mog_air.torch_ops  # noqa: F401
    ops = torch.ops.mog_air
    g = torch.Generator().manual_seed(5)
    R, HS, ks = 3000, 64, [1, 1, 2, 2, 1]
    hid = [torch.randn(R, HS, generator=g).to(DEV) for _ in ks]
    dout = [torch.randn(R, 2, generator=g).to(DEV) for _ in ks]
    gw0 = [(torch.randn(HS, k, generator=g) * 0.1).to(DEV) for k in ks]
    gb0 = [(torch.randn(k, generator=g) * 0.1).to(DEV) for k in ks]
    outs = []
    for _ in range(2):
        gw = [w.clone() for w in gw0]
        gb = [b.clone() for b in gb0]
        ops.heads_output_wgrad_(hid, dout, gw, gb, ks, R, HS)
        torch.cuda.synchronize()
        outs.append((gw, gb))
    for z, k in enumerate(ks):
        want_w = gw0[z].double() + hid[z].double().T @ dout[z][:, :k].double()
        want_b = gb0[z].double() + dout[z][:, :k].double().sum(0)
        got_w, got_b = outs[0][0][z], outs[0][1][z]
        assert torch.linalg.norm(got_w.double() - want_w) <= 1e-5 * torch.linalg.norm(want_w)
        assert torch.linalg.norm(got_b.double() - want_b) <= 1e-5 * torch.linalg.norm(want_b)
        assert torch.equal(outs[0][0][z], outs[1][0][z]) and torch.equal(outs[0][1][z], outs[1][1][z])
