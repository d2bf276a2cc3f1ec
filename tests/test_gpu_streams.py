"""Stream ordering of the forked train step, made deterministic.

From B = 1024 (AIRModel.SIDE_MIN_BATCH) the step forks work onto a side
stream and a third stream: the noise fills, loop-state resets and operand
splits under the x-projection, the VAE / heads / recurrent-rows weight
gradients under the backward's latency-bound chain (AIR), the per-loop-step
VAE and recurrent-rows gradients and the heads' gradients (AIR-ASR).  A fork
without its wait, a join without its event, or a buffer that the main stream
overwrites while the other stream still reads it would show only as a rare
timing accident.  Here a spin kernel (mog_spin) holds one side back for 20 ms:

* SPIN_MAIN at the head of the step's main stream: every forked segment that
  does not wait for its producers runs first, on the previous step's buffers;
* SPIN_FORK at the head of every forked segment: every main-stream consumer
  that does not wait for the segment (the dh GEMM's W1 pack, the x-rows
  gradient's X pieces, Adam's gradients) runs first, and every buffer the
  main stream rewrites before the join is rewritten under the segment.

The previous train step runs on a different batch, so a stale read sees other
values.  ONE_PASS_WGRADS makes every weight gradient one k pass (one atomic
add per element onto the zeroed gradient), so the step is reproducible bit for
bit and the three runs must agree exactly: means, every gradient element, and
the parameters after the following Adam step.  The reference semantics are
those of one TF session step (air/air_model.py:941-999)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
SPIN = 2_000_000  # 20 ms of the 100 MHz wall clock


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _air(scope, precision):
    from mog_air.air_model import AIRModel
    return AIRModel(max_steps=3, max_digits=3, canvas_size=50, scale_prior_variance=0.05,
                    z_pres_prior_log_odds=-0.01, learning_rate=1e-3, gradient_clipping_norm=1.0,
                    cnn=False, train=True, scope=scope, device=DEV, precision=precision,
                    seed=31, noise_seed=32)


def _asr(scope, precision):
    import bench
    return bench.make_asr_model(precision, torch.device(DEV), scope)


def _data(B, n=3):
    import bench
    out = []
    for i in range(n):
        x, k = bench.synthetic(B, 700 + i)
        out.append((torch.as_tensor(x).to(DEV), torch.as_tensor(k).to(DEV)))
    return out


def _run(make, scope, precision, data, spin_main=0, spin_fork=0):
    m = make(scope, precision)
    m.ONE_PASS_WGRADS = True
    m.train_step_async(*data[0])  # every buffer now holds batch 0's values
    torch.cuda.synchronize()
    m.SPIN_MAIN, m.SPIN_FORK = spin_main, spin_fork
    m.compute_gradients(*data[1])
    torch.cuda.synchronize()
    out = {"means": m._ws.means[:3].clone(), "grad": m.params.grad.clone()}
    m.train_step_async(*data[2])  # the join before Adam
    torch.cuda.synchronize()
    out["params"] = m.params.flat.clone()
    out["means2"] = m._ws.means[:3].clone()
    return out


def _same(a, b, what):
    for k in a:
        x, y = a[k], b[k]
        if not torch.equal(x.view(torch.int32), y.view(torch.int32)):
            d = (x - y).abs()
            raise AssertionError(f"{what}: {k} differs in {int((d != 0).sum())} elements "
                                 f"(max {float(d.max()):.3g}; scale {float(x.abs().max()):.3g})")


CASES = [("air", "fp32", 1024), ("air", "bf16", 1024), ("asr", "fp32", 1024),
         ("asr", "bf16", 1024), ("air", "fp32", 64), ("air", "bf16", 64)]


@pytest.mark.parametrize("model,precision,B", CASES)
def test_forked_step_is_order_independent(model, precision, B):
    make = _air if model == "air" else _asr
    data = _data(B)
    tag = f"so_{model}{precision}{B}"
    ref = _run(make, tag + "r", precision, data)
    again = _run(make, tag + "a", precision, data)
    _same(ref, again, "two plain runs (ONE_PASS_WGRADS must be reproducible)")
    _same(ref, _run(make, tag + "m", precision, data, spin_main=SPIN), "main stream held back")
    _same(ref, _run(make, tag + "f", precision, data, spin_fork=SPIN), "forked segments held back")


def test_small_batch_step_has_no_fork():
    """Below SIDE_MIN_BATCH (the reference's batch of 64) the whole step runs
    on one stream: no event is recorded on another stream."""
    from mog_air.air_model import AIRModel
    m = _air("so_nofork", "bf16")
    forks = []
    orig = AIRModel._fork
    m._fork = lambda s: forks.append(s) or orig(m, s)
    (x, k), = _data(64, 1)
    m.train_step_async(x, k)
    torch.cuda.synchronize()
    assert forks == []
    assert np.isfinite(float(m._ws.means[0]))


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_fused_step_kernels_beside_mfma_gemms(precision):
    """The fused STN-read -> VAE -> STN-write kernels (csrc/vae_step.hip) are
    built WITH compiler-packed fp32 (v_pk_*_f32) arithmetic, which DESIGN.md
    §2 found to return wrong halves when bf16 MFMA waves of another kernel
    shared the CU.  Their launches request the CU's whole 160 KiB of LDS
    (vae_step.hip lds_pad), so no GEMM workgroup can share a CU with them.
    Launched on the main stream while the bf16 TN / NT and x3 TN / NT GEMMs
    that triggered the fault run on the side stream (staggered by a spin so
    the launches overlap at different points), every output of 8 such launches
    must equal the launch run alone, bit for bit: r, z, the VAE KL, the canvas
    parts and their row ranges (B = 8192: the train step's T*B = 24,576 rows,
    three rounds of tiles over the CUs)."""
    from mog_air import ops
    from mog_air.ops import BF_ATOMIC, BF_STORE, gemm_bf16
    B = 8192
    m = _air(f"fx_{precision}", precision)
    (x, k), = _data(B, 1)
    m.infer(x, k)
    torch.cuda.synchronize()
    ws = m._ws
    assert m._batched_vae(B) and ws.cparts is not None
    if precision == "fp32":
        assert m.fused_f32 and 3 * B >= m.FUSED_F32_MIN_ROWS
    outs = ("r", "z", "vkl", "cparts", "prows")

    def launch():
        m._vae_forward_all(x, ws, 0.3, save=True)
        return {n: getattr(ws, n).clone() for n in outs}

    ref = launch()
    torch.cuda.synchronize()
    TB, dev = 3 * B, torch.device(DEV)
    g = torch.Generator(device="cpu").manual_seed(5)
    Xf = torch.randn(TB, 784, generator=g).to(dev)
    Yf = torch.randn(TB, 512, generator=g).to(dev)
    Xb, Yb = Xf.bfloat16(), Yf.bfloat16()
    Wb = torch.randn(512, 784, generator=g).to(dev).bfloat16()
    W3 = torch.empty((3, 512, 784), device=dev, dtype=torch.bfloat16)
    ops.split3_bf16(Wb.float(), W3, 512, 784, 784, 784, 512 * 784)
    acc = torch.zeros(784, 512, device=dev)
    outb = torch.zeros(TB, 512, device=dev)
    outx = torch.zeros(TB, 784, device=dev)
    aggressors = [
        lambda: gemm_bf16([Xb], [Yb], [acc], 784, 512, TB, 784, 512, 512, tn=True, epi=BF_ATOMIC,
                          splitk=4),
        lambda: gemm_bf16([Xb], [Wb], [outb], TB, 512, 784, 784, 784, 512, epi=BF_STORE),
        lambda: ops.gemm_x3_tn(Xf, Yf, acc, 784, 512, TB, 784, 512, 512, splitk=8, reduce=False),
        lambda: ops.gemm_x3_nt(Yf, W3, 512 * 784, outx, TB, 784, 512, 512, 512, 784),
    ]
    main, side = torch.cuda.current_stream(), m._side_stream()
    for r in range(8):
        ev = torch.cuda.Event()
        ev.record(main)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            for _ in range(2):
                for fn in aggressors:
                    fn()
        ops.spin(20_000 * r)  # the fused launch lands at a different point each time
        got = launch()
        torch.cuda.synchronize()
        for n in outs:
            a, b = got[n], ref[n]
            iv = torch.int32
            assert torch.equal(a.view(iv), b.view(iv)), (n, r)
