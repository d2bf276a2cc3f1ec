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
