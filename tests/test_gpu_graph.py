"""Captured train step (AIRModel.train_step_graphed: the forward + backward
replayed from one hipGraph, the noise fills, the annealed z_pres prior and TF
Adam outside it) against the eager train step, bit for bit: per-step loss /
accuracy / mse, the object counts and every parameter after several Adam
steps -- at the reference's own batch of 64 (training_air_original.py:22,
304-310), fp32 and bf16, with the z_pres prior annealed as the entry point
anneals it (training_air_original.py:193-201)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

ANNEAL = {"z_pres_prior_log_odds": {"init": 10000.0, "min": 1e-9, "factor": 0.1, "iters": 3000,
                                    "staircase": False, "log": True}}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _model(scope, precision):
    from mog_air.air_model import AIRModel
    return AIRModel(max_steps=3, max_digits=3, canvas_size=50, scale_prior_variance=0.05,
                    z_pres_prior_log_odds=-0.01, learning_rate=1e-3, gradient_clipping_norm=1.0,
                    cnn=False, train=True, scope=scope, device=DEV, precision=precision,
                    annealing_schedules=ANNEAL, seed=21, noise_seed=22)


def _batches(n, B=64):
    import bench
    out = []
    for i in range(n):
        x, k = bench.synthetic(B, 300 + i)
        out.append((torch.as_tensor(x).to(DEV), torch.as_tensor(k).to(DEV)))
    return out


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_graph_replay_matches_eager_bitwise(precision):
    data = _batches(4)
    me, mg = _model("ge" + precision, precision), _model("gg" + precision, precision)
    assert torch.equal(me.params.flat, mg.params.flat)
    for i, (x, k) in enumerate(data):
        me.train_step_async(x, k)
        mg.train_step_graphed(x, k)
        torch.cuda.synchronize()
        assert mg._graph is not None  # captured after the first (eager) step
        a, b = me._ws.means[:3].cpu().numpy(), mg._ws.means[:3].cpu().numpy()  # loss, acc, mse
        np.testing.assert_array_equal(a, b, err_msg=f"step {i} means")
        np.testing.assert_array_equal(me.rec_num_digits.cpu().numpy(),
                                      mg.rec_num_digits.cpu().numpy())
        assert me.global_step == mg.global_step == i + 1
    assert torch.equal(me.params.flat.view(torch.int32), mg.params.flat.view(torch.int32))
    assert torch.equal(me.params.m.view(torch.int32), mg.params.m.view(torch.int32))
    # the device prior was refreshed for the last replay (global step 3)
    from mog_air.air_model import annealed_value
    want = np.float32(annealed_value(ANNEAL["z_pres_prior_log_odds"], 3))
    assert np.float32(mg._prior_dev.item()) == want


def test_graph_replays_new_inputs_and_recaptures_on_shape_change():
    """The replay reads the static input buffers (new images every step), and
    a new batch shape captures a new graph; outputs stay equal to eager."""
    me, mg = _model("gs_e", "fp32"), _model("gs_g", "fp32")
    for B, n in ((64, 3), (128, 2)):
        for x, k in _batches(n, B):
            me.train_step_async(x, k)
            mg.train_step_graphed(x, k)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(me._ws.means[:3].cpu().numpy(),
                                          mg._ws.means[:3].cpu().numpy())
        assert mg._graph_key[0] == (B, 2500)
    assert torch.equal(me.params.flat.view(torch.int32), mg.params.flat.view(torch.int32))


def test_graph_outputs_accessible_after_replay():
    """loss / reconstruction accessors after a replay (materialised on demand
    from the graph's static inputs)."""
    me, mg = _model("go_e", "fp32"), _model("go_g", "fp32")
    for x, k in _batches(2):
        me.train_step_async(x, k)
        mg.train_step_graphed(x, k)
    torch.cuda.synchronize()
    assert me.loss == mg.loss
    np.testing.assert_array_equal(me.reconstruction.cpu().numpy(), mg.reconstruction.cpu().numpy())


def test_asr_graph_replay_matches_eager_bitwise():
    """The AIR-ASR train step (train_air_pr.py -dn 13 -gm 100 -gne 10 at the
    reference's batch of 64) captured and replayed: same bits as eager."""
    import bench
    me = bench.make_asr_model("fp32", torch.device(DEV), "gasr_e")
    mg = bench.make_asr_model("fp32", torch.device(DEV), "gasr_g")
    for x, k in _batches(3):
        me.train_step_async(x, k)
        mg.train_step_graphed(x, k)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(me._ws.means[:3].cpu().numpy(),
                                      mg._ws.means[:3].cpu().numpy())
    assert mg._graph is not None
    assert torch.equal(me.params.flat.view(torch.int32), mg.params.flat.view(torch.int32))


@pytest.mark.parametrize("rep", [0, 1, 2])
def test_graph_replay_after_other_batch_uses_captured_workspace(rep):
    """graphed(64) -> infer(100) -> graphed(64): the replay runs on the
    workspace it was captured on (the infer at another batch replaced
    self._ws), and still equals eager."""
    data = _batches(3)
    x100, k100 = _batches(1, 100)[0]
    me, mg = _model("gw_e%d" % rep, "fp32"), _model("gw_g%d" % rep, "fp32")
    for i, (x, k) in enumerate(data):
        me.train_step_async(x, k)
        mg.train_step_graphed(x, k)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(me._ws.means[:3].cpu().numpy(),
                                      mg._ws.means[:3].cpu().numpy(), err_msg=f"step {i}")
        np.testing.assert_array_equal(me.rec_num_digits.cpu().numpy(),
                                      mg.rec_num_digits.cpu().numpy())
        _assert_params_equal(me, mg, f"after step {i}")
        if i == 0:
            me.infer(x100, k100)
            mg.infer(x100, k100)
            torch.cuda.synchronize()
            assert mg._ws.B == 100 and mg._graph_ws.B == 64
            assert me.loss == mg.loss
    assert mg._ws is mg._graph_ws


def _assert_params_equal(ma, mb, what):
    fa, fb = ma.params.flat, mb.params.flat
    if torch.equal(fa.view(torch.int32), fb.view(torch.int32)):
        return
    bad = []
    for name, shape in ma.params.specs:
        o = ma.params.offsets[name]
        n = int(np.prod(shape))
        d = (fa[o:o + n] - fb[o:o + n]).abs().max().item()
        if d > 0 or not torch.equal(fa[o:o + n].view(torch.int32), fb[o:o + n].view(torch.int32)):
            bad.append((name, d))
    raise AssertionError(f"{what}: parameters differ: {bad[:8]}")


def test_eager_step_after_graph_reads_the_current_prior():
    """After graphed steps, an eager step uses the host's annealed z_pres
    prior of ITS global step (not the device copy the last replay read)."""
    data = _batches(4)
    me, mg = _model("gp_e", "fp32"), _model("gp_g", "fp32")
    for i, (x, k) in enumerate(data):
        me.train_step_async(x, k)
        if i < 2:
            mg.train_step_graphed(x, k)
        else:
            mg.train_step_async(x, k)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(me._ws.means[:3].cpu().numpy(),
                                      mg._ws.means[:3].cpu().numpy(), err_msg=f"step {i}")
    assert torch.equal(me.params.flat.view(torch.int32), mg.params.flat.view(torch.int32))


def _copy_state(dst, src):
    for n in ("flat", "m", "v"):
        getattr(dst.params, n).copy_(getattr(src.params, n))
    for n in ("beta1_power", "beta2_power", "adam_t", "global_step"):
        setattr(dst.params, n, getattr(src.params, n))
    dst.params.version += 1
    dst._noise_ctr = src._noise_ctr


def _grad_close(ga, gb, rel=1e-3, rel_small=1e-2):
    """Per tensor: max |a - b| <= rel * max |a| (split-K atomics reorder the
    weight-gradient sums from B = 1024 on, and the train loss's BCE cotangent
    -- ~1e10 x at canvas pixels equal to 0, DESIGN.md §2 -- makes some of
    those sums cancel by orders of magnitude: the heads' weight gradients move
    by up to ~3e-4 of their largest entry between two orders); tensors of at
    most 64 elements (biases of 1-2 wide output layers: one sum of thousands
    of cancelling terms each) to rel_small.  A race (a stale or overwritten
    operand) moves a gradient by O(1) of its scale."""
    bad = []
    for name in ga:
        a, b = ga[name], gb[name]
        scale = float(np.abs(a).max())
        err = float(np.abs(a - b).max())
        tol = rel_small if a.size <= 64 else rel
        if err > tol * max(scale, 1e-30):
            bad.append((name, err, scale))
    assert not bad, bad[:5]


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_side_streams_match_serial_at_b1024(precision):
    """From B = 1024 (SIDE_MIN_BATCH) the step forks noise fills, loop-state
    resets, the X split, the heads' and the recurrent-rows weight gradients
    onto a side stream: forward bitwise and gradients (split-K tolerance)
    equal to the same step with every fork off."""
    (x, k), = _batches(1, 1024)
    ms, mp = _model("sd_s" + precision, precision), _model("sd_p" + precision, precision)
    ms.HEADS_WGRAD_SIDE = ms.REC_WGRAD_SIDE = ms.NOISE_ON_SIDE = False
    assert mp.HEADS_WGRAD_SIDE and mp.REC_WGRAD_SIDE and mp.NOISE_ON_SIDE
    gs = ms.compute_gradients(x, k)
    gp = mp.compute_gradients(x, k)
    np.testing.assert_array_equal(ms._ws.means[:3].cpu().numpy(), mp._ws.means[:3].cpu().numpy())
    np.testing.assert_array_equal(ms.rec_num_digits.cpu().numpy(), mp.rec_num_digits.cpu().numpy())
    _grad_close(gs, gp)
    # and a full train step (clip + Adam) on each: parameters within Adam's
    # sensitivity to the reordered sums (lr 1e-3)
    ms.train_step_async(x, k)
    mp.train_step_async(x, k)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ms._ws.means[:3].cpu().numpy(), mp._ws.means[:3].cpu().numpy())
    # (Adam's first step moves every parameter by ~lr * sign(g): reordered sums
    # can flip the sign of near-zero gradient elements, so a few parameters
    # differ by up to 2 lr; the rest by rounding)
    d = (ms.params.flat - mp.params.flat).abs()
    assert float(d.max()) <= 2.5e-3 and float(d.mean()) < 2e-5, (float(d.max()), float(d.mean()))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_asr_side_streams_match_serial_at_b1024(precision):
    """AIR-ASR from B = 1024: the per-loop-step VAE and recurrent-rows weight
    gradients on the side stream and the heads' on the third stream give the
    gradients of the after-loop serial form (summation order aside: per-step
    accumulation against one pass over every step's rows), and the forward
    bit for bit."""
    import bench
    (x, k), = _batches(1, 1024)
    ms = bench.make_asr_model(precision, torch.device(DEV), "asd_s" + precision)
    mp = bench.make_asr_model(precision, torch.device(DEV), "asd_p" + precision)
    ms.VAE_WGRAD_PER_STEP = ms.U_WGRAD_PER_STEP = ms.HEADS_S3 = False
    assert mp.VAE_WGRAD_PER_STEP and mp.U_WGRAD_PER_STEP and mp.HEADS_S3
    for m in (ms, mp):
        m.ONE_PASS_WGRADS = True
    gs = ms.compute_gradients(x, k)
    gp = mp.compute_gradients(x, k)
    np.testing.assert_array_equal(ms._ws.means[:3].cpu().numpy(), mp._ws.means[:3].cpu().numpy())
    _grad_close(gs, gp, rel=1e-4, rel_small=1e-3)


def test_graph_replay_with_side_stream_forks_at_b1024():
    """The side-stream forks captured into the graph (B = 1024): a replay's
    forward equals the eager step from the same state bit for bit, its
    gradient within the split-K tolerance."""
    data = _batches(2, 1024)
    me, mg = _model("gb_e", "fp32"), _model("gb_g", "fp32")
    mg.train_step_graphed(*data[0])  # eager step + capture
    torch.cuda.synchronize()
    _copy_state(me, mg)
    me.train_step_async(*data[1])
    mg.train_step_graphed(*data[1])  # replay
    torch.cuda.synchronize()
    np.testing.assert_array_equal(me._ws.means[:3].cpu().numpy(), mg._ws.means[:3].cpu().numpy())
    np.testing.assert_array_equal(me.rec_num_digits.cpu().numpy(), mg.rec_num_digits.cpu().numpy())
    _grad_close(me.params.grad_dict(), mg.params.grad_dict())


def _poison(ws, value):
    """Overwrite every buffer of a workspace (what a recycled allocation may
    hold): a step must write before it reads."""
    n = 0
    for k, v in list(vars(ws).items()):
        if k in ws.ZERO_PADDED:  # (zero pad columns by design, see _Workspace)
            continue
        if isinstance(v, torch.Tensor) and v.is_cuda:
            if v.dtype.is_floating_point:
                v.fill_(value)
            else:
                v.fill_(-7 if value != 0 else 0)
            n += 1
    return n


@pytest.mark.parametrize("precision,B", [("fp32", 64), ("bf16", 64), ("fp32", 100)])
def test_step_reads_no_stale_workspace_memory(precision, B):
    """Two models in the same state; before the second train step one
    workspace is filled with NaN, the other with zeros: the step must give
    the same parameters bit for bit (no kernel reads a buffer element that
    this step has not written)."""
    data = _batches(2, B)
    ma, mb = _model("pz_a%s%d" % (precision, B), precision), _model("pz_b%s%d" % (precision, B), precision)
    ma.train_step_async(*data[0])
    mb.train_step_async(*data[0])
    torch.cuda.synchronize()
    _assert_params_equal(ma, mb, "after the first step")
    assert _poison(ma._ws, float("nan")) == _poison(mb._ws, 0.0) > 50
    ma.train_step_async(*data[1])
    mb.train_step_async(*data[1])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ma._ws.means[:3].cpu().numpy(), mb._ws.means[:3].cpu().numpy())
    _assert_params_equal(ma, mb, "after the poisoned step")
