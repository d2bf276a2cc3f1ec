"""AIRModel — drop-in host object for the reference's AIR baseline model
(air/air_model.py:13-1146), running the per-object-step loop on MI355X HIP
kernels (libmog_air.so) with a hand-scheduled forward and backward.

Reference surface kept (air_model.py:15-51, training_air_original.py:158-209):
the constructor keyword arguments, variable sharing between a train model and
a test model (``reuse``), annealing schedules (air_model.py:139-147,164-184)
and the result attributes ``loss, accuracy, mse_loss, global_step,
rec_num_digits, rec_scales, rec_shifts, rec_st_back, rec_windows, rec_latents,
reconstruction, reconstruction_loss, z_pres_probs, z_pres_kls, scale_kls,
shift_kls, vae_kls, accuracy_instance``.  TF's ``sess.run([model.training,
...])`` becomes ``model.step(images, targets)``; fetching the test model's
tensors becomes ``model.infer(images, targets)``.

Loop semantics: the data-dependent ``tf.while_loop`` (air_model.py:428-432)
runs max_steps iterations on the device with the predicate folded into a
per-step ``live`` flag; every loss term, count and gradient is identical to
the early exit, and the ``rec_*`` outputs are sliced to the executed steps.
No host synchronisation happens inside a train step.
"""
from __future__ import annotations

import contextlib
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from . import ops
from .ops import EPI_RELU, EPI_SIGMOID_NOISE, EPI_SOFTPLUS, EPI_SOFTPLUS_BWD, EPI_STORE, gemm
from .graph import GraphCapture
from .params import ParamStore, param_specs
from .results import Results
from .wgrads import WeightGradients

_ops = ops._ops  # torch.ops.mog_air (csrc/torch_ops.cpp)

# step-record slots (air_cell.hip enum)
R_SM, R_SLV, R_HM0, R_HM1, R_HLV0, R_HLV1, R_LO, R_S, R_TX, R_TY, R_Y, R_Z = range(12)
R_ACT_OLD, R_ACT, R_LIVE, R_ZC, R_ZTERM, R_NREC = 12, 13, 14, 15, 16, 17

_SCOPES: Dict[str, ParamStore] = {}


def _f32log(v: float) -> float:
    return float(np.log(np.float32(v), dtype=np.float32))


def annealed_value(schedule: dict, global_step: int, eps=1e-9) -> float:
    """tf.train.exponential_decay (+min/max/log) in fp32 (air_model.py:164-184)."""
    f = np.float32
    p = f(global_step) / f(schedule["iters"])
    if schedule.get("staircase", False):
        p = np.floor(p)
    v = f(schedule["init"]) * np.power(f(schedule["factor"]), p, dtype=np.float32)
    if "min" in schedule:
        v = np.maximum(v, f(schedule["min"]))
    if "max" in schedule:
        v = np.minimum(v, f(schedule["max"]))
    if schedule.get("log", False):
        v = np.log(v + f(eps), dtype=np.float32)
    return float(v)


def marginal_objective(num_prior, max_steps) -> np.ndarray:
    """The ``-ap`` per-step prior bias (air_model.py:86-107)."""
    obj = np.zeros([max_steps])
    buf = 1.0 - 1.0 / len(num_prior)
    for ind in range(max_steps):
        if ind not in num_prior and ind < max(num_prior):
            obj[ind] = 1.0
        else:
            if ind == max(num_prior):
                break
            obj[ind] = buf
            if ind in num_prior:
                buf -= 1.0 / len(num_prior)
    for ind in range(max_steps):
        if obj[ind] == 1.0:
            obj[ind] = 100
        elif obj[ind] == 0.0:
            obj[ind] = -100.0
        else:
            obj[ind] = np.log(obj[ind] / (1.0 - obj[ind]))
    return obj.astype(np.float32)


_STREAMS: Dict[torch.device, tuple] = {}


def _shared_streams(device):
    """The side stream and the third stream of AIRModel, created once per
    process and device.  HIP places a stream on one of its GPU_MAX_HW_QUEUES
    (4) hardware queues when the stream is created; with a pair created per
    model, every other model of a process had both on ONE queue, which
    serialised the third stream behind the side stream (fp32 step 3.09 ->
    3.43 ms, bf16 2.09 -> 2.29 ms; scripts/gpu_slot_trace.sh: queues 2 / 3 for
    the first model, 4 / 4 for the second).  The first pair of a process sits
    on two queues of its own, and every model now uses it."""
    key = torch.device(device)
    if key not in _STREAMS:
        _STREAMS[key] = (torch.cuda.Stream(device=key), torch.cuda.Stream(device=key))
    return _STREAMS[key]


class _Workspace:
    """All per-batch device buffers of one train step (HBM-resident, reused).
    Buffers in ZERO_PADDED carry zero pad columns written once at allocation
    (the bf16 latents' 50 -> 56 columns: the K padding of the GEMMs that read
    them); every other element is written by the step before it is read."""

    ZERO_PADDED = ("zb", "dmub", "dlvb", "Xb")

    def __init__(self, m: "AIRModel", B: int):
        dev = m.device
        T, H, C2, W2, Z = m.max_steps, m.rnn_units, m.C2, m.W2, m.vae_latent_dimensions
        R1, R2 = m.vae_recognition_units
        G1, G2 = m.vae_generative_units
        HS = m.scale_hidden_units
        e = lambda *s: torch.empty(s, device=dev, dtype=torch.float32)  # noqa: E731
        self.B = B
        self.Gx = e(B, 4 * H)
        self.G = e(T, B, 4 * H)
        self.c = e(T, B, H)
        self.h = e(T, B, H)
        self.hid = e(5, T, B, HS)
        self.rec = e(T, R_NREC, B)
        self.th_f = e(T, B, 6)
        self.th_b = e(T, B, 6)
        self.scale = e(T, B)
        self.shift = e(T, B, 2)
        self.zprob, self.zkl, self.skl, self.shkl = e(T, B), e(T, B), e(T, B), e(T, B)
        self.zmask, self.zval, self.vkl = e(T, B), e(T, B), e(T, B)
        self.zc = e(T, B)
        self.bf16 = m.precision == "bf16"
        self.mu, self.lv, self.z = e(T, B, Z), e(T, B, Z), e(T, B, Z)
        self.r = e(T, B, W2)
        if self.bf16:
            eb = lambda *s: torch.empty(s, device=dev, dtype=torch.bfloat16)  # noqa: E731
            Zp = (Z + 7) // 8 * 8
            self.gb, self.a1b, self.a2b = eb(T, B, W2), eb(T, B, R1), eb(T, B, R2)
            self.zb = torch.zeros((T, B, Zp), device=dev, dtype=torch.bfloat16)
            self.d1b, self.d2b = eb(T, B, G1), eb(T, B, G2)
        else:
            self.g = e(T, B, W2)
            # (post-activations only: the softplus backward reads sigmoid(x)
            # as 1 - exp(-softplus(x)), mog_gemm_f32 epi 4)
            self.a1, self.a2 = e(T, B, R1), e(T, B, R2)
            self.d1, self.d2 = e(T, B, G1), e(T, B, G2)
        self.canvas = e(B, C2)
        # fused bf16 step: per-step canvas contributions, summed by the loss kernel
        parts = m._parts_layout(B)
        self.cparts = e(T, B, C2) if parts else None
        self.prows = torch.empty((T, B), device=dev, dtype=torch.int32) if parts else None
        self.stop, self.runloss = e(B), e(B)
        self.digits = torch.empty(B, device=dev, dtype=torch.int32)
        self.live = torch.empty(T + 1, device=dev, dtype=torch.int32)
        self.recon = e(B, C2)
        self.bce, self.mse, self.loss_b, self.acc_b = e(B), e(B), e(B), e(B)
        self.means = e(4)
        # noise
        self.eps_scale, self.eps_shift = e(T, B), e(T, B, 2)
        self.eps_z, self.eps_x, self.u = e(T, B, Z), e(T, B, W2), e(T, B)
        self.eps_x_offset = None  # set when the fused kernel generates eps_x itself
        self._bwd = False
        self.materialized = False

    def alloc_backward(self, m: "AIRModel"):
        if self._bwd:
            return
        dev, B = m.device, self.B
        T, H, C2, W2, Z = m.max_steps, m.rnn_units, m.C2, m.W2, m.vae_latent_dimensions
        R1, R2 = m.vae_recognition_units
        G1, G2 = m.vae_generative_units
        HS = m.scale_hidden_units
        e = lambda *s: torch.empty(s, device=dev, dtype=torch.float32)  # noqa: E731
        self.dcanvas = e(B, C2)
        self.dr = e(B, W2)
        self.dz = e(B, Z)
        self.tmp_a2 = e(B, R2)
        self.dg = e(B, W2)
        if self.bf16:
            eb = lambda *s: torch.empty(s, device=dev, dtype=torch.bfloat16)  # noqa: E731
            Zp = (Z + 7) // 8 * 8
            self.dmb, self.dd2b, self.dd1b = eb(T, B, W2), eb(T, B, G2), eb(T, B, G1)
            self.dmub = torch.zeros((T, B, Zp), device=dev, dtype=torch.bfloat16)
            self.dlvb = torch.zeros((T, B, Zp), device=dev, dtype=torch.bfloat16)
            self.da2b, self.da1b = eb(T, B, R2), eb(T, B, R1)
        else:
            self.dm = e(T, B, W2)
            self.dd2, self.dd1 = e(T, B, G2), e(T, B, G1)
            self.dmu, self.dlv = e(T, B, Z), e(T, B, Z)
            self.da2, self.da1 = e(T, B, R2), e(T, B, R1)
        self.dth_f, self.dth_b, self.dot = e(B, 6), e(B, 6), e(B)
        # all loop steps at once (AIR: only the LSTM chain is sequential)
        self.dr_all, self.dg_all = e(T, B, W2), e(T, B, W2)
        self.dz_all, self.tmp_a2_all = e(T, B, Z), e(T, B, R2)
        self.dth_f_all, self.dth_b_all, self.dot_all = e(T, B, 6), e(T, B, 6), e(T, B)
        self.dout = e(5, T, B, 2)
        # heads side by side per row ([T, B, 5, HS]): dh is one GEMM over K = 5 HS;
        # 4 HS floats of slack after it, so that head z's column view spans
        # T*B whole rows from its origin (the grouped weight-gradient kernels
        # read K x ld elements of an operand, mog_wgrad_tn_x3)
        self.dhid = e(T * B * 5 * HS + 4 * HS)[:T * B * 5 * HS].view(T, B, 5, HS)
        self.dh = e(T, B, H)
        self.dc = e(2, B, H)
        self.dG = e(T, B, 4 * H)
        self.dGsum = e(B, 4 * H)
        self._bwd = True


class AIRModel(WeightGradients, GraphCapture, Results):
    """See module docstring.  Extra keyword-only arguments (not in the
    reference): ``device``, ``seed`` (weight init), ``noise_seed`` (device
    Philox noise), ``grad_world`` (data-parallel world size folded into the
    loss-mean gradient scale)."""

    def __init__(self, input_images=None, target_num_digits=None, max_steps=3, max_digits=2,
                 rnn_units=256, canvas_size=50, windows_size=28, vae_latent_dimensions=50,
                 vae_recognition_units=(512, 256), vae_generative_units=(256, 512),
                 scale_prior_mean=-1.0, scale_prior_variance=0.1, shift_prior_mean=0.0,
                 shift_prior_variance=1.0, vae_prior_mean=0.0, vae_prior_variance=1.0,
                 vae_likelihood_std=0.3, scale_hidden_units=64, shift_hidden_units=64,
                 z_pres_hidden_units=64, z_pres_prior_log_odds=-2.0, z_pres_temperature=1.0,
                 stopping_threshold=0.99, learning_rate=1e-3, gradient_clipping_norm=100.0,
                 cnn=True, cnn_filters=8, num_summary_images=60, train=False, reuse=False,
                 scope="air", annealing_schedules=None, generation_batch_size=64,
                 num_prior=None, *, device=None, seed: int = 1235, noise_seed: int = 1235,
                 grad_world: int = 1, precision: str = "fp32", fused_step: bool = True,
                 batch_vae: bool = True):
        if precision not in ("fp32", "bf16"):
            raise ValueError("precision must be 'fp32' (bit-exact parity) or 'bf16'")
        self.precision = precision
        # bf16: one fused STN-read -> VAE -> STN-write launch per loop step
        # (vae_step.hip) when the VAE has the reference's default shape
        self.fused_step = bool(fused_step) and precision == "bf16" and (
            windows_size == 28 and tuple(vae_recognition_units) == (512, 256)
            and vae_latent_dimensions == 50 and tuple(vae_generative_units) == (256, 512))
        # fp32: the same fused step at the reference precision over the T*B
        # rows of the batched VAE (stn_vae_step_f32_kernel; fused_step=False
        # runs the unfused sequence it is bit-identical to)
        self.fused_f32 = bool(fused_step) and precision == "fp32" and (
            windows_size == 28 and tuple(vae_recognition_units) == (512, 256)
            and vae_latent_dimensions == 50 and tuple(vae_generative_units) == (256, 512))
        # the glimpse VAE of all T steps after the loop, over T*B rows (AIR).
        # (Measured and not kept: step 0's VAE on a second stream under the
        # rest of the recurrent loop -- no gain at B = 8192, slower at 64.)
        self.batch_vae = bool(batch_vae)
        if cnn:
            raise NotImplementedError(
                "cnn=True (air_model.py:763-810) is outside the hot-path scope; the entry "
                "points use cnn=False")
        if not (scale_hidden_units == shift_hidden_units == z_pres_hidden_units):
            raise NotImplementedError("heads must share one hidden width")
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        if self.device.type != "cuda":
            raise RuntimeError("AIRModel runs on a HIP device only (no CPU fallback)")
        _lib.load_torch_ops()
        self.input_images = input_images
        self.target_num_digits = target_num_digits
        self.max_steps, self.max_digits = int(max_steps), max_digits
        self.rnn_units = int(rnn_units)
        self.canvas_size, self.windows_size = int(canvas_size), int(windows_size)
        self.C2, self.W2 = self.canvas_size ** 2, self.windows_size ** 2
        self.vae_latent_dimensions = int(vae_latent_dimensions)
        self.vae_recognition_units = tuple(vae_recognition_units)
        self.vae_generative_units = tuple(vae_generative_units)
        self.scale_prior_mean, self.scale_prior_variance = scale_prior_mean, scale_prior_variance
        self.shift_prior_mean, self.shift_prior_variance = shift_prior_mean, shift_prior_variance
        self.vae_prior_mean, self.vae_prior_variance = vae_prior_mean, vae_prior_variance
        self.vae_likelihood_std = vae_likelihood_std
        self.scale_hidden_units = scale_hidden_units
        self.shift_hidden_units = shift_hidden_units
        self.z_pres_hidden_units = z_pres_hidden_units
        self.z_pres_prior_log_odds = z_pres_prior_log_odds
        self.z_pres_temperature = z_pres_temperature
        self.stopping_threshold = stopping_threshold
        self.learning_rate = learning_rate
        self.gradient_clipping_norm = gradient_clipping_norm
        self.num_summary_images = num_summary_images
        self.train = bool(train)
        self.scope = scope
        self.annealing_schedules = dict(annealing_schedules or {})
        self.generation_batch_size = generation_batch_size
        self.num_prior = num_prior
        self.noise_seed = int(noise_seed)
        self.grad_world = int(grad_world)
        self._noise_ctr = 0
        self.scale_prior_log_variance = _f32log(scale_prior_variance)
        self.shift_prior_log_variance = _f32log(shift_prior_variance)
        self.vae_prior_log_variance = _f32log(vae_prior_variance)
        self.marginal = (marginal_objective(num_prior, self.max_steps)
                         if num_prior is not None else None)
        specs = param_specs(self.C2, self.rnn_units, self.W2, self.vae_recognition_units,
                            self.vae_generative_units, self.vae_latent_dimensions,
                            scale_hidden_units, z_pres_hidden_units)
        if reuse:
            if scope not in _SCOPES:
                raise ValueError(f"reuse=True but scope {scope!r} has no variables yet")
            self.params = _SCOPES[scope]
            if self.params.specs != specs:
                raise ValueError("reused scope has different variable shapes")
        else:
            self.params = ParamStore(specs, self.device, seed=seed)
            _SCOPES[scope] = self.params
        self._ws: Optional[_Workspace] = None
        self._last_T = None
        self._outputs_ready = False

    # ----------------------------------------------------------- helpers ---
    # Optional per-kernel HIP-event timing (bench.py roofline): when
    # ``kernel_events`` is a dict, every tagged launch records (start, end,
    # work, side) on the stream it is launched on; work = (bound, amount,
    # peak[, "x3"]) -- algorithmic flops ("mfma", peak "fp32" / "bf16"; "x3":
    # fp32 flops issued as six bf16 products) or bytes ("hbm") of that one
    # launch, or None (bench.kernel_work prices the tag); side: launched on
    # one of the shared side streams.
    kernel_events = None

    class _NoTimer:
        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

    class _Timer:
        def __init__(self, sink, name, work):
            self.sink, self.name, self.work = sink, name, work

        def __enter__(self):
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            s = torch.cuda.current_stream()
            self.e0.record(s)
            # a launch on a side stream: its events also count the time its
            # first workgroups wait for CUs the main stream's kernels hold
            self.side = any(s == o for o in _STREAMS.get(s.device, ()))
            return self

        def __exit__(self, *a):
            self.e1.record(torch.cuda.current_stream())
            self.sink.setdefault(self.name, []).append((self.e0, self.e1, self.work, self.side))
            return False

    def _timed(self, name, work=None):
        if self.kernel_events is None:
            return AIRModel._NoTimer()
        return AIRModel._Timer(self.kernel_events, name, work)

    @property
    def global_step(self) -> int:
        return self.params.global_step

    # Data parallelism (parallel.attach): the loss is the mean over the GLOBAL
    # batch, so each rank scales its loss gradient by 1/B_global and the SUM
    # all-reduce of the shards' gradients is the full-batch gradient even for
    # unequal shards.  B_global defaults to B_local * grad_world; the trainer
    # passes the true global batch of each step (global_batch=...).
    _global_batch: Optional[int] = None

    def _gscale(self, B: int) -> float:
        gb = self._global_batch if self._global_batch is not None else B * self.grad_world
        return 1.0 / float(gb)

    # set by parallel.attach: bucketed async SUM all-reduce of params.grad
    # (launch(view) as buckets become final during the backward, wait() before
    # the optimizer) and, for the data-dependent loop exit, a MAX all-reduce of
    # each step's live flag (only where the exit changes the loss: ``-ap``)
    grad_reducer = None
    live_hook = None

    def _reduce_bucket(self, lo: int, hi: int) -> None:
        if self.grad_reducer is not None:
            self.grad_reducer.launch(self.params.grad[lo:hi])

    def _bucket_split(self) -> int:
        """Flat offset where the glimpse-side variables (heads, VAE) start:
        [0, split) is the LSTM kernel + bias, [split, total) everything else
        (params.param_specs order)."""
        return self.params.offsets[self._SCOPE_PREFIX + "scale/mean/hidden/weights"]

    def hyper(self, name: str) -> float:
        """Current value of a possibly-annealed hyper-parameter, evaluated at
        the pre-increment global step (as in the reference forward pass)."""
        if name in self.annealing_schedules:
            return annealed_value(self.annealing_schedules[name], self.params.global_step)
        return float(getattr(self, name))

    def _workspace(self, B: int) -> _Workspace:
        if self._ws is None or self._ws.B != B:
            self._ws = _Workspace(self, B)
        return self._ws

    _SCOPE_PREFIX = "air/rnn/"  # variable scope of the loop body (air_model.py:127,812)

    def _P(self, name):
        return self.params.view(self._SCOPE_PREFIX + name)

    def _G(self, name):
        return self.params.g(self._SCOPE_PREFIX + name)

    _HEADS = ("scale/mean", "scale/log_variance", "shift/mean", "shift/log_variance",
              "z_pres/log_odds")
    _VAE = ("recognition_1", "recognition_2", "rec_mean", "rec_log_variance", "generative_1",
            "generative_2", "gen_mean")

    def _fill_noise(self, ws: _Workspace, noise: Optional[Dict[str, torch.Tensor]]):
        ws.eps_x_offset = None  # injected noise: every consumer reads the buffers
        ws.noise_side = False
        if noise is not None:
            for k in ("eps_scale", "eps_shift", "eps_z", "eps_x", "u"):
                src = noise[k]
                dst = getattr(ws, k)
                if tuple(src.shape) != tuple(dst.shape):
                    raise ValueError(f"noise[{k}] has shape {tuple(src.shape)}, "
                                     f"expected {tuple(dst.shape)}")
                dst.copy_(src)
            return
        side = None
        if self.NOISE_ON_SIDE and ws.B >= self.SIDE_MIN_BATCH:
            # on the side stream, under the x-projection (which needs none of
            # it); _forward joins it after that GEMM
            side = self._fork(self._side_stream())
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            # the step's noise buffers in one launch, each with its own Philox
            # counter range (bit-identical to one mog_rng_fill per buffer)
            outs, offs, nrm = [], [], []
            for k, normal in (("eps_scale", True), ("eps_shift", True), ("eps_z", True),
                              ("eps_x", True), ("u", False)):
                buf = getattr(ws, k)
                if k == "eps_x" and self._eps_x_in_kernel(ws.B) and not self._graph_noise:
                    # generated inside the fused step kernel / the fp32 output
                    # layer's epilogue from the same Philox counters
                    # (bit-identical to filling the buffer)
                    ws.eps_x_offset = self._noise_ctr
                else:
                    outs.append(buf)
                    offs.append(ops._i64(self._noise_ctr))
                    nrm.append(1 if normal else 0)
                self._noise_ctr += (buf.numel() + 3) // 4
            _ops.rng_fill_batch_(outs, ops._i64(self.noise_seed), offs, nrm)
        ws.noise_side = side is not None

    def _reset_loop_state(self, ws):
        """tf.while_loop's initial state (air_model.py:815-826): stopping sum,
        running loss, counts 0, live flags 1 for step 0 and 0 after (and the
        running canvas when the step does not use parts) -- one launch (a
        fill kernel: capturable, unlike a host copy)."""
        bufs = [ws.stop, ws.runloss, ws.digits, ws.live[:1], ws.live[1:]]
        vals = [0, 0, 0, 1, 0]
        if ws.cparts is None:
            bufs.append(ws.canvas)
            vals.append(0)
        _ops.fill32_batch_(bufs, vals)

    # AIR's _forward joins side-stream noise after the x-projection (the ASR
    # subclass fills on the current stream)
    NOISE_ON_SIDE = True
    # batched VAE: every step's heads and scalars in one launch each after
    # the LSTM chain (False: per step, as the unbatched loop;
    # tests/test_gpu_steps_fwd.py compares the two bitwise)
    STEPS_ONE_LAUNCH = True

    # ----------------------------------------------------------- forward ---
    def _forward(self, X: torch.Tensor, targets: Optional[torch.Tensor], ws: _Workspace,
                 need_grad: bool, outputs: bool = True) -> None:
        B, T, H = ws.B, self.max_steps, self.rnn_units
        C, W, C2, W2 = self.canvas_size, self.windows_size, self.C2, self.W2
        Z = self.vae_latent_dimensions
        R1, R2 = self.vae_recognition_units
        G1, G2 = self.vae_generative_units
        HS = self.scale_hidden_units
        K = self._P("rnn/basic_lstm_cell/kernel")
        bK = self._P("rnn/basic_lstm_cell/bias")
        Wx, Wh = K[:C2], K[C2:]
        side = self._side_stream() if getattr(ws, "noise_side", False) else None
        ws.noise_side = False
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            # (after the noise on the side stream, when it went there)
            self._reset_loop_state(ws)
            if need_grad and self._x3p_xgrad(B):
                # the x-part gradient's A operand, split once per step
                C2p = self._pad8(C2)
                if getattr(ws, "X3", None) is None:
                    ws.X3 = torch.empty((3, B, C2p), device=self.device, dtype=torch.bfloat16)
                ops.split3_bf16(X, ws.X3, B, C2, C2, C2p, B * C2p)
            if need_grad and self.precision == "bf16":
                self._x_bf16(X, ws)  # (likewise: the bf16 x-part gradient's A operand)
            if (need_grad and self.precision == "fp32" and self.VAE_DX_X3
                    and B * self.max_steps >= self.X3_DX_MIN_ROWS):
                # the x3 input gradients' weight pieces, split here instead of
                # on the backward's path (fp32 step 3.05 -> 3.02 ms)
                self._w3()
            if side is not None:
                pre_done = torch.cuda.Event()
                pre_done.record(side)
        prior_lo = self.hyper("z_pres_prior_log_odds")
        temperature = self.hyper("z_pres_temperature")
        thr = self.hyper("stopping_threshold")
        lik_std = self.hyper("vae_likelihood_std")
        batched = self._batched_vae(B)
        # hoisted x-projection of the LSTM input (input is loop-invariant in AIR)
        with self._timed("lstm_x_projection"):
            gemm([X], [Wx], [ws.Gx], B, 4 * H, C2, C2, 4 * H, 4 * H)
        if side is not None:
            torch.cuda.current_stream().wait_event(pre_done)
        w1 = [self._P(h + "/hidden/weights") for h in self._HEADS]
        b1 = [self._P(h + "/hidden/biases") for h in self._HEADS]
        w2 = [self._P(h + "/output/weights") for h in self._HEADS]
        b2 = [self._P(h + "/output/biases") for h in self._HEADS]
        # batched VAE: the LSTM chain first, then every step's heads over T*B
        # rows and every step's scalars in one launch each (the heads read h_t
        # only; mog_air_step_forward_steps)
        steps_all = batched and T <= 8 and self.STEPS_ONE_LAUNCH
        for t in range(T):
            if t == 0:
                _ops.lstm_cell_forward_(ws.Gx, bK, None, ws.c[0], ws.h[0], B, H)
            else:
                gemm([ws.h[t - 1]], [Wh], [ws.G[t]], B, 4 * H, H, H, 4 * H, 4 * H, bias=[bK],
                     Cin=[ws.Gx])
                _ops.lstm_cell_forward_(ws.G[t], None, ws.c[t - 1], ws.c[t], ws.h[t], B, H)
            if steps_all:
                continue
            hid_t = [ws.hid[z, t] for z in range(5)]
            gemm([ws.h[t]] * 5, w1, hid_t, B, HS, H, H, HS, HS, epi=EPI_RELU, bias=b1)
            bias_t = float(self.marginal[t]) if self.marginal is not None else 0.0
            rec = ws.rec[t]
            _ops.air_step_forward_(
                B, HS, HS, t, self.train, self.marginal is not None, thr, temperature, prior_lo,
                bias_t, float(self.scale_prior_mean), float(self.scale_prior_variance),
                self.scale_prior_log_variance, float(self.shift_prior_mean),
                float(self.shift_prior_variance), self.shift_prior_log_variance, hid_t, w2, b2,
                ws.eps_scale[t], ws.eps_shift[t], ws.u[t], ws.stop, ws.runloss, ws.digits,
                ws.live, rec, ws.th_f[t], ws.th_b[t], ws.scale[t], ws.shift[t], ws.zprob[t],
                ws.zkl[t], ws.skl[t], ws.shkl[t], ws.zmask[t], ws.zval[t], ws.zc[t],
                self._prior_arg())
            if self.live_hook is not None:
                self.live_hook(ws.live, t)
            if batched:
                continue
            if self.fused_step:
                with self._timed("stn_vae_step"):
                    self._step_fused(X, ws, t, float(lik_std), save=need_grad)
                continue
            # STN read -> glimpse VAE (air_model.py:523-550, vae.py:5-48)
            if self.precision == "bf16":
                self._vae_forward_bf16(X, ws, t, float(lik_std))
            else:
                self._vae_forward_fp32(X, ws, t, float(lik_std))
            # STN write + masked canvas accumulation (air_model.py:580-588, 665-675)
            ops.stn_forward(ws.r[t], ws.th_b[t], (C, C), out=ws.canvas, z=ws.zval[t],
                            mask=ws.zmask[t], accumulate=True)
        if steps_all:
            TB = T * B
            gemm([ws.h.view(TB, H)] * 5, w1, [ws.hid[z].view(TB, HS) for z in range(5)], TB, HS,
                 H, H, HS, HS, epi=EPI_RELU, bias=b1)
            biases = [float(self.marginal[t]) if self.marginal is not None else 0.0
                      for t in range(T)]
            _ops.air_step_forward_steps_(
                T, B, HS, HS, self.train, self.marginal is not None, thr, temperature, prior_lo,
                biases, float(self.scale_prior_mean), float(self.scale_prior_variance),
                self.scale_prior_log_variance, float(self.shift_prior_mean),
                float(self.shift_prior_variance), self.shift_prior_log_variance,
                [ws.hid[z] for z in range(5)], w2, b2, ws.eps_scale, ws.eps_shift, ws.u, ws.stop,
                ws.digits, ws.live, ws.rec, ws.th_f, ws.th_b, ws.scale, ws.shift, ws.zprob,
                ws.zkl, ws.skl, ws.shkl, ws.zmask, ws.zval, ws.zc, self._prior_arg())
            if self.live_hook is not None:
                for t in range(T):
                    self.live_hook(ws.live, t)
        if batched:
            self._vae_forward_all(X, ws, float(lik_std), save=need_grad)
            # the running loss in the loop's order (z_pres term, scale, shift
            # and VAE KLs per step), replayed from the step records; with the
            # one-launch steps, the loop predicate live[t] applied here first
            _ops.air_runloss_(T, B, ws.rec, R_NREC * B, ws.skl, ws.shkl, ws.vkl, ws.runloss,
                              ws.live if steps_all else None)
        self._forward_loss(X, targets, ws, need_grad, outputs)

    def _parts_layout(self, B: int) -> bool:
        """Per-step canvas parts [T, B, C*C] (+ stored row ranges) summed in
        step order by the loss kernel, instead of one running canvas: the
        fused step kernel and the all-steps STN write."""
        return self.fused_step or self._batched_vae(B)

    def _eps_x_in_kernel(self, B: int) -> bool:
        """The likelihood noise eps_x is generated where it is consumed: in the
        fused step kernel (bf16) or in the fp32 output layer's epilogue (the
        batched VAE), never materialised."""
        return self.fused_step or (self.precision == "fp32" and self._batched_vae(B))

    def _batched_vae(self, B: int) -> bool:
        """AIR's VAE output never feeds the recurrence (the LSTM input is the
        image alone, air_model.py:454-456), so the glimpse VAE of every step
        can run after the loop over all T*B rows at once: taller GEMMs and one
        fused launch instead of T.  Rows of one image stay independent, so
        every output is bit-identical to the per-step schedule; the canvas is
        still accumulated in step order.  Tiles of the fused kernel must not
        straddle two steps (B % 64)."""
        return self.batch_vae and B % 64 == 0

    FUSED_F32_MIN_ROWS = 8192

    def _vae_forward_all(self, X, ws, lik_std, t0=0, t1=None, save=True):
        """The glimpse VAE (STN read -> VAE -> STN write into the canvas
        parts) of loop steps [t0, t1) as one set of launches over their rows.
        save=False: no backward follows (the fused kernel skips the saved
        activations)."""
        B, C, W = ws.B, self.canvas_size, self.windows_size
        t1 = self.max_steps if t1 is None else t1
        T, TB = t1 - t0, (t1 - t0) * B
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        r_ = lambda a: a[t0:t1]  # noqa: E731
        if self.fused_step:
            self._pack_bf16()
            if self.windows_size != 28 or (R1, R2, Z, G1, G2) != (512, 256, 50, 256, 512):
                raise ValueError("the fused step kernel is compiled for the reference VAE shape")
            wt = [self._wf[n] for n in self._VAE]
            gen = getattr(ws, "eps_x_offset", None) is not None
            off = ws.eps_x_offset + t0 * B * (W2 // 4) if gen else 0
            bias = [self._P("vae/" + n + "/biases") for n in self._VAE]
            # forward only (no backward follows): the backward's saved
            # activations are not written (vae_step.hip moves its own bytes)
            sv = r_ if save else (lambda a: None)  # noqa: E731
            with self._timed("stn_vae_step_all"):
                self._stn_vae_step_bf16(TB, C, X, r_, sv, gen, off, wt, bias, lik_std, ws, B)
            return
        # the fused fp32 kernel runs one 32-row tile per workgroup with a long
        # serial chain per tile (~200 us): below one tile per CU (T*B < 8192
        # rows, e.g. the reference's batch of 64) the unfused launches, which
        # spread every layer over the chip, finish first -- same bits either way
        if self.precision == "fp32" and self.fused_f32 and TB >= self.FUSED_F32_MIN_ROWS:
            self._pack_f32()
            gen = getattr(ws, "eps_x_offset", None) is not None
            off = ws.eps_x_offset + t0 * B * (W2 // 4) if gen else 0
            bias = [self._P("vae/" + n + "/biases") for n in self._VAE]
            # (the pre-activations are not stored: None in their slots)
            saved = [r_(getattr(ws, n)) if save and n is not None else None
                     for n in ("g", None, "a1", None, "a2", "mu", "lv", None, "d1", None, "d2")]
            with self._timed("stn_vae_step_f32_all"):
                _ops.stn_vae_step_f32_(TB, C, X, r_(ws.th_f), r_(ws.th_b), r_(ws.zmask),
                                       r_(ws.zval), r_(ws.eps_z), r_(ws.eps_x),
                                       ops._i64(self.noise_seed), ops._i64(off), gen, self._wf32,
                                       bias, lik_std, float(self.vae_prior_mean),
                                       float(self.vae_prior_variance), self.vae_prior_log_variance,
                                       r_(ws.cparts), r_(ws.prows), None, r_(ws.vkl), saved,
                                       r_(ws.z), r_(ws.r), B)
            return
        v = lambda a: a[t0:t1].reshape(TB, -1)  # noqa: E731
        vb = {n: self._P("vae/" + n + "/biases") for n in self._VAE}
        if self.precision == "bf16":
            from .ops import BF_SIGMOID_NOISE, BF_SOFTPLUS, BF_STORE, gemm_bf16
            Zp = self._pad8(Z)
            self._pack_bf16()
            wt = self._wt
            # every step's glimpse read of the shared input canvas in one launch
            ops.stn_forward(X, v(ws.th_f), (W, W), out=v(ws.gb), n=TB)
            gemm_bf16([v(ws.gb)], [wt["recognition_1"]], [v(ws.a1b)], TB, R1, W2, W2, W2, R1,
                      epi=BF_SOFTPLUS, bias=[vb["recognition_1"]])
            gemm_bf16([v(ws.a1b)], [wt["recognition_2"]], [v(ws.a2b)], TB, R2, R1, R1, R1, R2,
                      epi=BF_SOFTPLUS, bias=[vb["recognition_2"]])
            gemm_bf16([v(ws.a2b), v(ws.a2b)], [wt["rec_mean"], wt["rec_log_variance"]],
                      [v(ws.mu), v(ws.lv)], TB, Z, R2, R2, R2, Z, epi=BF_STORE,
                      bias=[vb["rec_mean"], vb["rec_log_variance"]])
            self._vae_sample_fwd_all(ws, v(ws.zb), Zp, t0, t1)
            gemm_bf16([v(ws.zb)], [wt["generative_1"]], [v(ws.d1b)], TB, G1, Zp, Zp, Zp, G1,
                      epi=BF_SOFTPLUS, bias=[vb["generative_1"]])
            gemm_bf16([v(ws.d1b)], [wt["generative_2"]], [v(ws.d2b)], TB, G2, G1, G1, G1, G2,
                      epi=BF_SOFTPLUS, bias=[vb["generative_2"]])
            gemm_bf16([v(ws.d2b)], [wt["gen_mean"]], [v(ws.r)], TB, W2, G2, G2, G2, W2,
                      epi=BF_SIGMOID_NOISE, bias=[vb["gen_mean"]], aux=[v(ws.eps_x)], ldaux=W2,
                      aux_scale=lik_std)
        else:
            vw = {n: self._P("vae/" + n + "/weights") for n in self._VAE}
            ops.stn_forward(X, v(ws.th_f), (W, W), out=v(ws.g), n=TB)
            gemm([v(ws.g)], [vw["recognition_1"]], [v(ws.a1)], TB, R1, W2, W2, R1, R1,
                 epi=EPI_SOFTPLUS, bias=[vb["recognition_1"]])
            gemm([v(ws.a1)], [vw["recognition_2"]], [v(ws.a2)], TB, R2, R1, R1, R2, R2,
                 epi=EPI_SOFTPLUS, bias=[vb["recognition_2"]])
            if self._latent_nt(TB):
                # a small batch: the latent layers as NT products of W^T copies
                # (N = Z / K = Z miss the LDS-DMA alignment, and their row-major
                # form ran on 64 x 64 tiles, a few workgroups); the same
                # k-ordered chains, so the same bits
                wt = self._vae_wT()
                gemm([v(ws.a2), v(ws.a2)], [wt[0], wt[1]], [v(ws.mu), v(ws.lv)], TB, Z, R2, R2,
                     R2, Z, transB=True, bias=[vb["rec_mean"], vb["rec_log_variance"]])
                self._vae_sample_fwd_all(ws, None, 0, t0, t1)
                gemm([v(ws.z)], [wt[2]], [v(ws.d1)], TB, G1, Z, Z, Z, G1, transB=True,
                     epi=EPI_SOFTPLUS, bias=[vb["generative_1"]])
            else:
                gemm([v(ws.a2), v(ws.a2)], [vw["rec_mean"], vw["rec_log_variance"]],
                     [v(ws.mu), v(ws.lv)], TB, Z, R2, R2, Z, Z,
                     bias=[vb["rec_mean"], vb["rec_log_variance"]])
                self._vae_sample_fwd_all(ws, None, 0, t0, t1)
                gemm([v(ws.z)], [vw["generative_1"]], [v(ws.d1)], TB, G1, Z, Z, G1, G1,
                     epi=EPI_SOFTPLUS, bias=[vb["generative_1"]])
            gemm([v(ws.d1)], [vw["generative_2"]], [v(ws.d2)], TB, G2, G1, G1, G2, G2,
                 epi=EPI_SOFTPLUS, bias=[vb["generative_2"]])
            if ws.eps_x_offset is not None:
                # eps_x of steps t0.. in the epilogue: [T, B, W2] fill order
                ops.gemm_sigmoid_philox(v(ws.d2), vw["gen_mean"], v(ws.r), vb["gen_mean"], TB, W2,
                                        G2, G2, W2, W2, lik_std, self.noise_seed,
                                        ws.eps_x_offset + t0 * B * W2 // 4)
            else:
                gemm([v(ws.d2)], [vw["gen_mean"]], [v(ws.r)], TB, W2, G2, G2, W2, W2,
                     epi=EPI_SIGMOID_NOISE, bias=[vb["gen_mean"]],
                     aux=[v(ws.eps_x)], ldaux=W2, aux_scale=lik_std)
        # STN write of every step into its canvas part (air_model.py:580-588);
        # the loss kernel adds the parts in step order (:665-675)
        _ops.stn_write_parts_(v(ws.r), TB, W, W, r_(ws.th_b), C, C, r_(ws.zval), r_(ws.zmask),
                              r_(ws.cparts), r_(ws.prows))

    def _vae_wT(self):
        """W^T of rec_mean, rec_log_variance [Z][R2] and generative_1 [G1][Z],
        transposed in one launch when the parameters changed (a captured step
        records the launch: GraphCapture._capture resets the version)."""
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        buf = self.__dict__.get("_vae_wT_buf")
        if buf is None:
            buf = self.__dict__["_vae_wT_buf"] = [
                torch.empty((Z, R2), device=self.device), torch.empty((Z, R2), device=self.device),
                torch.empty((G1, Z), device=self.device)]
        if getattr(self, "_vae_wT_version", None) != self.params.version:
            _ops.transpose32_batch_(buf, [self._P("vae/" + n + "/weights") for n in
                                          ("rec_mean", "rec_log_variance", "generative_1")])
            self._vae_wT_version = self.params.version
        return buf

    def _latent_nt(self, rows):
        """The latent layers as NT products of W^T copies (_vae_wT) below
        SIDE_MIN_BATCH rows: their N or K = Z misses the LDS-DMA alignment."""
        return self.vae_latent_dimensions % 4 != 0 and rows < self.SIDE_MIN_BATCH

    def _stn_vae_step_bf16(self, TB, C, X, r_, sv, gen, off, wt, bias, lik_std, ws, B):
        """The bf16 fused step over the TB rows of loop steps r_ (x row = row % B)."""
        _ops.stn_vae_step_(TB, C, X, r_(ws.th_f), r_(ws.th_b), r_(ws.zmask), r_(ws.zval),
                           r_(ws.eps_z), r_(ws.eps_x), ops._i64(self.noise_seed), ops._i64(off),
                           gen, wt, bias, lik_std, float(self.vae_prior_mean),
                           float(self.vae_prior_variance), self.vae_prior_log_variance,
                           r_(ws.cparts), r_(ws.prows), None, r_(ws.vkl), sv(ws.gb), sv(ws.a1b),
                           sv(ws.a2b), sv(ws.mu), sv(ws.lv), r_(ws.z), sv(ws.zb), sv(ws.d1b),
                           sv(ws.d2b), r_(ws.r), B)

    def _vae_sample_fwd_all(self, ws, zb, ldzb, t0=0, t1=None):
        t1 = self.max_steps if t1 is None else t1
        TB = ws.B * (t1 - t0)
        r_ = lambda a: a[t0:t1]  # noqa: E731
        _ops.vae_sample_forward_(TB, self.vae_latent_dimensions, float(self.vae_prior_mean),
                                 float(self.vae_prior_variance), self.vae_prior_log_variance,
                                 r_(ws.mu), r_(ws.lv), r_(ws.eps_z), r_(ws.z), zb, ldzb,
                                 r_(ws.zmask), None, r_(ws.vkl))

    def _forward_loss(self, X, targets, ws, need_grad, outputs=True):
        """reconstruction loss (air_model.py:866-900) + batch means.  With
        outputs=False (train steps) the clipped reconstruction and, in the
        fused configuration, the summed canvas are not stored; the
        ``reconstruction`` / ``canvas`` accessors materialize them on demand."""
        B, C2 = ws.B, self.C2
        parts = ws.cparts
        self._loss_inputs = (X, targets)
        ws.materialized = bool(outputs)
        gscale = self._gscale(B)
        canvas = ws.canvas if (outputs or parts is None) else None
        _ops.recon_loss_(X, canvas, parts, self.max_steps if parts is not None else 0, B * C2,
                         ws.prows, self.canvas_size, ws.runloss, ws.digits, targets, B, C2,
                         float(gscale), ws.recon if outputs else None, ws.bce, ws.mse, ws.loss_b,
                         ws.acc_b if targets is not None else None,
                         ws.dcanvas if need_grad else None)
        _ops.batch_mean_(ws.loss_b, ws.acc_b if targets is not None else None, ws.mse, None, B,
                         ws.means)
        self._outputs_ready = True

    def _materialize(self):
        """Store the canvas / reconstruction of the last forward (recomputes
        the loss kernel once with its output pointers; same values)."""
        ws = self._ws
        if ws is None or ws.materialized:
            return
        X, targets = self._loss_inputs
        self._forward_loss(X, targets, ws, need_grad=False, outputs=True)

    # ---------------------------------------------------------- backward ---
    def _backward(self, X: torch.Tensor, ws: _Workspace) -> None:
        """Every loop step's glimpse-path backward (STN write, VAE, STN read,
        heads) depends only on that step's records and dL/dcanvas, so it runs
        once over all T*B rows; only the LSTM chain is sequential."""
        B, T, H = ws.B, self.max_steps, self.rnn_units
        C, W, C2 = self.canvas_size, self.windows_size, self.C2
        HS = self.scale_hidden_units
        TB = T * B
        st = self.params
        # the gradient buffer and the LSTM chain's dG sum, zeroed in one launch
        # (the fp32 x3p x-rows gradient reads every step's dG instead of the
        # sum: mog_split3_sum_bf16)
        if self._x3p_xgrad(B):
            _ops.fill32_batch_([st.grad], [0])
        else:
            _ops.fill32_batch_([st.grad, ws.dGsum], [0, 0])
        # small batch, one GPU: the fp32-chain weight gradients are collected
        # and run as one grouped launch at the end (_wgrad_group_end)
        self._wgroup = (self._wgroup_obj if (self.WGRAD_GROUP and B < self.SIDE_MIN_BATCH
                                             and self.grad_reducer is None) else None)
        wg = self._wgroup
        if wg is not None:
            wg.probs = []  # (a fresh collection: nothing left from a failed step)
        try:
            self._backward_body(X, ws)
        except BaseException:
            if wg is not None:
                wg.probs = []  # a failed body's partial problems never launch
            raise
        finally:
            self._wgroup = None
        if wg is not None and wg.probs:
            flops = sum(2.0 * p[4] * p[5] * p[6] for p in wg.probs)
            with self._timed("wgrad_group", ("mfma", flops, "fp32")):
                wg.launch()

    # the grouped weight-gradient launch below SIDE_MIN_BATCH (batch 64: 11
    # launches of a few k-steps each -> one)
    WGRAD_GROUP = True
    _wgroup = None

    @property
    def _wgroup_obj(self):
        g = self.__dict__.get("_wgroup_obj_")
        if g is None:
            g = self.__dict__["_wgroup_obj_"] = ops.WgradGroup()
        return g

    def _backward_body(self, X: torch.Tensor, ws: _Workspace) -> None:
        B, T, H = ws.B, self.max_steps, self.rnn_units
        C, W, C2 = self.canvas_size, self.windows_size, self.C2
        HS = self.scale_hidden_units
        TB = T * B
        st = self.params
        K = self._P("rnn/basic_lstm_cell/kernel")
        bK = self._P("rnn/basic_lstm_cell/bias")
        Wh = K[C2:]
        w1 = [self._P(h + "/hidden/weights") for h in self._HEADS]
        w2 = [self._P(h + "/output/weights") for h in self._HEADS]
        gscale = self._gscale(B)
        prior_lo = self.hyper("z_pres_prior_log_odds")
        temperature = self.hyper("z_pres_temperature")
        # STN write backward of all steps against the shared canvas gradient
        with self._timed("stn_write_bwd", self._stn_bwd_work(TB, write=True)):
            if self.precision == "bf16":
                # dr leaves through the output sigmoid as bf16 straight from the kernel
                ops.stn_backward(ws.r.view(TB, -1), ws.th_b, (C, C), ws.dcanvas, gscale=ws.zc,
                                 dtheta=ws.dth_b_all, dot=ws.dot_all, want_dot=True, n=TB,
                                 dm_bf16=ws.dmb.view(TB, -1))
            else:  # fp32 dm through the output sigmoid, likewise
                ops.stn_backward(ws.r.view(TB, -1), ws.th_b, (C, C), ws.dcanvas, gscale=ws.zc,
                                 dtheta=ws.dth_b_all, dot=ws.dot_all, want_dot=True, n=TB,
                                 dm=ws.dm.view(TB, -1))
        if self.precision == "bf16":
            self._vae_backward_bf16_all(ws, gscale)
        else:
            self._vae_backward_fp32_all(ws, gscale)
        # The VAE weight gradients need only the activations and the VAE input
        # gradients, final here: they run on a second stream (MFMA-bound
        # split-K GEMMs) under the latency-bound STN read backward and the
        # heads' backward.  Data parallel: the main stream joins them before
        # the glimpse-side all-reduce bucket and the LSTM chain.  One GPU: the
        # heads' weight gradients follow them on the side stream and the join
        # is before Adam, so both overlap the LSTM chain (3.49 -> 3.45 ms;
        # the VAE's alone joined before Adam, heads on the main stream, was
        # measured slower in round 2: 3.74 -> 3.81 ms).
        # (measured: forking them after the STN read backward instead, so that
        # kernel runs alone, is neutral -- 3.097 / 3.094 vs 3.098 / 3.097 ms).
        # Below SIDE_MIN_BATCH everything stays on the main stream (see
        # _vae_weight_grads_async).
        w1_done, vae_done = self._vae_weight_grads_async(ws)
        # STN read backward of all steps against the shared input canvas
        with self._timed("stn_read_bwd", self._stn_bwd_work(TB, write=False)):
            ops.stn_backward(X, ws.th_f, (W, W), ws.dg_all, want_dU=False, dtheta=ws.dth_f_all,
                             n=TB)
        if self.marginal is None:
            # every step's inputs are final here (the STN backwards ran over
            # all T*B rows above): the T steps' head backward in one launch
            _ops.air_step_backward_(
                B, HS, self.train, False, temperature, prior_lo, 0.0,
                float(self.scale_prior_mean), float(self.scale_prior_variance),
                float(self.shift_prior_mean), float(self.shift_prior_variance), float(gscale),
                None, ws.rec, ws.eps_scale, ws.eps_shift, ws.dth_f_all, ws.dth_b_all, ws.dot_all,
                [ws.hid[z] for z in range(5)], w2, ws.dout[0], T * B * 2, ws.dhid, HS,
                self._prior_arg(), T)
        for t in range(T if self.marginal is not None else 0):
            hid_t = [ws.hid[z, t] for z in range(5)]
            _ops.air_step_backward_(
                B, HS, self.train, self.marginal is not None, temperature, prior_lo,
                float(self.marginal[t]) if self.marginal is not None else 0.0,
                float(self.scale_prior_mean), float(self.scale_prior_variance),
                float(self.shift_prior_mean), float(self.shift_prior_variance), float(gscale),
                None, ws.rec[t], ws.eps_scale[t], ws.eps_shift[t], ws.dth_f_all[t], ws.dth_b_all[t],
                ws.dot_all[t], hid_t, w2, ws.dout[0, t], T * B * 2, ws.dhid[t], HS,
                self._prior_arg())
        # dh[t] = sum_z dhid_z W1_z^T for every step: one plain GEMM over
        # K = 5 HS ([dhid_0 .. dhid_4] rows against [W1_0 .. W1_4]), the same
        # k-ordered chain as the per-head sum
        if w1_done is not None:
            torch.cuda.current_stream().wait_event(w1_done)
        if B < self.SIDE_MIN_BATCH and HS % 16 == 0:
            # small batch: the same chain as five k-segments read from the
            # heads' own W1 (no concatenation launch per step)
            dhid = ws.dhid.view(TB, 5 * HS)
            ops.gemm_kseg([dhid[:, z * HS:] for z in range(5)],
                          [self._P(h + "/hidden/weights") for h in self._HEADS], ws.dh, TB, H,
                          HS, 5 * HS, HS, H, transB=True)
        else:
            gemm([ws.dhid], [self._w1cat()], [ws.dh], TB, H, 5 * HS, 5 * HS, 5 * HS, H,
                 transB=True)
        heads_side = (self.grad_reducer is None and self.HEADS_WGRAD_SIDE
                      and B >= self.SIDE_MIN_BATCH)
        if heads_side:
            # one GPU, no bucket to hand over: the heads' weight gradients
            # follow the VAE's on the side stream, under the latency-bound
            # LSTM chain; the main stream joins them before Adam
            # -- on a third stream, beside the VAE's instead of queued after
            # them (fp32 step 3.10 -> 3.05 ms)
            with torch.cuda.stream(self._fork(self._stream3())):
                self._weight_grads_heads(ws)
        else:
            # the heads' and the VAE's weight gradients are final here: their
            # all-reduce bucket runs while the LSTM chain below computes
            self._weight_grads_heads(ws)
            if vae_done is not None:
                torch.cuda.current_stream().wait_event(vae_done)
            split = self._bucket_split()
            self._reduce_bucket(split, self.params.total)
        rec_early = T > 1 and heads_side and self.REC_WGRAD_SIDE
        dGsum = None if self._x3p_xgrad(B) else ws.dGsum
        # a small batch's dh GEMM (K = 4H walked serially by a dozen workgroups)
        # split over K into DH_PARTS products that the next cell backward adds
        # to the heads' dh in part order (mog_lstm_cell_backward_parts)
        parts = self.DH_PARTS if (B < self.SIDE_MIN_BATCH and self.DH_PARTS > 1
                                  and (4 * H) % (4 * self.DH_PARTS) == 0) else 0
        if parts and getattr(ws, "dh_parts", None) is None:
            ws.dh_parts = torch.empty((parts, B, H), device=self.device)
        for t in reversed(range(T)):
            dc_in = ws.dc[(t + 1) % 2] if t < T - 1 else None
            G_t, b_t = (ws.Gx, bK) if t == 0 else (ws.G[t], None)
            c_prev = ws.c[t - 1] if t > 0 else None
            if parts and t < T - 1:
                _ops.lstm_cell_backward_parts_(G_t, b_t, c_prev, ws.c[t], ws.dh[t], ws.dh_parts,
                                               parts, dc_in, ws.dG[t], ws.dc[t % 2], dGsum, B, H)
            else:
                _ops.lstm_cell_backward_(G_t, b_t, c_prev, ws.c[t], ws.dh[t], dc_in, ws.dG[t],
                                         ws.dc[t % 2], dGsum, B, H)
            if t == 1 and rec_early:
                # dG[1:] is final: the recurrent rows' gradient runs beside the
                # chain's last step instead of beside the x-rows gradient
                self._weight_grads_rec_side(ws)
            if t > 0 and parts:
                kp = 4 * H // parts
                gemm([ws.dG[t][:, j * kp:] for j in range(parts)],
                     [Wh[:, j * kp:] for j in range(parts)], [ws.dh_parts[j] for j in range(parts)],
                     B, H, kp, 4 * H, 4 * H, H, transB=True)
            elif t > 0:
                gemm([ws.dG[t]], [Wh], [ws.dh[t - 1]], B, H, 4 * H, 4 * H, 4 * H, H,
                     transB=True, Cin=[ws.dh[t - 1]])
        self._weight_grads_lstm(X, ws, side=heads_side, rec_done=rec_early)
        if heads_side:  # (everything on the side stream: VAE, heads, dW_rec)
            torch.cuda.current_stream().wait_stream(self._side_stream())
            torch.cuda.current_stream().wait_stream(self._stream3())

    # single GPU: heads' weight gradients on the side stream (see _backward)
    HEADS_WGRAD_SIDE = True
    # ... and the LSTM kernel's recurrent-rows gradient beside the x-rows one
    REC_WGRAD_SIDE = True
    # K-split of the small-batch dh GEMM (0: one chain per output, Cin = the
    # heads' dh)
    DH_PARTS = 4
    # the round-3 side-stream moves (noise + resets under the x-projection,
    # heads' weight gradients under the LSTM chain) from this batch: below it
    # the launches are too short to hide the cross-stream waits (batch 64:
    # eager 0.90 -> 1.00 ms, captured 0.60 -> 0.65 ms with them)
    SIDE_MIN_BATCH = 1024

    # fp32 configuration: the VAE input gradients dX = dY W^T of the 256- to
    # 784-wide layers on the bf16 matrix cores with exact three-piece splits
    # (gemm_x3.hip NT form: dY split in the kernel, W split once per optimizer
    # step) -- the chain is on the step's critical path; fp32-level accuracy
    # like the weight gradients.  False: the fp32 MFMA GEMMs.
    VAE_DX_X3 = True
    _X3_DX = ("gen_mean", "generative_2", "recognition_2", "recognition_1")

    def _w3(self):
        """The three bf16 pieces of the VAE weights the x3 input gradients read
        (W [in][out] -> [3][in][out]), refreshed when the parameters change."""
        if getattr(self, "_w3_version", None) != self.params.version:
            if getattr(self, "_w3_buf", None) is None:
                self._w3_buf = {}
                for n in self._X3_DX:
                    I, O = self._P("vae/" + n + "/weights").shape
                    self._w3_buf[n] = torch.empty((3, I, O), device=self.device,
                                                  dtype=torch.bfloat16)
            for n in self._X3_DX:
                w = self._P("vae/" + n + "/weights")
                I, O = w.shape
                ops.split3_bf16(w, self._w3_buf[n], I, O, O, O, I * O)
            self._w3_version = self.params.version
        return self._w3_buf

    def _stn_bwd_work(self, rows, write):
        """Algorithmic HBM bytes of one STN backward launch over `rows` image-
        steps: write -- r and dm (C2... of the glimpse), the
        canvas cotangent shared by the T steps of an image, theta / dtheta /
        dot; read -- the input canvas shared likewise, the glimpse cotangent,
        theta / dtheta."""
        W2, C2, T = self.W2, self.C2, self.max_steps
        if write:
            dm = 2 if self.precision == "bf16" else 4
            return ("hbm", rows * (W2 * 4 + W2 * dm + C2 * 4 / T + 52), None)
        return ("hbm", rows * (C2 * 4 / T + W2 * 4 + 48), None)

    def _dx(self, dY, name, out, M, N, K, aux=None):
        """out[M,N] = dY W^T (W = vae/name/weights [N][K]) [* sigmoid(aux)]."""
        if self.VAE_DX_X3 and K % 8 == 0 and N % 4 == 0 and M >= self.X3_DX_MIN_ROWS:
            w3 = self._w3()[name]
            # six bf16 MFMA products per fp32 product (gemm_x3.hip)
            with self._timed("vae_dgrad_x3", ("mfma", 2.0 * M * N * K, "fp32", "x3")):
                ops.gemm_x3_nt(dY, w3, N * K, out, M, N, K, K, K, N, aux=aux,
                               ldaux=N if aux is not None else 0)
            return
        with self._timed("vae_dgrad_f32", ("mfma", 2.0 * M * N * K, "fp32")):
            gemm([dY], [self._P("vae/" + name + "/weights")], [out], M, N, K, K, K, N, transB=True,
                 epi=EPI_SOFTPLUS_BWD if aux is not None else EPI_STORE,
                 aux=[aux] if aux is not None else None, ldaux=N if aux is not None else 0)

    def _vae_backward_fp32_all(self, ws, gscale):
        TB = ws.B * self.max_steps
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        vw = {n: self._P("vae/" + n + "/weights") for n in self._VAE}
        # dm = SigmoidGrad(r, dr) was written by the STN write backward
        # (aux = the softplus outputs: epi 4 / NT epi 1 take sigmoid(x) as
        # 1 - exp(-softplus(x)))
        self._dx(ws.dm, "gen_mean", ws.dd2, TB, G2, W2, aux=ws.d2)
        self._dx(ws.dd2, "generative_2", ws.dd1, TB, G1, G2, aux=ws.d1)
        gemm([ws.dd1], [vw["generative_1"]], [ws.dz_all], TB, Z, G1, G1, G1, Z, transB=True)
        _ops.vae_sample_backward_(TB, Z, float(self.vae_prior_mean),
                                  float(self.vae_prior_variance), float(gscale), ws.mu, ws.lv,
                                  ws.eps_z, ws.dz_all, ws.zmask, ws.dmu, ws.dlv, None, None, 0)
        gemm([ws.dmu], [vw["rec_mean"]], [ws.tmp_a2_all], TB, R2, Z, Z, Z, R2, transB=True)
        gemm([ws.dlv], [vw["rec_log_variance"]], [ws.da2], TB, R2, Z, Z, Z, R2,
             transB=True, epi=EPI_SOFTPLUS_BWD, Cin=[ws.tmp_a2_all], aux=[ws.a2], ldaux=R2)
        self._dx(ws.da2, "recognition_2", ws.da1, TB, R1, R2, aux=ws.a1)
        self._dx(ws.da1, "recognition_1", ws.dg_all, TB, W2, R1)

    def _vae_backward_bf16_all(self, ws, gscale):
        from .ops import BF_SOFTPLUS_BWD, BF_STORE, gemm_bf16
        TB = ws.B * self.max_steps
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        Zp = self._pad8(Z)
        wn = self._wn
        # dmb = bf16(SigmoidGrad(r, dr)) was written by the STN write backward
        gemm_bf16([ws.dmb], [wn["gen_mean"]], [ws.dd2b], TB, G2, W2, W2, W2, G2,
                  epi=BF_SOFTPLUS_BWD, aux=[ws.d2b], ldaux=G2)
        gemm_bf16([ws.dd2b], [wn["generative_2"]], [ws.dd1b], TB, G1, G2, G2, G2, G1,
                  epi=BF_SOFTPLUS_BWD, aux=[ws.d1b], ldaux=G1)
        gemm_bf16([ws.dd1b], [wn["generative_1"]], [ws.dz_all], TB, Z, G1, G1, G1, Z,
                  epi=BF_STORE)
        _ops.vae_sample_backward_(TB, Z, float(self.vae_prior_mean),
                                  float(self.vae_prior_variance), float(gscale), ws.mu, ws.lv,
                                  ws.eps_z, ws.dz_all, ws.zmask, None, None, ws.dmub, ws.dlvb, Zp)
        gemm_bf16([ws.dmub], [wn["rec_mean"]], [ws.tmp_a2_all], TB, R2, Zp, Zp, Zp, R2,
                  epi=BF_STORE)
        gemm_bf16([ws.dlvb], [wn["rec_log_variance"]], [ws.da2b], TB, R2, Zp, Zp, Zp, R2,
                  epi=BF_SOFTPLUS_BWD, Cin=[ws.tmp_a2_all], aux=[ws.a2b], ldaux=R2)
        gemm_bf16([ws.da2b], [wn["recognition_2"]], [ws.da1b], TB, R1, R2, R2, R2, R1,
                  epi=BF_SOFTPLUS_BWD, aux=[ws.a1b], ldaux=R1)
        gemm_bf16([ws.da1b], [wn["recognition_1"]], [ws.dg_all], TB, W2, R1, R1, R1, W2,
                  epi=BF_STORE)

    # ------------------------------------------------------ glimpse VAE ----
    def _vae_dims(self):
        R1, R2 = self.vae_recognition_units
        G1, G2 = self.vae_generative_units
        return self.W2, R1, R2, self.vae_latent_dimensions, G1, G2

    def _vae_forward_fp32(self, X, ws, t, lik_std):
        self._vae_encoder_fp32(X, ws, t)
        self._vae_decoder_fp32(ws, lik_std, t, t + 1)

    def _vae_encoder_fp32(self, X, ws, t):
        """STN read -> recognition layers -> z sample of loop step t."""
        B, W = ws.B, self.windows_size
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        vw = {n: self._P("vae/" + n + "/weights") for n in self._VAE}
        vb = {n: self._P("vae/" + n + "/biases") for n in self._VAE}
        ops.stn_forward(X, ws.th_f[t], (W, W), out=ws.g[t])
        gemm([ws.g[t]], [vw["recognition_1"]], [ws.a1[t]], B, R1, W2, W2, R1, R1,
             epi=EPI_SOFTPLUS, bias=[vb["recognition_1"]])
        gemm([ws.a1[t]], [vw["recognition_2"]], [ws.a2[t]], B, R2, R1, R1, R2, R2,
             epi=EPI_SOFTPLUS, bias=[vb["recognition_2"]])
        if self._latent_nt(B):
            wt = self._vae_wT()
            gemm([ws.a2[t], ws.a2[t]], wt[:2], [ws.mu[t], ws.lv[t]], B, Z, R2, R2, R2, Z,
                 transB=True, bias=[vb["rec_mean"], vb["rec_log_variance"]])
        else:
            gemm([ws.a2[t], ws.a2[t]], [vw["rec_mean"], vw["rec_log_variance"]],
                 [ws.mu[t], ws.lv[t]], B, Z, R2, R2, Z, Z,
                 bias=[vb["rec_mean"], vb["rec_log_variance"]])
        self._vae_sample_fwd(ws, t, None, 0)

    def _vae_decoder_fp32(self, ws, lik_std, t0, t1):
        """Generative layers of loop steps [t0, t1) over their rows at once
        (rows are independent: the same chains as step by step)."""
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        n = (t1 - t0) * ws.B
        v = lambda a: a[t0:t1].reshape(n, -1)  # noqa: E731
        vw = {k: self._P("vae/" + k + "/weights") for k in self._VAE[4:]}
        vb = {k: self._P("vae/" + k + "/biases") for k in self._VAE[4:]}
        if self._latent_nt(n):
            gemm([v(ws.z)], [self._vae_wT()[2]], [v(ws.d1)], n, G1, Z, Z, Z, G1, transB=True,
                 epi=EPI_SOFTPLUS, bias=[vb["generative_1"]])
        else:
            gemm([v(ws.z)], [vw["generative_1"]], [v(ws.d1)], n, G1, Z, Z, G1, G1,
                 epi=EPI_SOFTPLUS, bias=[vb["generative_1"]])
        gemm([v(ws.d1)], [vw["generative_2"]], [v(ws.d2)], n, G2, G1, G1, G2, G2,
             epi=EPI_SOFTPLUS, bias=[vb["generative_2"]])
        gemm([v(ws.d2)], [vw["gen_mean"]], [v(ws.r)], n, W2, G2, G2, W2, W2,
             epi=EPI_SIGMOID_NOISE, bias=[vb["gen_mean"]],
             aux=[v(ws.eps_x)], ldaux=W2, aux_scale=lik_std)

    def _vae_sample_fwd(self, ws, t, zb, ldzb):
        _ops.vae_sample_forward_(ws.B, self.vae_latent_dimensions, float(self.vae_prior_mean),
                                 float(self.vae_prior_variance), self.vae_prior_log_variance,
                                 ws.mu[t], ws.lv[t], ws.eps_z[t], ws.z[t], zb, ldzb,
                                 ws.zmask[t], ws.runloss, ws.vkl[t])

    def _dz_hook(self, ws, t, dz):
        """Extra gradient reaching the latent z of step t (in dz) before the
        sample backward (none in AIR; the ASR model adds the next step's
        LSTM-input gradient here)."""

    def _vae_decoder_backward_all(self, ws):
        """The decoder half of every loop step's VAE backward over all T*B
        rows (dm -> dd2 -> dd1 -> dz_all; dm already through the output
        sigmoid), for a loop that needs only the encoder half per step: the
        AIR-ASR reversed loop, whose dz_t takes the next step's carry (the
        same chains as the per-step launches, so the same values)."""
        T, B = self.max_steps, ws.B
        TB = T * B
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        if getattr(ws, "dz_all", None) is None:
            ws.dz_all = torch.empty((T, B, Z), device=self.device)
        v = lambda x: x.view(TB, -1)  # noqa: E731
        if self.precision == "bf16":
            from .ops import BF_SOFTPLUS_BWD, BF_STORE, gemm_bf16
            wn = self._wn
            gemm_bf16([v(ws.dmb)], [wn["gen_mean"]], [v(ws.dd2b)], TB, G2, W2, W2, W2, G2,
                      epi=BF_SOFTPLUS_BWD, aux=[v(ws.d2b)], ldaux=G2)
            gemm_bf16([v(ws.dd2b)], [wn["generative_2"]], [v(ws.dd1b)], TB, G1, G2, G2, G2, G1,
                      epi=BF_SOFTPLUS_BWD, aux=[v(ws.d1b)], ldaux=G1)
            gemm_bf16([v(ws.dd1b)], [wn["generative_1"]], [v(ws.dz_all)], TB, Z, G1, G1, G1, Z,
                      epi=BF_STORE)
        else:
            self._dx(v(ws.dm), "gen_mean", v(ws.dd2), TB, G2, W2, aux=v(ws.d2))
            self._dx(v(ws.dd2), "generative_2", v(ws.dd1), TB, G1, G2, aux=v(ws.d1))
            gemm([v(ws.dd1)], [self._P("vae/generative_1/weights")], [v(ws.dz_all)], TB, Z, G1, G1,
                 G1, Z, transB=True)
        ws.dec_ready = True

    def _vae_backward_fp32(self, ws, t, gscale):
        B = ws.B
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        vw = {n: self._P("vae/" + n + "/weights") for n in self._VAE}
        if getattr(ws, "dec_ready", False):  # (the decoder half ran over T*B rows)
            dz = ws.dz_all[t]
        else:
            dz = ws.dz
            if not getattr(ws, "dm_ready", False):
                _ops.sigmoid_backward_(ws.r[t], ws.dr, ws.dm[t], B * W2)
            self._dx(ws.dm[t], "gen_mean", ws.dd2[t], B, G2, W2, aux=ws.d2[t])
            self._dx(ws.dd2[t], "generative_2", ws.dd1[t], B, G1, G2, aux=ws.d1[t])
            gemm([ws.dd1[t]], [vw["generative_1"]], [dz], B, Z, G1, G1, G1, Z, transB=True)
        self._dz_hook(ws, t, dz)
        _ops.vae_sample_backward_(B, Z, float(self.vae_prior_mean),
                                  float(self.vae_prior_variance), float(gscale), ws.mu[t],
                                  ws.lv[t], ws.eps_z[t], dz, ws.zmask[t], ws.dmu[t], ws.dlv[t],
                                  None, None, 0)
        gemm([ws.dmu[t]], [vw["rec_mean"]], [ws.tmp_a2], B, R2, Z, Z, Z, R2, transB=True)
        gemm([ws.dlv[t]], [vw["rec_log_variance"]], [ws.da2[t]], B, R2, Z, Z, Z, R2,
             transB=True, epi=EPI_SOFTPLUS_BWD, Cin=[ws.tmp_a2], aux=[ws.a2[t]], ldaux=R2)
        self._dx(ws.da2[t], "recognition_2", ws.da1[t], B, R1, R2, aux=ws.a1[t])
        self._dx(ws.da1[t], "recognition_1", ws.dg, B, W2, R1)

    # bf16 configuration: VAE GEMM operands bf16 (fp32 accumulate), activations
    # stored bf16 (post-activation only: softplus' = 1 - exp(-softplus)), the
    # LSTM / heads / STN / canvas / losses stay fp32.
    @staticmethod
    def _pad8(n):
        return (n + 7) // 8 * 8

    def _pack_bf16(self):
        """Refresh the bf16 weight packs after a parameter update (one batched
        launch): wn[name] = W [in][out8] (dX B operand) and either
        wf[name] = W^T in MFMA B-fragment order (fused step kernel) or
        wt[name] = W^T [out][in8] (unfused forward GEMMs)."""
        if getattr(self, "_pack_version", None) == self.params.version:
            return
        if not hasattr(self, "_pack_args"):
            bf = dict(device=self.device, dtype=torch.bfloat16)
            self._wt, self._wn, self._wf = {}, {}, {}
            srcs, dsts, dims = [], [], []
            for n in self._VAE:
                w = self._P("vae/" + n + "/weights")
                I, O = w.shape
                wn = self._wn[n] = torch.zeros((I, self._pad8(O)), **bf)
                if self.fused_step:
                    Np, Kp = (O + 15) // 16 * 16, (I + 31) // 32 * 32
                    wf = self._wf[n] = torch.zeros((Np, Kp), **bf)
                    fwd, fdims = wf, [I, O, O, Np, Kp, Kp, 2]
                else:
                    wt = self._wt[n] = torch.zeros((O, self._pad8(I)), **bf)
                    fwd, fdims = wt, [I, O, O, O, wt.shape[1], wt.shape[1], 1]
                srcs += [w, w]
                dsts += [fwd, wn]
                dims += fdims + [I, O, O, I, wn.shape[1], wn.shape[1], 0]
            self._pack_args = (srcs, dsts, dims)
        _ops.cvt_bf16_batch_(*self._pack_args)
        self._pack_version = self.params.version

    def _pack_f32(self):
        """Refresh the fp32 MFMA B-fragment packs of the VAE weights (the fp32
        fused step's weight operand) after a parameter update: one launch."""
        if getattr(self, "_pack32_version", None) == self.params.version:
            return
        if not hasattr(self, "_pack32_args"):
            ws_, ks, ns, outs = [], [], [], []
            for n in self._VAE:
                w = self._P("vae/" + n + "/weights")
                K, N = w.shape
                ws_.append(w)
                ks.append(int(K))
                ns.append(int(N))
                outs.append(torch.empty(((K + 15) // 16) * ((N + 15) // 16) * 256,
                                        device=self.device))
            self._wf32 = outs
            self._pack32_args = (ws_, ks, ns, outs)
        _ops.pack_frag_f32_(*self._pack32_args)
        self._pack32_version = self.params.version

    def _vae_forward_bf16(self, X, ws, t, lik_std):
        from .ops import BF_SIGMOID_NOISE, BF_SOFTPLUS, BF_STORE, gemm_bf16
        B, W = ws.B, self.windows_size
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        Zp = self._pad8(Z)
        self._pack_bf16()
        wt = self._wt
        vb = {n: self._P("vae/" + n + "/biases") for n in self._VAE}
        ops.stn_forward(X, ws.th_f[t], (W, W), out=ws.gb[t])
        gemm_bf16([ws.gb[t]], [wt["recognition_1"]], [ws.a1b[t]], B, R1, W2, W2, W2, R1,
                  epi=BF_SOFTPLUS, bias=[vb["recognition_1"]])
        gemm_bf16([ws.a1b[t]], [wt["recognition_2"]], [ws.a2b[t]], B, R2, R1, R1, R1, R2,
                  epi=BF_SOFTPLUS, bias=[vb["recognition_2"]])
        gemm_bf16([ws.a2b[t], ws.a2b[t]], [wt["rec_mean"], wt["rec_log_variance"]],
                  [ws.mu[t], ws.lv[t]], B, Z, R2, R2, R2, Z, epi=BF_STORE,
                  bias=[vb["rec_mean"], vb["rec_log_variance"]])
        self._vae_sample_fwd(ws, t, ws.zb[t], Zp)
        gemm_bf16([ws.zb[t]], [wt["generative_1"]], [ws.d1b[t]], B, G1, Zp, Zp, Zp, G1,
                  epi=BF_SOFTPLUS, bias=[vb["generative_1"]])
        gemm_bf16([ws.d1b[t]], [wt["generative_2"]], [ws.d2b[t]], B, G2, G1, G1, G1, G2,
                  epi=BF_SOFTPLUS, bias=[vb["generative_2"]])
        gemm_bf16([ws.d2b[t]], [wt["gen_mean"]], [ws.r[t]], B, W2, G2, G2, G2, W2,
                  epi=BF_SIGMOID_NOISE, bias=[vb["gen_mean"]], aux=[ws.eps_x[t]], ldaux=W2,
                  aux_scale=lik_std)

    def _step_fused(self, X, ws, t, lik_std, save=True):
        """STN read + VAE + latent sample/KL + STN write-accumulate in one launch
        (vae_step.hip; same arithmetic as the unfused bf16 sequence).
        save=False: forward only, the backward's activations are not written."""
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        self._pack_bf16()
        if self.windows_size != 28 or (R1, R2, Z, G1, G2) != (512, 256, 50, 256, 512):
            raise ValueError("the fused step kernel is compiled for the reference VAE shape")
        wt = [self._wf[n] for n in self._VAE]
        gen = getattr(ws, "eps_x_offset", None) is not None
        off = ws.eps_x_offset + t * ws.B * (W2 // 4) if gen else 0
        bias = [self._P("vae/" + n + "/biases") for n in self._VAE]
        _ops.stn_vae_step_(ws.B, self.canvas_size, X, ws.th_f[t], ws.th_b[t], ws.zmask[t],
                           ws.zval[t], ws.eps_z[t], ws.eps_x[t], ops._i64(self.noise_seed),
                           ops._i64(off), gen, wt, bias, lik_std, float(self.vae_prior_mean),
                           float(self.vae_prior_variance), self.vae_prior_log_variance,
                           ws.cparts[t], ws.prows[t], ws.runloss, ws.vkl[t], ws.gb[t],
                           *(a[t] if save else None for a in (ws.a1b, ws.a2b, ws.mu, ws.lv)),
                           ws.z[t], ws.zb[t] if save else None, ws.d1b[t] if save else None,
                           ws.d2b[t] if save else None, ws.r[t])

    def _vae_backward_bf16(self, ws, t, gscale):
        from .ops import BF_SOFTPLUS_BWD, BF_STORE, gemm_bf16
        B = ws.B
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        Zp = self._pad8(Z)
        wn = self._wn
        if getattr(ws, "dec_ready", False):  # (the decoder half ran over T*B rows)
            dz = ws.dz_all[t]
        else:
            dz = ws.dz
            if not getattr(ws, "dm_ready", False):
                _ops.sigmoid_backward_(ws.r[t], ws.dr, ws.dmb[t], B * W2)
            gemm_bf16([ws.dmb[t]], [wn["gen_mean"]], [ws.dd2b[t]], B, G2, W2, W2, W2, G2,
                      epi=BF_SOFTPLUS_BWD, aux=[ws.d2b[t]], ldaux=G2)
            gemm_bf16([ws.dd2b[t]], [wn["generative_2"]], [ws.dd1b[t]], B, G1, G2, G2, G2, G1,
                      epi=BF_SOFTPLUS_BWD, aux=[ws.d1b[t]], ldaux=G1)
            gemm_bf16([ws.dd1b[t]], [wn["generative_1"]], [dz], B, Z, G1, G1, G1, Z,
                      epi=BF_STORE)
        self._dz_hook(ws, t, dz)
        _ops.vae_sample_backward_(B, Z, float(self.vae_prior_mean),
                                  float(self.vae_prior_variance), float(gscale), ws.mu[t],
                                  ws.lv[t], ws.eps_z[t], dz, ws.zmask[t], None, None,
                                  ws.dmub[t], ws.dlvb[t], Zp)
        gemm_bf16([ws.dmub[t]], [wn["rec_mean"]], [ws.tmp_a2], B, R2, Zp, Zp, Zp, R2,
                  epi=BF_STORE)
        gemm_bf16([ws.dlvb[t]], [wn["rec_log_variance"]], [ws.da2b[t]], B, R2, Zp, Zp, Zp, R2,
                  epi=BF_SOFTPLUS_BWD, Cin=[ws.tmp_a2], aux=[ws.a2b[t]], ldaux=R2)
        gemm_bf16([ws.da2b[t]], [wn["recognition_2"]], [ws.da1b[t]], B, R1, R2, R2, R2, R1,
                  epi=BF_SOFTPLUS_BWD, aux=[ws.a1b[t]], ldaux=R1)
        gemm_bf16([ws.da1b[t]], [wn["recognition_1"]], [ws.dg], B, W2, R1, R1, R1, W2,
                  epi=BF_STORE)

    # the side and third streams are created once per process and device and
    # shared by every model (see _shared_streams)
    def _stream3(self):
        return _shared_streams(self.device)[1]

    def _side_stream(self):
        return _shared_streams(self.device)[0]

    # stream-ordering test instrument (tests/test_gpu_streams.py): ticks of the
    # 100 MHz wall clock that a spin kernel holds back the head of every forked
    # segment (SPIN_FORK) or the main stream at the start of a step (SPIN_MAIN)
    SPIN_FORK = 0
    SPIN_MAIN = 0

    def _fork(self, stream):
        """Order `stream` after everything issued so far on the current
        stream; returns it."""
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream())
        stream.wait_event(ready)
        if self.SPIN_FORK:
            with torch.cuda.stream(stream):
                ops.spin(self.SPIN_FORK)
        return stream

    # ------------------------------------------------------------- API ----
    def _prep(self, images, targets):
        X = torch.as_tensor(images, dtype=torch.float32).to(self.device).reshape(-1, self.C2)
        X = X.contiguous()
        tg = None
        if targets is not None:
            tg = torch.as_tensor(targets).to(self.device, torch.int32).contiguous()
        return X, tg

    def train_step_async(self, images, targets=None, noise=None,
                         global_batch: Optional[int] = None) -> None:
        """One train step (forward, backward, [bucketed all-reduce], clip,
        Adam) with no host synchronisation.  ``global_batch``: images over all
        data-parallel ranks this step (default: local batch x grad_world)."""
        if not self.train:
            raise RuntimeError("train_step on a model built with train=False")
        X, tg = self._prep(images, targets)
        ws = self._workspace(X.shape[0])
        ws.alloc_backward(self)
        if self.SPIN_MAIN:
            ops.spin(self.SPIN_MAIN)
        self._fill_noise(ws, noise)
        self._global_batch = global_batch
        self._forward(X, tg, ws, need_grad=True, outputs=False)
        self._backward(X, ws)
        if self.grad_reducer is not None:
            self.grad_reducer.wait()
        self.params.apply_adam(self.hyper("learning_rate"), self.gradient_clipping_norm)
        self.params.global_step += 1
        self._X = X

    def step(self, images, targets=None, noise=None, global_batch: Optional[int] = None):
        """``sess.run([training, loss, accuracy, mse_loss, global_step])``
        (training_air_original.py:304-310)."""
        self.train_step_async(images, targets, noise, global_batch)
        m = self._ws.means.detach().cpu().numpy()
        return float(m[0]), float(m[1]), float(m[2]), self.params.global_step

    def compute_gradients(self, images, targets=None, noise=None, canvas_cotangent=None,
                          global_batch: Optional[int] = None):
        """Forward + backward (+ the data-parallel all-reduce when attached),
        no optimizer update; returns the gradient dict.  ``canvas_cotangent``
        [B, C*C] replaces dL/dcanvas of the BCE term (used by the gradient
        parity tests)."""
        X, tg = self._prep(images, targets)
        ws = self._workspace(X.shape[0])
        ws.alloc_backward(self)
        if self.SPIN_MAIN:
            ops.spin(self.SPIN_MAIN)
        self._fill_noise(ws, noise)
        self._global_batch = global_batch
        self._forward(X, tg, ws, need_grad=True)
        if canvas_cotangent is not None:
            ws.dcanvas.copy_(torch.as_tensor(canvas_cotangent, dtype=torch.float32))
        self._backward(X, ws)
        if self.grad_reducer is not None:
            self.grad_reducer.wait()
        return self.params.grad_dict()

    def infer(self, images, targets=None, noise=None):
        """Forward pass only (the test model's fetches)."""
        X, tg = self._prep(images, targets)
        ws = self._workspace(X.shape[0])
        self._fill_noise(ws, noise)
        self._forward(X, tg, ws, need_grad=False)
        self._X = X
        return self
