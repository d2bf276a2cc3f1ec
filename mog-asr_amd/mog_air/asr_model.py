"""AIRModel of AIR-ASR — drop-in host object for the reference's
air/air_number_bbox_location.py:13-1361 (the model train_air_pr.py builds),
running on MI355X HIP kernels: the inference and generative LSTMCells (fp32
MFMA GEMMs with the loop-invariant x-projection hoisted), the heads and the
structural regularisers (asr_cell.hip), and the glimpse path shared with the
AIR model (STN read, glimpse VAE — fused bf16 step kernel or fp32 GEMMs —,
STN write, reconstruction loss).

Reference surface kept (air_number_bbox_location.py:15-56, train_air_pr.py:
160-213): the constructor keyword arguments (cnn=True and
fix_scale_distribution=False are rejected: the entry point uses neither), the
train / test pair sharing one scope via ``reuse``, the loss of :1078-1079
with every regulariser, and the result attributes (``loss, accuracy,
mse_loss, rec_num_digits, rec_scales, rec_shifts, rec_st_back, rec_windows,
rec_latents, z_pres_probs, reconstruction, log_variables``).

Loop: max_steps iterations on the device, the data-dependent predicate
(:386-390) folded into a live flag per step; losses, counts and gradients
equal the early exit.  The KL records are summed per type over the executed
steps at the end, as the reference's TensorArrays are (:917-923).
"""
from __future__ import annotations

from typing import Dict

import torch

from . import _lib, ops
from .air_model import AIRModel as _AirBase
from .air_model import _SCOPES, _Workspace, _f32log
from .ops import EPI_RELU, EPI_STORE, gemm
from .params import ParamStore

_ops = ops._ops  # torch.ops.mog_air (csrc/torch_ops.cpp)

# asr_cell.hip record slots
Q = {n: i for i, n in enumerate(
    ("sm0 sm1 slv0 slv1 sl0 sl1 cm clv cl s tx ty gsm0 gsm1 gslv0 gslv1 plo lo y z act_old act "
     "live zkl skl shkl prn zprob").split())}
NQ = 28
D_N = 12
LU = 312  # packed LSTM-input row: z (50) | latents (3) | h (256) | pad (3)

ROOT = "air/air_model/"


def asr_param_specs(C2, H, W2, R, G, Z, HS, HZ):
    """(TF variable name, shape): inference / generative LSTMCell kernels on
    the concatenated inputs, tf.layers.dense heads numbered in creation order
    within their scopes (:414-474, :590-609), the glimpse VAE (vae.py)."""
    p = ROOT
    specs = [(p + "infer_rnn_running/kernel", (C2 + Z + 3 + H, 4 * H)),
             (p + "infer_rnn_running/bias", (4 * H,)),
             (p + "gen_rnn_running/kernel", (Z + 3 + H, 4 * H)),
             (p + "gen_rnn_running/bias", (4 * H,))]

    def four(scope, kin, kout, extra):
        return [(p + scope + "/dense/kernel", (kin, HS)), (p + scope + "/dense/bias", (HS,)),
                (p + scope + "/dense_1/kernel", (HS + extra, kout)),
                (p + scope + "/dense_1/bias", (kout,)),
                (p + scope + "/dense_2/kernel", (kin, HS)), (p + scope + "/dense_2/bias", (HS,)),
                (p + scope + "/dense_3/kernel", (HS + extra, kout)),
                (p + scope + "/dense_3/bias", (kout,))]

    specs += four("inf_shift", H, 2, 0) + four("inf_scale", H + 2, 1, 2) + four("gen_shift", H, 2, 0)
    for scope in ("z_pres/prior", "z_pres/log_odds"):
        specs += [(p + scope + "/dense/kernel", (H, HZ)), (p + scope + "/dense/bias", (HZ,)),
                  (p + scope + "/dense_1/kernel", (HZ, 1)), (p + scope + "/dense_1/bias", (1,))]
    v = p + "vae/"
    R1, R2 = R
    G1, G2 = G
    specs += [(v + "recognition_1/weights", (W2, R1)), (v + "recognition_1/biases", (R1,)),
              (v + "recognition_2/weights", (R1, R2)), (v + "recognition_2/biases", (R2,)),
              (v + "rec_mean/weights", (R2, Z)), (v + "rec_mean/biases", (Z,)),
              (v + "rec_log_variance/weights", (R2, Z)), (v + "rec_log_variance/biases", (Z,)),
              (v + "generative_1/weights", (Z, G1)), (v + "generative_1/biases", (G1,)),
              (v + "generative_2/weights", (G1, G2)), (v + "generative_2/biases", (G2,)),
              (v + "gen_mean/weights", (G2, W2)), (v + "gen_mean/biases", (W2,))]
    return specs


class _AsrWorkspace(_Workspace):
    def __init__(self, m: "AIRModel", B: int):
        super().__init__(m, B)
        dev = m.device
        T, H = m.max_steps, m.rnn_units
        e = lambda *s: torch.empty(s, device=dev, dtype=torch.float32)  # noqa: E731
        self.U, self.Ug = e(T, B, LU), e(T, B, LU)
        self.Gg, self.cg, self.hg = e(T, B, 4 * H), e(T, B, H), e(T, B, H)
        self.hid8 = e(8, T, B, 64)
        self.arec = e(T, NQ, B)
        self.ss = e(T, B, 3)
        self.zc = e(T, B)
        self.klsum, self.pr, self.element = e(B), e(B), e(B)
        self.area, self.outl, self.size, self.over = e(B), e(B), e(B), e(B)
        self.zsum = e(T)
        self.margin = e(1)
        # hg_{-1}: the zero state the learned prior reads at step 0
        self.hg_zero = torch.zeros((B, H), device=dev, dtype=torch.float32)

    def alloc_backward(self, m):
        if self._bwd:
            return
        super().alloc_backward(m)
        dev, B = m.device, self.B
        T, H, Z = m.max_steps, m.rnn_units, m.vae_latent_dimensions
        e = lambda *s: torch.empty(s, device=dev, dtype=torch.float32)  # noqa: E731
        self.dreg = e(T, 4, B)
        self.douts = e(T, B, D_N)
        self.dpre = e(8, T, B, 64)
        self.dhg = e(T, B, H)
        self.dcg = e(2, B, H)
        self.dGg = e(T, B, 4 * H)
        self.dGgsum = e(B, 4 * H)
        self.dU, self.dUg = e(B, LU), e(B, LU)
        self.dz_carry, self.dss_carry = e(B, Z), e(B, 3)


class AIRModel(_AirBase):
    """See module docstring.  Extra keyword-only arguments as the AIR model
    (device, seed, noise_seed, grad_world, precision, fused_step)."""

    NOISE_ON_SIDE = False  # _forward below uses the noise from its first launch

    _SCOPE_PREFIX = ROOT

    def __init__(self, input_images=None, target_num_digits=None, max_steps=3, max_digits=2,
                 rnn_units=256, canvas_size=50, windows_size=28, vae_latent_dimensions=50,
                 vae_recognition_units=(512, 256), vae_generative_units=(256, 512),
                 fix_scale_distribution=True, vae_prior_mean=0.0, vae_prior_variance=1.0,
                 vae_likelihood_std=0.3, scale_hidden_units=64, shift_hidden_units=64,
                 z_pres_hidden_units=64, z_pres_prior_log_odds=-2.0, z_pres_temperature=1.0,
                 stopping_threshold=0.99, learning_rate=1e-3, gradient_clipping_norm=100.0,
                 cnn=True, cnn_filters=8, num_summary_images=60, train=False, reuse=False,
                 scope="air", annealing_schedules=None, generation_batch_size=64,
                 reuse_shift_scale_network=True, constrains_x_y=None, constrains_num=None,
                 constrains_num_gamma=0.0, constrains_bbox_gamma=0.0, constrains_margin_gamma=0.0,
                 constrains_num_element_gamma=0.0, constrains_sharesize_gamma=0.0,
                 constrains_area_gamma=0.0, constrains_area_minmax=(0.0, 0.0), fix_steps=None, *,
                 device=None, seed: int = 1235, noise_seed: int = 1235, grad_world: int = 1,
                 precision: str = "fp32", fused_step: bool = True):
        if cnn:
            raise NotImplementedError("cnn=True is outside the hot-path scope (train_air_pr.py "
                                      "uses cnn=False)")
        if not fix_scale_distribution:
            raise NotImplementedError("fix_scale_distribution=False (learned scale prior) is not "
                                      "used by train_air_pr.py")
        if not (scale_hidden_units == shift_hidden_units == z_pres_hidden_units == 64):
            raise NotImplementedError("the ASR heads are compiled for 64 hidden units")
        if rnn_units + vae_latent_dimensions + 3 > LU:
            raise NotImplementedError("rnn_units + latent + 3 must fit the packed input row")
        if max_steps > 8:
            raise NotImplementedError("at most 8 loop steps (regulariser kernels)")
        cons = list(constrains_num) if constrains_num is not None else [max_steps]
        if not 1 <= len(cons) <= 8:
            raise ValueError("1..8 allowed object counts")
        if precision not in ("fp32", "bf16"):
            raise ValueError("precision must be 'fp32' or 'bf16'")
        self.precision = precision
        self.fused_step = bool(fused_step) and precision == "bf16" and (
            windows_size == 28 and tuple(vae_recognition_units) == (512, 256)
            and vae_latent_dimensions == 50 and tuple(vae_generative_units) == (256, 512))
        # fp32: the fused fp32 step kernel per loop step (AIRModel._vae_forward_all)
        self.fused_f32 = bool(fused_step) and precision == "fp32" and (
            windows_size == 28 and tuple(vae_recognition_units) == (512, 256)
            and vae_latent_dimensions == 50 and tuple(vae_generative_units) == (256, 512))
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        if self.device.type != "cuda":
            raise RuntimeError("AIRModel runs on a HIP device only (no CPU fallback)")
        _lib.load_torch_ops()
        self.input_images, self.target_num_digits = input_images, target_num_digits
        self.max_steps, self.max_digits = int(max_steps), max_digits
        self.rnn_units = int(rnn_units)
        self.canvas_size, self.windows_size = int(canvas_size), int(windows_size)
        self.C2, self.W2 = self.canvas_size ** 2, self.windows_size ** 2
        self.vae_latent_dimensions = int(vae_latent_dimensions)
        self.vae_recognition_units = tuple(vae_recognition_units)
        self.vae_generative_units = tuple(vae_generative_units)
        self.fix_scale_distribution = True
        self.scale_prior_mean, self.scale_prior_variance = -1.0, 0.05  # :70-72
        self.shift_prior_mean, self.shift_prior_variance = 0.0, 1.0    # generation only
        self.vae_prior_mean, self.vae_prior_variance = vae_prior_mean, vae_prior_variance
        self.vae_likelihood_std = vae_likelihood_std
        self.scale_hidden_units = self.shift_hidden_units = self.z_pres_hidden_units = 64
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
        self.fix_steps = fix_steps
        self.constrains_num = cons
        self.constrains_num_gamma = constrains_num_gamma
        self.constrains_margin_gamma = constrains_margin_gamma
        self.constrains_num_element_gamma = constrains_num_element_gamma
        self.constrains_bbox_gamma = constrains_bbox_gamma
        self.constrains_sharesize_gamma = constrains_sharesize_gamma
        self.constrains_area_gamma = constrains_area_gamma
        self.constrains_area_minmax = tuple(float(v) for v in constrains_area_minmax)
        self.num_prior = None
        self.marginal = None
        self.noise_seed = int(noise_seed)
        self.grad_world = int(grad_world)
        self._noise_ctr = 0
        self.scale_prior_log_variance = _f32log(self.scale_prior_variance)
        self.shift_prior_log_variance = _f32log(self.shift_prior_variance)
        self.vae_prior_log_variance = _f32log(vae_prior_variance)
        specs = asr_param_specs(self.C2, self.rnn_units, self.W2, self.vae_recognition_units,
                                self.vae_generative_units, self.vae_latent_dimensions, 64, 64)
        key = "asr:" + scope
        if reuse:
            if key not in _SCOPES:
                raise ValueError(f"reuse=True but scope {scope!r} has no variables yet")
            self.params = _SCOPES[key]
            if self.params.specs != specs:
                raise ValueError("reused scope has different variable shapes")
        else:
            # the LSTM GEMMs run over LU = 312 packed rows (16-byte operand
            # rows): 3 zero rows behind each LSTM kernel are the rows past its
            # Z + 3 + H, so no launch reads or accumulates into a neighbour
            kpad = (LU - (self.vae_latent_dimensions + 3 + self.rnn_units)) * 4 * self.rnn_units
            self.params = ParamStore(specs, self.device, seed=seed,
                                     pad={ROOT + "infer_rnn_running/kernel": kpad,
                                          ROOT + "gen_rnn_running/kernel": kpad})
            _SCOPES[key] = self.params
        self._ws = None
        self._last_T = None
        self._outputs_ready = False
        self._cons = [int(c) for c in cons]

    # zsum_hook / live_hook: data-parallel collectives (parallel.attach)
    zsum_hook = None

    def _workspace(self, B):
        if self._ws is None or self._ws.B != B:
            self._ws = _AsrWorkspace(self, B)
        return self._ws

    def _N(self, name):
        return self.params.view(ROOT + name)

    def _Kpad(self, name, buf="flat"):
        """An LSTM kernel with its zero pad rows: [rows + pad, 4H] (the GEMMs
        over LU packed rows read / accumulate rows up to C2 + LU)."""
        key = ("kpad", buf, name)
        hit = self.params._views.get(key)
        t = getattr(self.params, buf)
        if hit is not None and hit[0] is t:
            return hit[1]
        o = self.params.offsets[ROOT + name]
        rows, cols = self.params.shapes[ROOT + name]
        pad_rows = LU - (self.vae_latent_dimensions + 3 + self.rnn_units)
        v = t[o:o + (rows + pad_rows) * cols].view(rows + pad_rows, cols)
        self.params._views[key] = (t, v)
        return v

    def _Ng(self, name):
        return self.params.g(ROOT + name)

    _OUT_W = ("inf_shift/dense_1", "inf_shift/dense_3", "inf_scale/dense", "inf_scale/dense_1",
              "inf_scale/dense_2", "inf_scale/dense_3", "gen_shift/dense_1", "gen_shift/dense_3",
              "z_pres/prior/dense_1", "z_pres/log_odds/dense_1")

    def _w20(self):
        ts = []
        for n in self._OUT_W:
            ts += [self._N(n + "/kernel"), self._N(n + "/bias")]
        return ts

    def _gammas(self):
        return [float(v) for v in (
            self.hyper("constrains_num_gamma"), self.hyper("constrains_margin_gamma"),
            self.hyper("constrains_num_element_gamma"), self.hyper("constrains_bbox_gamma"),
            self.hyper("constrains_sharesize_gamma"), self.hyper("constrains_area_gamma"),
            self.constrains_area_minmax[0], self.constrains_area_minmax[1])]

    def _fill_noise(self, ws, noise):
        """eps_shift [T,B,2], eps_scale [T,B], eps_z, eps_x, u (injected or
        device Philox; the fused kernel generates eps_x itself)."""
        if noise is not None:
            for k in ("eps_shift", "eps_scale", "eps_z", "eps_x", "u"):
                dst = ws.eps_scale if k == "eps_scale" else getattr(ws, k)
                src = torch.as_tensor(noise[k], dtype=torch.float32)
                if tuple(src.shape) != tuple(dst.shape):
                    raise ValueError(f"noise[{k}] has shape {tuple(src.shape)}, expected "
                                     f"{tuple(dst.shape)}")
                dst.copy_(src)
            ws.eps_x_offset = None
            return
        super()._fill_noise(ws, None)

    # ---------------------------------------------------------- forward ---
    def _f32_parts(self, B: int) -> bool:
        """fp32 with B >= FUSED_F32_MIN_ROWS: each step's VAE is the fused fp32
        step kernel over that step's rows (AIRModel._vae_forward_all), writing
        the step's canvas part (summed in step order by the loss kernel: the
        running canvas bit for bit).  Smaller batches keep the per-step
        launches (the fused kernel would leave most CUs idle, and the extra
        host work of the parts path shows at the reference's batch of 64)."""
        return self.precision == "fp32" and self.fused_f32 and B >= self.FUSED_F32_MIN_ROWS

    def _parts_layout(self, B: int) -> bool:
        return self.fused_step or self._f32_parts(B)

    def _eps_x_in_kernel(self, B: int) -> bool:
        return self.fused_step or self._f32_parts(B)

    def _batched_vae(self, B: int) -> bool:
        return False  # per step: the ASR loop feeds z of step t into step t+1's input

    def _x3_asr(self, B: int) -> bool:
        """fp32: the inference LSTM's x-rows weight gradient X^T dGsum on the
        three-piece bf16-core form (X_GRAD_X3 = 2, the default, as for AIR)
        from the batch where the side stream pays (SIDE_MIN_BATCH)."""
        return self.precision == "fp32" and self.X_GRAD_X3 == 2 and B >= self.SIDE_MIN_BATCH

    def _forward(self, X, targets, ws, need_grad, outputs=True):
        B, T, H, Z = ws.B, self.max_steps, self.rnn_units, self.vae_latent_dimensions
        C, W, C2 = self.canvas_size, self.windows_size, self.C2
        Ki = self._Kpad("infer_rnn_running/kernel")
        Kg = self._Kpad("gen_rnn_running/kernel")
        bi, bg = self._N("infer_rnn_running/bias"), self._N("gen_rnn_running/bias")
        self._reset_loop_state(ws)
        thr = self.hyper("stopping_threshold")
        temp = self.hyper("z_pres_temperature")
        lik_std = float(self.hyper("vae_likelihood_std"))
        fix = -1 if self.fix_steps is None else int(self.fix_steps)
        w20 = self._w20()
        x3 = need_grad and self._x3_asr(B)
        if x3:
            # the x-rows gradient's A operand split into three bf16 pieces on
            # the side stream, under the x-projection (AIRModel._forward does
            # the same); joined in _weight_grads
            side = self._fork(self._side_stream())
            with torch.cuda.stream(side):
                C2p = self._pad8(C2)
                if getattr(ws, "X3", None) is None:
                    ws.X3 = torch.empty((3, B, C2p), device=self.device, dtype=torch.bfloat16)
                ops.split3_bf16(X, ws.X3, B, C2, C2, C2p, B * C2p)
                ws.x3_ready = torch.cuda.Event()
                ws.x3_ready.record(side)
        elif need_grad and self.precision == "bf16" and B >= self.SIDE_MIN_BATCH:
            # bf16: X converted once for the x-rows gradient, likewise
            with torch.cuda.stream(self._fork(self._side_stream())):
                self._x_bf16(X, ws)
                ws.xb_ready = torch.cuda.Event()
                ws.xb_ready.record(torch.cuda.current_stream())
        # loop-invariant x-projection of the inference LSTM (chain over x first)
        with self._timed("lstm_x_projection"):
            gemm([X], [Ki[:C2]], [ws.Gx], B, 4 * H, C2, C2, 4 * H, 4 * H)
        relu_w = [self._N(n + "/kernel") for n in ("inf_shift/dense", "inf_shift/dense_2",
                                                   "z_pres/log_odds/dense")]
        relu_b = [self._N(n + "/bias") for n in ("inf_shift/dense", "inf_shift/dense_2",
                                                 "z_pres/log_odds/dense")]
        gen_w = [self._N(n + "/kernel") for n in ("gen_shift/dense", "gen_shift/dense_2")]
        gen_b = [self._N(n + "/bias") for n in ("gen_shift/dense", "gen_shift/dense_2")]
        sc_w = [self._N("inf_scale/dense/kernel")[:H], self._N("inf_scale/dense_2/kernel")[:H]]
        for t in range(T):
            prev = t > 0
            # both cells' input rows in one launch
            _ops.asr_pack_(B, Z, H, LU, ws.z[t - 1] if prev else None,
                           ws.ss[t - 1] if prev else None, ws.h[t - 1] if prev else None, ws.U[t],
                           ws.hg[t - 1] if prev else None, ws.Ug[t])
            # K = LU: the packed rows end in zeros, so the chain's last terms are
            # 0 * w (exactly +-0: the sum is unchanged bit for bit) and the
            # operands are 16-byte rows (LDS-DMA GEMM); the 3 weight rows past
            # the U-part are the kernels' own zero pad rows (ParamStore pad)
            # (both LSTMCells' gate GEMMs in one batched launch; the inference
            # cell continues the hoisted x-projection's chain through Cin)
            gemm([ws.U[t], ws.Ug[t]], [Ki[C2:], Kg], [ws.G[t], ws.Gg[t]], B, 4 * H, LU, LU,
                 4 * H, 4 * H, bias=[bi, bg], Cin=[ws.Gx, None])
            # (both cells' gates in one launch)
            _ops.lstm_cell_forward2_(ws.G[t], ws.c[t - 1] if prev else None, ws.c[t], ws.h[t],
                                     ws.Gg[t], ws.cg[t - 1] if prev else None, ws.cg[t],
                                     ws.hg[t], B, H)
            hid = [ws.hid8[k, t] for k in range(8)]
            # (the inference and generative ReLU heads in one batched launch, with
            # the learned prior from the previous generative output (:596-602):
            # hg_{t-1}, the rows asr_pack_ copied into Ug[t])
            ra, rw = [ws.h[t]] * 3 + [ws.hg[t]] * 2, list(relu_w) + list(gen_w)
            rb = list(relu_b) + list(gen_b)
            if fix < 0:
                ra.append(ws.hg[t - 1] if prev else ws.hg_zero)
                rw.append(self._N("z_pres/prior/dense/kernel"))
                rb.append(self._N("z_pres/prior/dense/bias"))
            gemm(ra, rw, hid[0:len(ra)], B, 64, H, H, 64, 64, epi=EPI_RELU, bias=rb)
            gemm([ws.h[t]] * 2, sc_w, hid[6:8], B, 64, H, H, 64, 64, epi=EPI_STORE)
            hid_l = [x if (k != 5 or fix < 0) else None for k, x in enumerate(hid)]
            _ops.asr_step_forward_(B, t, self.train, fix, thr, temp, float(self.scale_prior_mean),
                                   float(self.scale_prior_variance), self.scale_prior_log_variance,
                                   float(self.hyper("constrains_num_gamma")), w20, hid_l,
                                   ws.eps_shift[t], ws.eps_scale[t], ws.u[t], ws.stop, ws.digits,
                                   ws.live, ws.arec[t], ws.th_f[t], ws.th_b[t], ws.ss[t],
                                   ws.scale[t], ws.shift[t], ws.zprob[t], ws.zmask[t], ws.zval[t],
                                   ws.zc[t])
            if self.live_hook is not None:
                self.live_hook(ws.live, t)
            if self.fused_step:
                self._step_fused(X, ws, t, lik_std)
                continue
            if self._f32_parts(B):
                self._vae_forward_all(X, ws, lik_std, t, t + 1, save=need_grad)
                continue
            if self.precision == "bf16":
                self._vae_forward_bf16(X, ws, t, lik_std)
            elif self.DEFER_DECODER:
                # only z feeds the recurrence: the generative half waits
                self._vae_encoder_fp32(X, ws, t)
                continue
            else:
                self._vae_forward_fp32(X, ws, t, lik_std)
            ops.stn_forward(ws.r[t], ws.th_b[t], (C, C), out=ws.canvas, z=ws.zval[t],
                            mask=ws.zmask[t], accumulate=True)
        if (self.precision == "fp32" and self.DEFER_DECODER and not self.fused_step
                and not self._f32_parts(B)):
            # the decoder of every step over T*B rows in one set of launches,
            # then the canvas accumulated in step order (the same bits)
            self._vae_decoder_fp32(ws, lik_std, 0, T)
            for t in range(T):
                ops.stn_forward(ws.r[t], ws.th_b[t], (C, C), out=ws.canvas, z=ws.zval[t],
                                mask=ws.zmask[t], accumulate=True)
        self._forward_loss(X, targets, ws, need_grad, outputs)

    # fp32 below FUSED_F32_MIN_ROWS: the generative half of each step's VAE
    # (which feeds only the canvas, never the loop) after the loop, over T*B
    # rows (DEFER_DECODER = False: inside the loop, step by step)
    DEFER_DECODER = True

    def _forward_loss(self, X, targets, ws, need_grad, outputs=True):
        """elbo (:917-935, recon :937-962) + pr_loss + element + margin
        (:964-1079)."""
        B, T, C2 = ws.B, self.max_steps, self.C2
        g = self._gammas()
        _ops.asr_terms_(B, T, self.canvas_size, self._cons, g, ws.arec, ws.vkl, ws.zmask, ws.live,
                        ws.klsum, ws.pr, ws.area, ws.outl, ws.size, ws.over, ws.zsum)
        if self.zsum_hook is not None:
            self.zsum_hook(ws.zsum)
        parts = ws.cparts
        self._loss_inputs = (X, targets)
        ws.materialized = bool(outputs)
        gscale = self._gscale(B)
        _ops.recon_loss_(X, ws.canvas if (outputs or parts is None) else None, parts,
                         T if parts is not None else 0, B * C2, ws.prows, self.canvas_size,
                         ws.klsum, ws.digits, targets, B, C2, float(gscale),
                         ws.recon if outputs else None, ws.bce, ws.mse, ws.loss_b,
                         ws.acc_b if targets is not None else None,
                         ws.dcanvas if need_grad else None)
        _ops.asr_finalize_(B, T, self.canvas_size, self._cons, g, float(self._gscale(B)), ws.arec,
                           ws.live, ws.zsum, ws.pr, ws.loss_b, ws.element, ws.margin)
        _ops.batch_mean_(ws.loss_b, ws.acc_b if targets is not None else None, ws.mse, None, B,
                         ws.means)
        _ops.add_(ws.means, ws.margin, ws.means, 1)
        self._outputs_ready = True

    # --------------------------------------------------------- backward ---
    def _dz_hook(self, ws, t, dz):
        # (with the batched decoder half, asr_unpack_ added the carry already)
        if t < self.max_steps - 1 and not getattr(ws, "dec_ready", False):
            _ops.add_(dz, ws.dz_carry, dz, ws.B * self.vae_latent_dimensions)

    def _backward(self, X, ws):
        # small batch, one GPU: the fp32-chain weight gradients as grouped
        # launches at the end (as AIRModel._backward)
        self._wgroup = (self._wgroup_obj if (self.WGRAD_GROUP and ws.B < self.SIDE_MIN_BATCH
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
            ws.dm_ready = ws.dec_ready = False
        if wg is not None and wg.probs:
            flops = sum(2.0 * p[4] * p[5] * p[6] for p in wg.probs)
            with self._timed("wgrad_group", ("mfma", flops, "fp32")):
                wg.launch()

    def _backward_body(self, X, ws):
        B, T, H, Z = ws.B, self.max_steps, self.rnn_units, self.vae_latent_dimensions
        C, W, C2 = self.canvas_size, self.windows_size, self.C2
        # the gradient buffer and the LSTM chains' accumulators in one launch
        _ops.fill32_batch_([self.params.grad, ws.dh, ws.dhg, ws.dGsum, ws.dGgsum], [0] * 5)
        Ki = self._Kpad("infer_rnn_running/kernel")
        Kg = self._Kpad("gen_rnn_running/kernel")
        KU = Z + 3 + H
        gscale = self._gscale(B)
        fix = -1 if self.fix_steps is None else int(self.fix_steps)
        w20 = self._w20()
        _ops.asr_terms_backward_(B, T, self.canvas_size, self._cons, self._gammas(), float(gscale),
                                 float(gscale), ws.arec, ws.live, ws.zsum, ws.dreg)
        head_w = [self._N(n + "/kernel")[:H] for n in ("inf_shift/dense", "inf_shift/dense_2",
                                                     "z_pres/log_odds/dense", "inf_scale/dense",
                                                     "inf_scale/dense_2")]
        gen_w = [self._N(n + "/kernel") for n in ("gen_shift/dense", "gen_shift/dense_2")]
        steps_side = (self.VAE_WGRAD_PER_STEP and self.grad_reducer is None
                      and B >= self.SIDE_MIN_BATCH)
        side = self._side_stream() if steps_side else None
        ws.vae_wgrads_done = steps_side
        ws.u_wgrads_done = steps_side and self.U_WGRAD_PER_STEP
        # every step's STN write backward in ONE launch over T*B rows, before
        # the loop (it reads only the forward's records and the canvas
        # gradient, shared by the steps; AIRModel._backward does the same),
        # the glimpse gradient taken through the output sigmoid (dm, bit-identical
        # to dU + mog_sigmoid_backward): six launches of B rows -> one
        TB = T * B
        if self.precision == "bf16":
            ops.stn_backward(ws.r.view(TB, -1), ws.th_b, (C, C), ws.dcanvas, gscale=ws.zc,
                             dtheta=ws.dth_b_all, dot=ws.dot_all, want_dot=True, n=TB,
                             dm_bf16=ws.dmb.view(TB, -1))
        else:
            ops.stn_backward(ws.r.view(TB, -1), ws.th_b, (C, C), ws.dcanvas, gscale=ws.zc,
                             dtheta=ws.dth_b_all, dot=ws.dot_all, want_dot=True, n=TB,
                             dm=ws.dm.view(TB, -1))
        ws.dm_ready = True
        # and the decoder half of every step's VAE backward (dz_t before the
        # loop's carry), likewise over T*B rows
        self._vae_decoder_backward_all(ws)
        # a small batch's recurrent-input gradient in DH_PARTS K slices
        # (AIRModel.DH_PARTS: the serial K = 4H chain per workgroup cut)
        parts = self.DH_PARTS if (B < self.SIDE_MIN_BATCH and self.DH_PARTS > 1
                                  and (4 * H) % (4 * self.DH_PARTS) == 0) else 0
        if parts and getattr(ws, "dUp", None) is None:
            ws.dUp = torch.empty((parts,) + tuple(ws.dU.shape), device=self.device)
            ws.dUgp = torch.empty((parts,) + tuple(ws.dUg.shape), device=self.device)
        for t in reversed(range(T)):
            if self.precision == "bf16":
                self._vae_backward_bf16(ws, t, gscale)
            else:
                self._vae_backward_fp32(ws, t, gscale)
            if steps_side:
                # step t's VAE weight gradients are final: accumulate them on
                # the side stream under the rest of the loop
                with torch.cuda.stream(self._fork(side)):
                    if self.precision == "bf16":
                        self._vae_weight_grads_bf16(ws, t)
                    else:
                        self._vae_weight_grads_fp32(ws, t)
            ops.stn_backward(X, ws.th_f[t], (W, W), ws.dg, want_dU=False, dtheta=ws.dth_f)
            hid = [ws.hid8[k, t] for k in range(8)]
            dpre = [ws.dpre[k, t] for k in range(8)]
            _ops.asr_step_backward_(B, self.train, fix, float(self.hyper("z_pres_temperature")),
                                    float(self.scale_prior_mean),
                                    float(self.scale_prior_variance), float(gscale), w20,
                                    [x if (k != 5 or fix < 0) else None for k, x in enumerate(hid)],
                                    ws.arec[t], ws.eps_shift[t], ws.eps_scale[t], ws.dth_f,
                                    ws.dth_b_all[t], ws.dot_all[t], ws.dreg[t],
                                    ws.dss_carry if t < T - 1 else None, ws.douts[t],
                                    [x if (k != 5 or fix < 0) else None
                                     for k, x in enumerate(dpre)])
            # dh[t] += the five heads reading h_t; dhg[t] += the generative shift
            # heads; dhg[t-1] += the prior at step t (it reads hg_{t-1}): three
            # chains of one shape in one launch
            probs = [([dpre[k] for k in (0, 1, 2, 6, 7)], head_w, ws.dh[t], ws.dh[t]),
                     ([dpre[3], dpre[4]], gen_w, ws.dhg[t], ws.dhg[t])]
            if fix < 0 and t > 0:
                probs.append(([dpre[5]], [self._N("z_pres/prior/dense/kernel")], ws.dhg[t - 1],
                              ws.dhg[t - 1]))
            ops.gemm_kseg_group(probs, B, H, 64, 64, 64, H, transB=True)
            dc_in = ws.dc[(t + 1) % 2] if t < T - 1 else None
            dcg_in = ws.dcg[(t + 1) % 2] if t < T - 1 else None
            # (both cells in one launch)
            _ops.lstm_cell_backward2_(ws.G[t], ws.c[t - 1] if t > 0 else None, ws.c[t], ws.dh[t],
                                      dc_in, ws.dG[t], ws.dc[t % 2], ws.dGsum, ws.Gg[t],
                                      ws.cg[t - 1] if t > 0 else None, ws.cg[t], ws.dhg[t],
                                      dcg_in, ws.dGg[t], ws.dcg[t % 2], ws.dGgsum, B, H)
            if steps_side and self.U_WGRAD_PER_STEP:
                # step t's recurrent-rows gradients likewise (dG_t, dGg_t final)
                with torch.cuda.stream(self._fork(side)):
                    self._u_rows_wgrad(ws, t)
            if t > 0 and parts:
                # a small batch: the same product in `parts` K slices (one batched
                # launch of 2 x parts), summed in part order by the unpack
                kp = 4 * H // parts
                gemm([ws.dG[t][:, j * kp:] for j in range(parts)]
                     + [ws.dGg[t][:, j * kp:] for j in range(parts)],
                     [Ki[C2:][:, j * kp:] for j in range(parts)]
                     + [Kg[:, j * kp:] for j in range(parts)],
                     [ws.dUp[j] for j in range(parts)] + [ws.dUgp[j] for j in range(parts)],
                     B, LU, kp, 4 * H, 4 * H, LU, transB=True)
                _ops.asr_unpack_parts_(B, Z, H, LU, ws.dUp, ws.dUgp, parts, ws.dz_all[t - 1],
                                       ws.dss_carry, ws.dh[t - 1], ws.dhg[t - 1], 1)
            elif t > 0:
                # N = LU: the 3 pad columns of dU / dUg are scratch (unpack skips them)
                # (both LSTMCells in one batched launch: same shapes and chains)
                gemm([ws.dG[t], ws.dGg[t]], [Ki[C2:], Kg], [ws.dU, ws.dUg], B, LU, 4 * H,
                     4 * H, 4 * H, LU, transB=True)
                # the latent carry added straight into step t-1's dz (its decoder
                # half is there already: no separate add launch)
                _ops.asr_unpack_(B, Z, H, LU, ws.dU, ws.dUg, ws.dz_all[t - 1], ws.dss_carry,
                                 ws.dh[t - 1], ws.dhg[t - 1], 1)
        ws.dm_ready = ws.dec_ready = False
        self._weight_grads(X, ws)
        if steps_side:
            torch.cuda.current_stream().wait_stream(side)
        self._reduce_bucket(0, self.params.total)

    def _u_rows_wgrad(self, ws, t):
        """The LSTMCells' recurrent-rows kernel gradients U^T dG (all T*B rows,
        or loop step t's B rows, accumulated)."""
        B, T, H = ws.B, self.max_steps, self.rnn_units
        K = B if t is not None else B * T
        v = (lambda x: x[t]) if t is not None else (lambda x: x)  # noqa: E731
        gKi = self._Kpad("infer_rnn_running/kernel", "grad")
        gKg = self._Kpad("gen_rnn_running/kernel", "grad")
        if self.REC_WGRAD_X3 and K >= self.WGRAD_TN_MIN_ROWS:
            # both cells in one grouped x3 launch (as AIR's recurrent rows,
            # AIRModel._dw_rec): 312 x 1024 x K each, deterministic
            with self._timed("rec_wgrad_x3", ("mfma", 2 * 2.0 * K * LU * 4 * H, "fp32", "x3")):
                ops.wgrad_tn_x3([v(ws.U), v(ws.Ug)], [v(ws.dG), v(ws.dGg)],
                                [gKi[self.C2:], gKg], [None, self._Ng("gen_rnn_running/bias")],
                                [(LU, 4 * H, LU, 4 * H, 4 * H)] * 2, K, self.WGRAD_TN_X3_SPLITS)
            return
        self._dw(v(ws.U), v(ws.dG), gKi[self.C2:], K, LU, 4 * H, LU, 4 * H)
        self._dw(v(ws.Ug), v(ws.dGg), gKg, K, LU, 4 * H, LU, 4 * H,
                 self._Ng("gen_rnn_running/bias"))

    # (with VAE_WGRAD_PER_STEP) the recurrent-rows gradients per step too (9.20 ->
    # 8.96 ms; the heads' gradients per step as well measured neutral, 9.01 vs
    # 9.26 ms for neither on a slower box, and stay after the loop)
    U_WGRAD_PER_STEP = True

    # one GPU, from SIDE_MIN_BATCH: the VAE weight gradients of loop step
    # t accumulate on the side stream as soon as that step's VAE backward is
    # done, under the latency-bound rest of the reversed loop, instead of over
    # all T*B rows after it (VAE_WGRAD_PER_STEP = False: after the loop)
    VAE_WGRAD_PER_STEP = True

    def _weight_grads(self, X, ws):
        B, T, H, Z = ws.B, self.max_steps, self.rnn_units, self.vae_latent_dimensions
        C2, TB, KU = self.C2, ws.B * self.max_steps, Z + 3 + H
        fix = -1 if self.fix_steps is None else int(self.fix_steps)
        heads_s3 = getattr(ws, "vae_wgrads_done", False) and self.HEADS_S3
        if heads_s3:
            # the heads' weight gradients on the third stream, beside the
            # x-rows gradient (main) and step 0's on the side stream
            with torch.cuda.stream(self._fork(self._stream3())):
                self._heads_wgrad(ws, None)
        if getattr(ws, "vae_wgrads_done", False):
            pass  # (per loop step, on the side stream)
        elif self.precision == "bf16":
            self._vae_weight_grads_bf16(ws)
        else:
            self._vae_weight_grads_fp32(ws)
        ws.vae_wgrads_done = False
        G = self._Ng
        gKi = self._Kpad("infer_rnn_running/kernel", "grad")
        gKg = self._Kpad("gen_rnn_running/kernel", "grad")
        # LSTMCells: x rows from sum_t dG (the x input is loop-invariant)
        if self.precision == "bf16":
            self._x_grad_bf16(X, ws, gKi, G("infer_rnn_running/bias"), 0, C2)
        elif getattr(ws, "x3_ready", None) is not None:
            # X^T dGsum on the bf16 matrix cores from exact three-piece
            # splits of both operands (gemm_x3.hip): the
            # AIR x-rows gradient's form
            torch.cuda.current_stream().wait_event(ws.x3_ready)
            ws.x3_ready = None
            if getattr(ws, "dG3", None) is None:
                ws.dG3 = torch.empty((3, B, 4 * H), device=self.device, dtype=torch.bfloat16)
            ops.split3_bf16(ws.dGsum, ws.dG3, B, 4 * H, 4 * H, 4 * H, B * 4 * H)
            C2p = self._pad8(C2)
            with self._timed("lstm_x_projection_grad", ("mfma", 2.0 * B * C2 * 4 * H, "fp32", "x3")):
                ops.gemm_x3p_tn(ws.X3.view(-1), B * C2p, ws.dG3, B * 4 * H, gKi[:C2], C2, 4 * H,
                                B, C2p, 4 * H, 4 * H,
                                splitk=self._sk(max(1, min(B // 256, self.X3_SPLITK))),
                                colsum=G("infer_rnn_running/bias"))
        else:
            self._dw(X, ws.dGsum, gKi[:C2], B, C2, 4 * H, C2, 4 * H,
                     G("infer_rnn_running/bias"))
        # M = LU (16-byte aligned LDS-DMA operands): rows Z+3+H.. of the
        # product land in the kernels' own pad rows (ParamStore pad), never in
        # a neighbouring variable's gradient
        if not getattr(ws, "u_wgrads_done", False):
            self._u_rows_wgrad(ws, None)
        ws.u_wgrads_done = False
        if heads_s3:
            torch.cuda.current_stream().wait_stream(self._stream3())
        else:
            self._heads_wgrad(ws, None)

    # (with the per-step gradients) the heads' gradients on the third stream
    HEADS_S3 = True

    def _heads_wgrad(self, ws, t):
        """The heads' weight gradients (all T*B rows, or loop step t's B rows,
        accumulated)."""
        B, T, H, Z = ws.B, self.max_steps, self.rnn_units, self.vae_latent_dimensions
        K = B if t is not None else B * T
        v = (lambda x: x[t]) if t is not None else (lambda x: x)  # noqa: E731
        G = self._Ng
        fix = -1 if self.fix_steps is None else int(self.fix_steps)
        # hidden layers reading h_t, hg_t, hg_{t-1}
        hs = ("inf_shift/dense", "inf_shift/dense_2", "z_pres/log_odds/dense", "inf_scale/dense",
              "inf_scale/dense_2")
        self._dw([v(ws.h)] * 5, [v(ws.dpre[k]) for k in (0, 1, 2, 6, 7)],
                 [G(n + "/kernel")[:H] for n in hs], K, H, 64, H, 64,
                 [G(n + "/bias") for n in hs])
        self._dw([v(ws.hg)] * 2, [v(ws.dpre[3]), v(ws.dpre[4])],
                 [G("gen_shift/dense/kernel"), G("gen_shift/dense_2/kernel")], K, H, 64, H, 64,
                 [G("gen_shift/dense/bias"), G("gen_shift/dense_2/bias")])
        if fix < 0:
            self._dw(v(ws.Ug)[..., Z + 3:], v(ws.dpre[5]), G("z_pres/prior/dense/kernel"), K, H, 64,
                     LU, 64, G("z_pres/prior/dense/bias"))
        # the shift-latent rows of the scale hidden layers
        self._dw([v(ws.ss)] * 2, [v(ws.dpre[6]), v(ws.dpre[7])],
                 [G("inf_scale/dense/kernel")[H:], G("inf_scale/dense_2/kernel")[H:]], K, 2, 64,
                 3, 64)
        # output layers from douts [T, B, 12]
        d = v(ws.douts)
        outs = (("inf_shift/dense_1", 0, 0, 2), ("inf_shift/dense_3", 1, 2, 2),
                ("z_pres/log_odds/dense_1", 2, 4, 1), ("gen_shift/dense_1", 3, 5, 2),
                ("gen_shift/dense_3", 4, 7, 2))
        # grouped by shape, one batched launch per group (each is a tiny
        # [64 x 1..2] product over K = T*B rows: launch-bound one by one)
        one = [(v(ws.hid8[hk]), d[..., col:], G(n + "/kernel"), G(n + "/bias"))
               for n, hk, col, k in outs if k == 1]
        two = [(v(ws.hid8[hk]), d[..., col:], G(n + "/kernel"), G(n + "/bias"))
               for n, hk, col, k in outs if k == 2]
        if fix < 0:
            one.append((v(ws.hid8[5]), d[..., 9:], G("z_pres/prior/dense_1/kernel"),
                        G("z_pres/prior/dense_1/bias")))
        scl = (("inf_scale/dense_1", 6, 10), ("inf_scale/dense_3", 7, 11))
        one += [(v(ws.hid8[hk]), d[..., col:], G(n + "/kernel")[:64], G(n + "/bias"))
                for n, hk, col in scl]
        for grp, k in ((two, 2), (one, 1)):
            self._dw([g[0] for g in grp], [g[1] for g in grp], [g[2] for g in grp], K, 64, k,
                     64, D_N, [g[3] for g in grp])
        self._dw([v(ws.ss)] * 2, [d[..., col:] for _, _, col in scl],
                 [G(n + "/kernel")[64:] for n, _, _ in scl], K, 2, 1, 3, D_N)

    # ------------------------------------------------------- outputs -----
    @property
    def rec_scales(self):
        return self._bt(self._ws.scale).unsqueeze(-1)

    @property
    def z_pres_probs(self):
        return self._bt(self._ws.zprob)

    def _records(self, name):
        return self._bt(self._ws.arec[:, Q[name]])

    @property
    def z_pres_kls(self):
        return self._records("zkl")

    @property
    def scale_kls(self):
        return self._records("skl")

    @property
    def shift_kls(self):
        return self._records("shkl")

    @property
    def vae_kls(self):
        ws = self._ws
        return self._bt(ws.vkl * ws.zmask)

    @property
    def log_variables(self) -> Dict[str, float]:
        """Batch means of the reference's log_variables (:1080-1084)."""
        ws = self._ws
        T = self._T()
        m = lambda v: float(v.mean())  # noqa: E731
        kls = {k: float(self._records(k).sum(1).mean()) for k in ("zkl", "skl", "shkl")}
        return {"z_pres_kl": kls["zkl"], "scale_kl": kls["skl"], "shift_kl": kls["shkl"],
                "vae_kl": float((ws.vkl * ws.zmask)[:T].sum(0).mean()),
                "pr_num": float(self._records("prn").sum(1).mean()),
                "recon": m(ws.bce), "mse": m(ws.mse), "area_loss": m(ws.area),
                "out_loss": m(ws.outl), "size_loss": m(ws.size), "over_loss": m(ws.over),
                "num_margin": float(ws.margin[0]), "num_min_KL": m(ws.element),
                "TotLoss": self.loss, "elbo": m(ws.klsum + ws.bce), "accu": self.accuracy}

    def generate(self, *a, **k):
        raise NotImplementedError("ASR generation (air_number_bbox_location.py:1124-1361) runs "
                                  "the generative LSTM prior; not part of this build")
