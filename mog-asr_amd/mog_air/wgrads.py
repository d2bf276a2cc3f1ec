"""Weight gradients of the AIR train step (the TF MatMul / BiasAdd gradients
of air/vae.py:18-46, the heads of air/air_model.py:458-520 and the LSTM
kernel of :454-456): which GEMM form each runs on, how far it splits K, and
on which stream (AIRModel mixes this in; it reads the model's workspace and
parameters).

Forms: the fp32 chain split-K GEMM (gemm_f32.hip, float atomics), the
grouped one-launch form of a small batch (gemm_group.hip), fp32 operands on
the bf16 matrix cores with exact three-piece splits (gemm_x3.hip: in-kernel
or pre-split) and the bf16 configuration's bf16 GEMMs
(gemm_bf16.hip).  Streams: from AIRModel.SIDE_MIN_BATCH the VAE's weight
gradients run on the side stream, the heads' and the recurrent rows' on the
third stream.
"""
from __future__ import annotations

import torch

from . import ops
from .ops import EPI_ATOMIC, gemm

_ops = ops._ops


class WeightGradients:
    # every weight gradient in one k pass (split-K 1, one atomic add per
    # element onto the zeroed gradient): a bitwise-reproducible step, for the
    # stream-ordering tests (tests/test_gpu_streams.py)
    ONE_PASS_WGRADS = False

    # workgroups the split-K weight gradients aim for (bf16 sweep of 128-2048:
    # 256 best; fp32 512 / 1024 / 2048: 2048 best)
    DW_BF16_TARGET = 256
    DW_F32_TARGET = 2048

    def _sk(self, splitk):
        return 1 if self.ONE_PASS_WGRADS else splitk

    def _dw_bf16(self, X, dY, out, K, M, N, lda, ldb, bias_out):
        from .ops import BF_ATOMIC, gemm_bf16
        big = M >= 128 and N >= 128
        tiles = ((M + 127) // 128) * ((N + 127) // 128) if big else \
            ((M + 63) // 64) * ((N + 63) // 64)
        target = self.DW_BF16_TARGET
        splitk = self._sk(max(1, min(K // 512, (target + tiles - 1) // tiles)))
        with self._timed("wgrad_bf16", ("mfma", 2.0 * K * M * N, "bf16")):
            gemm_bf16([X], [dY], [out], M, N, K, lda, ldb, N, tn=True, epi=BF_ATOMIC,
                      splitk=splitk, colsum=[bias_out])

    # the grouped tall-K kernel (wgrad_tn.hip: all seven layers in one launch,
    # K split over the XCDs, partials added in order) from this many rows;
    # below it the per-layer split-K GEMMs
    WGRAD_TN_MIN_ROWS = 2048
    WGRAD_TN_SPLITS = 8
    # the x3 form: 16 splits (350 vs 427 us at 8 for the four layers at
    # 24,576 rows, scripts/wgrad_shapes.py)
    WGRAD_TN_X3_SPLITS = 16

    def _vae_weight_grads_bf16(self, ws, t=None):
        """The VAE weight gradients over all T*B rows (bf16 operands), or over
        loop step t's B rows (accumulated: the per-step form of AIR-ASR)."""
        TB = ws.B * self.max_steps if t is None else ws.B
        v = (lambda x: x) if t is None else (lambda x: x[t])  # noqa: E731
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        Zp = self._pad8(Z)
        g = lambda n: self._G("vae/" + n + "/weights")  # noqa: E731
        gb = lambda n: self._G("vae/" + n + "/biases")  # noqa: E731
        # (X, dY, layer, M, N, lda, ldb) of the seven layers
        probs = [(v(ws.gb), v(ws.da1b), "recognition_1", W2, R1, W2, R1),
                 (v(ws.a1b), v(ws.da2b), "recognition_2", R1, R2, R1, R2),
                 (v(ws.a2b), v(ws.dmub), "rec_mean", R2, Z, R2, Zp),
                 (v(ws.a2b), v(ws.dlvb), "rec_log_variance", R2, Z, R2, Zp),
                 (v(ws.zb), v(ws.dd1b), "generative_1", Z, G1, Zp, G1),
                 (v(ws.d1b), v(ws.dd2b), "generative_2", G1, G2, G1, G2),
                 (v(ws.d2b), v(ws.dmb), "gen_mean", G2, W2, G2, W2)]
        if TB >= self.WGRAD_TN_MIN_ROWS:
            flops = sum(2.0 * TB * M * N for _, _, _, M, N, _, _ in probs)
            with self._timed("vae_wgrad_bf16", ("mfma", flops, "bf16")):
                ops.wgrad_tn_bf16([p[0] for p in probs], [p[1] for p in probs],
                                  [g(p[2]) for p in probs], [gb(p[2]) for p in probs],
                                  [(M, N, lda, ldb, N) for _, _, _, M, N, lda, ldb in probs],
                                  TB, self.WGRAD_TN_SPLITS)
            return
        for X, dY, name, M, N, lda, ldb in probs:
            self._dw_bf16(X, dY, g(name), TB, M, N, lda, ldb, gb(name))

    def _dw(self, X, dY, out, K, M, N, lda, ldb, bias_out=None):
        """out[M,N] += X^T dY over K rows (split-K, atomics); bias_out += colsum(dY).
        X, dY, out, bias_out may be lists (one batched launch)."""
        if not isinstance(out, (list, tuple)):
            X, dY, out = [X], [dY], [out]
            bias_out = None if bias_out is None else [bias_out]
        if self._wgroup is not None:  # collected: one grouped launch ends the backward
            for x, dy, o, b in zip(X, dY, out, bias_out or [None] * len(out)):
                self._wgroup.add(x, dy, o, M, N, K, lda, ldb, N, b)
            return
        tiles = ((M + 63) // 64) * ((N + 63) // 64) * len(out)
        target = self.DW_F32_TARGET
        splitk = self._sk(max(1, min(K // 256, (target + tiles - 1) // tiles)))
        with self._timed("wgrad_f32", ("mfma", 2.0 * K * M * N * len(out), "fp32")):
            gemm(X, dY, out, M, N, K, lda, ldb, N, transA=True, epi=EPI_ATOMIC,
                 splitk=splitk, colsum=bias_out)

    # fp32 configuration: the VAE weight gradients whose operands are 16-byte
    # rows (M, N multiples of 4: the 784/512/256-wide layers, 98 % of the
    # flops) on the bf16 matrix cores with exact three-piece splits inside the
    # GEMM (gemm_x3.hip: fp32-level accuracy, as the LSTM x-rows gradient,
    # DESIGN.md §4.4); False keeps them on the fp32 split-K GEMM
    VAE_WGRAD_X3 = True

    # the x3 forms from this many rows: below it (the reference's batch of 64:
    # 192 rows) their 128 x 128 tiles leave most CUs idle, and the fp32 GEMMs'
    # small-M tiles finish first
    X3_MIN_ROWS = 2048
    # the NT input-gradient form from this many rows (the AIR step's T*B =
    # 24,576 and the ASR step's per-step 8,192): below it its 128 x 128 tiles
    # leave CUs idle and the fp32 GEMM finishes first.  (Round 4, after the
    # NT load fixes: ASR fp32 step 9.46 -> 9.43 ms with 8,192 in; before
    # them the NT form lost there, 9.6 -> 10.1 ms.)
    X3_DX_MIN_ROWS = 8192

    def _dw_x3(self, X, dY, out, K, M, N, lda, ldb, bias_out):
        """out[M,N] += X^T dY over K rows (gemm_x3_tn), bias_out += colsum(dY)."""
        if not (self.VAE_WGRAD_X3 and M % 4 == 0 and N % 4 == 0 and K >= self.X3_MIN_ROWS):
            return self._dw(X, dY, out, K, M, N, lda, ldb, bias_out)
        tiles = ((M + 127) // 128) * ((N + 127) // 128)
        splitk = self._sk(max(1, min(K // 256, (512 + tiles - 1) // tiles)))
        # six bf16 MFMA products per fp32 product (gemm_x3.hip); float atomics
        # for the 19-64 split-K partials of these <= 0.4 M-element outputs
        # (through the workspace: 160 -> 229 us per launch in the step)
        with self._timed("vae_wgrad_x3", ("mfma", 2.0 * K * M * N, "fp32", "x3")):
            ops.gemm_x3_tn(X, dY, out, M, N, K, lda, ldb, N, splitk=splitk, colsum=bias_out,
                           reduce=False)

    def _vae_wgrad_fp32(self, ws, name, t=None):
        """One VAE layer's weight / bias gradient over all T*B rows (fp32), or
        over loop step t's B rows (accumulated: the per-step form of AIR-ASR)."""
        TB = ws.B * self.max_steps
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        g = lambda n: self._G("vae/" + n + "/weights")  # noqa: E731
        gb = lambda n: self._G("vae/" + n + "/biases")  # noqa: E731
        if t is None:
            v = lambda x: x  # noqa: E731
        else:
            TB = ws.B
            v = lambda x: x[t]  # noqa: E731
        if name == "recognition_1":
            self._dw_x3(v(ws.g), v(ws.da1), g(name), TB, W2, R1, W2, R1, gb(name))
        elif name == "recognition_2":
            self._dw_x3(v(ws.a1), v(ws.da2), g(name), TB, R1, R2, R1, R2, gb(name))
        elif name == "rec_mean":  # (with rec_log_variance: one batched launch)
            self._dw([v(ws.a2)] * 2, [v(ws.dmu), v(ws.dlv)], [g("rec_mean"),
                     g("rec_log_variance")], TB, R2, Z, R2, Z,
                     [gb("rec_mean"), gb("rec_log_variance")])
        elif name == "generative_1":
            self._dw(v(ws.z), v(ws.dd1), g(name), TB, Z, G1, Z, G1, gb(name))
        elif name == "generative_2":
            self._dw_x3(v(ws.d1), v(ws.dd2), g(name), TB, G1, G2, G1, G2, gb(name))
        elif name == "gen_mean":
            self._dw_x3(v(ws.d2), v(ws.dm), g(name), TB, G2, W2, G2, W2, gb(name))

    def _vae_weight_grads_fp32(self, ws, t=None):
        """The fp32 VAE weight gradients over all T*B rows, or over loop step
        t's B rows (the per-step form of AIR-ASR): from WGRAD_TN_MIN_ROWS the
        seven layers in ONE grouped x3 launch (wgrad_tn.hip: fp32-level
        accuracy, K split over the XCDs, partials added in order --
        deterministic)."""
        TB = ws.B * self.max_steps if t is None else ws.B
        v = (lambda x: x) if t is None else (lambda x: x[t])  # noqa: E731
        W2, R1, R2, Z, G1, G2 = self._vae_dims()
        probs = [(v(ws.g), v(ws.da1), "recognition_1", W2, R1),
                 (v(ws.a1), v(ws.da2), "recognition_2", R1, R2),
                 (v(ws.a2), v(ws.dmu), "rec_mean", R2, Z),
                 (v(ws.a2), v(ws.dlv), "rec_log_variance", R2, Z),
                 (v(ws.z), v(ws.dd1), "generative_1", Z, G1),
                 (v(ws.d1), v(ws.dd2), "generative_2", G1, G2),
                 (v(ws.d2), v(ws.dm), "gen_mean", G2, W2)]
        if (self.VAE_WGRAD_X3 and TB >= self.WGRAD_TN_MIN_ROWS
                and all(M % 2 == 0 and N % 2 == 0 for _, _, _, M, N in probs)):
            g = lambda n: self._G("vae/" + n + "/weights")  # noqa: E731
            gb = lambda n: self._G("vae/" + n + "/biases")  # noqa: E731
            flops = sum(2.0 * TB * M * N for _, _, _, M, N in probs)
            with self._timed("vae_wgrad_x3", ("mfma", flops, "fp32", "x3")):
                ops.wgrad_tn_x3([p[0] for p in probs], [p[1] for p in probs],
                                [g(p[2]) for p in probs], [gb(p[2]) for p in probs],
                                [(M, N, M, N, N) for _, _, _, M, N in probs], TB,
                                self.WGRAD_TN_X3_SPLITS)
            return
        for name in ("recognition_1", "recognition_2", "rec_mean", "generative_1",
                     "generative_2", "gen_mean"):
            self._vae_wgrad_fp32(ws, name, t)

    def _weight_grads_glimpse(self, ws):
        """Weight gradients of the VAE and the five heads (every loop step at
        once, K = T*B rows)."""
        if self.precision == "bf16":
            self._vae_weight_grads_bf16(ws)
        else:
            self._vae_weight_grads_fp32(ws)
        self._weight_grads_heads(ws)

    def _vae_weight_grads_async(self, ws):
        """The VAE weight gradients on the side stream (ordered after
        everything issued so far on the current stream); returns the events
        that mark the heads' W1 refresh and their completion.  Below
        SIDE_MIN_BATCH they run in line on the current stream (events None):
        at the reference's batch of 64 the launches are a few microseconds
        each, too short to hide a cross-stream wait."""
        if ws.B < self.SIDE_MIN_BATCH:
            if self.precision == "bf16":
                self._vae_weight_grads_bf16(ws)
            else:
                self._vae_weight_grads_fp32(ws)
            return None, None
        side = self._fork(self._side_stream())
        with torch.cuda.stream(side):
            # the heads' concatenated W1 (B operand of the dh GEMM) first:
            # off the main stream, which waits for it only at that GEMM
            self._w1cat()
            w1_done = torch.cuda.Event()
            w1_done.record(side)
            if self.precision == "bf16":
                self._vae_weight_grads_bf16(ws)
            else:
                self._vae_weight_grads_fp32(ws)
            done = torch.cuda.Event()
            done.record(side)
        return w1_done, done

    def _w1cat(self):
        """[W1_0 .. W1_4] side by side ([H, 5 HS]): the B operand of the heads'
        dh GEMM, refreshed when the parameters change."""
        if getattr(self, "_w1cat_version", None) != self.params.version:
            if getattr(self, "_w1cat_buf", None) is None:
                H, HS = self.rnn_units, self.scale_hidden_units
                self._w1cat_buf = torch.empty((H, 5 * HS), device=self.device)
            torch.cat([self._P(h + "/hidden/weights") for h in self._HEADS], dim=1,
                      out=self._w1cat_buf)
            self._w1cat_version = self.params.version
        return self._w1cat_buf

    def _weight_grads_heads(self, ws):
        H, HS, TB = self.rnn_units, self.scale_hidden_units, ws.B * self.max_steps
        heads = list(enumerate(self._HEADS))
        dhid = ws.dhid.view(TB, 5, HS)
        g = self._G
        if (self._wgroup is None and TB >= self.WGRAD_TN_MIN_ROWS
                and H % 2 == 0 and HS % 2 == 0 and HS < 128):
            # deterministic from the split-K batch sizes on: the five hidden
            # layers on the grouped x3 kernel (splits added in order), the 1- /
            # 2-column output layers by chunk partials added in chunk order
            # (mog_heads_output_wgrad)
            flops = 2.0 * TB * H * HS * 5
            with self._timed("heads_wgrad_x3", ("mfma", flops, "fp32", "x3")):
                ops.wgrad_tn_x3([ws.h] * 5, [dhid[:, zi] for zi, _ in heads],
                                [g(h + "/hidden/weights") for _, h in heads],
                                [g(h + "/hidden/biases") for _, h in heads],
                                [(H, HS, H, 5 * HS, HS)] * 5, TB, self.WGRAD_TN_X3_SPLITS)
            _ops.heads_output_wgrad_([ws.hid[zi] for zi, _ in heads],
                                     [ws.dout[zi] for zi, _ in heads],
                                     [g(h + "/output/weights") for _, h in heads],
                                     [g(h + "/output/biases") for _, h in heads],
                                     [2 if h.startswith("shift") else 1 for _, h in heads], TB, HS)
            return
        self._dw([ws.h] * 5, [dhid[:, zi] for zi, _ in heads],
                 [g(h + "/hidden/weights") for _, h in heads], TB, H, HS, H, 5 * HS,
                 [g(h + "/hidden/biases") for _, h in heads])
        for k in (1, 2):
            sel = [(zi, h) for zi, h in heads if (2 if h.startswith("shift") else 1) == k]
            self._dw([ws.hid[zi] for zi, _ in sel], [ws.dout[zi] for zi, _ in sel],
                     [g(h + "/output/weights") for _, h in sel], TB, HS, k, HS, 2,
                     [g(h + "/output/biases") for _, h in sel])

    # fp32 configuration: the x-part of the LSTM kernel gradient on the bf16
    # matrix cores with exact three-piece operand splits (gemm_x3.hip,
    # DESIGN.md §4.4).  2 (default): the operands split once per step, X on
    # the side stream under the x-projection, dG before the GEMM (gemm_x3p_tn:
    # 244 vs 428 us stand-alone, step 3.44 -> 3.37 ms); 1: split inside the
    # GEMM (318 us, no change in the step); 0: the fp32 MFMA split-K GEMM.
    X_GRAD_X3 = 2
    # the pre-split form from this batch: below it (the reference's batch of
    # 64) the two split launches cost more than the fp32 chain's K = B pass
    # (batch 64: x3p 12.3 + splits 9.6 us)
    X3P_MIN_B = 256

    def _x3p_xgrad(self, B):
        return self.precision == "fp32" and self.X_GRAD_X3 == 2 and B >= self.X3P_MIN_B
    X3_SPLITK = 8

    # rows of the x-part of the LSTM kernel gradient per all-reduce bucket
    # (multiple of the 64-row GEMM tile; data parallel only)
    X_GRAD_CHUNK = 640

    def _weight_grads_rec_side(self, ws):
        """One GPU: the LSTM kernel's recurrent-rows gradient sum_t h[t-1]^T
        dG[t] on a side stream, forked as soon as dG[1:] is final (before the
        chain's step 0), so it overlaps that step instead of the x-rows
        gradient."""
        # (on the third stream after the heads' weight gradients: 3.06 ->
        # 3.04 ms against the side stream)
        with torch.cuda.stream(self._fork(self._stream3())):
            self._dw_rec(ws)

    def _dw_rec(self, ws):
        """The LSTM kernel's recurrent rows: gK[C2:] += sum_t h[t-1]^T dG[t]
        over (T-1) B rows.  From WGRAD_TN_MIN_ROWS (either precision:
        fp32-level, and faster than the fp32 chain): on the bf16 matrix cores
        with exact three-piece splits (the grouped x3 kernel of the fp32 VAE
        weight gradients, one problem, 256 x 1024 x 16,384 at B = 8192), else
        the fp32 split-K GEMM."""
        B, T, H, C2 = ws.B, self.max_steps, self.rnn_units, self.C2
        gK = self._G("rnn/basic_lstm_cell/kernel")
        K = (T - 1) * B
        if self.REC_WGRAD_X3 and K >= self.WGRAD_TN_MIN_ROWS:
            # the grouped x3 kernel with one problem: deterministic
            with self._timed("rec_wgrad_x3", ("mfma", 2.0 * K * H * 4 * H, "fp32", "x3")):
                ops.wgrad_tn_x3([ws.h], [ws.dG[1:]], [gK[C2:]], [None],
                                [(H, 4 * H, H, 4 * H, 4 * H)], K, self.WGRAD_TN_X3_SPLITS)
        else:
            self._dw(ws.h, ws.dG[1:], gK[C2:], K, H, 4 * H, H, 4 * H)

    REC_WGRAD_X3 = True

    def _weight_grads_lstm(self, X, ws, side=False, rec_done=False):
        """LSTM kernel / bias gradients.  Data parallel: the x-part X^T dGsum
        (2500 x 1024, 10 MB) is produced in row chunks, each handed to the
        all-reduce as soon as it is final, so the collective of chunk i runs
        under the GEMM of chunk i+1; the recurrent rows and the bias go last.
        rec_done: the recurrent rows were forked already (_weight_grads_rec_side)."""
        B, T, H, C2 = ws.B, self.max_steps, self.rnn_units, self.C2
        gK = self._G("rnn/basic_lstm_cell/kernel")
        gbK = self._G("rnn/basic_lstm_cell/bias")
        if rec_done:
            pass
        elif T > 1 and side and self.REC_WGRAD_SIDE:
            self._weight_grads_rec_side(ws)
        elif T > 1:
            self._dw_rec(ws)
        chunk = self.X_GRAD_CHUNK if self.grad_reducer is not None else C2
        base = self.params.offsets[self._SCOPE_PREFIX + "rnn/basic_lstm_cell/kernel"]
        # bias gradient = colsum(sum_t dG_t) = colsum(dGsum), fused into chunk 0
        m_last = 0
        # (the x-rows gradient GEMM of every chunk is tagged; its operand
        # conversions / splits are not: they are other launches)
        x3p = self._x3p_xgrad(B)
        for m0 in range(0, C2, chunk):
            m_last = m0
            m1 = min(C2, m0 + chunk)
            bias = gbK if m0 == 0 else None
            if self.precision == "bf16":
                # bf16 configuration: X^T dGsum on bf16 operands (fp32
                # accumulate); the forward x-projection stays fp32
                self._x_grad_bf16(X, ws, gK, bias, m0, m1)
            elif x3p:
                if m0 == 0:
                    if getattr(ws, "dG3", None) is None:
                        ws.dG3 = torch.empty((3, B, 4 * H), device=self.device,
                                             dtype=torch.bfloat16)
                    # the pieces of sum_t dG_t, summed in the reversed loop's
                    # order without the running sum (mog_split3_sum_bf16)
                    _ops.split3_sum_bf16_(ws.dG, T, B * 4 * H, ws.dG3, B, 4 * H, 4 * H, 4 * H,
                                          B * 4 * H)
                C2p = self._pad8(C2)
                with self._timed("lstm_x_projection_grad",
                                 ("mfma", 2.0 * B * (m1 - m0) * 4 * H, "fp32", "x3")):
                    ops.gemm_x3p_tn(ws.X3.view(-1)[m0:], B * C2p, ws.dG3, B * 4 * H, gK[m0:m1],
                                    m1 - m0, 4 * H, B, C2p, 4 * H, 4 * H,
                                    splitk=self._sk(max(1, min(B // 256, self.X3_SPLITK))),
                                    colsum=bias, reduce=True)
            elif self.X_GRAD_X3 == 1:
                # fp32 operands split exactly into three bf16 pieces on the
                # bf16 matrix cores (gemm_x3.hip: fp32-level accuracy)
                with self._timed("lstm_x_projection_grad",
                                 ("mfma", 2.0 * B * (m1 - m0) * 4 * H, "fp32", "x3")):
                    ops.gemm_x3_tn(X[:, m0:], ws.dGsum, gK[m0:m1], m1 - m0, 4 * H, B, C2, 4 * H,
                                   4 * H, splitk=self._sk(max(1, min(B // 256, self.X3_SPLITK))),
                                   colsum=bias)
            else:
                self._dw(X[:, m0:], ws.dGsum, gK[m0:m1], B, m1 - m0, 4 * H, C2, 4 * H, bias)
            if m1 < C2:
                self._reduce_bucket(base + m0 * 4 * H, base + m1 * 4 * H)
        self._reduce_bucket(base + m_last * 4 * H, self._bucket_split())

    def _x_bf16(self, X, ws):
        """X in bf16 [B][C2p] (zero pad columns): the A operand of the bf16
        configuration's x-rows gradient, converted once per step -- in the
        forward's side-stream prologue from SIDE_MIN_BATCH (X is the step's
        input, final before the x-projection)."""
        B, C2 = ws.B, self.C2
        C2p = self._pad8(C2)
        if getattr(ws, "Xb", None) is None:
            ws.Xb = torch.zeros((B, C2p), device=self.device, dtype=torch.bfloat16)
        _ops.cvt_bf16_batch_([X], [ws.Xb], [B, C2, C2, B, C2p, C2p, 0])
        ws.xb_fresh = True

    def _x_grad_bf16(self, X, ws, gK, bias_out, m0, m1):
        """The bf16 configuration's x-rows gradient X^T dGsum on gemm_x3p_tn's
        one-piece form (plain bf16 operands, 128 x 128 tiles): X was
        converted in the forward (_x_bf16), dGsum is converted here."""
        B, H, C2 = ws.B, self.rnn_units, self.C2
        C2p = self._pad8(C2)
        if m0 == 0:
            if not getattr(ws, "xb_fresh", False):  # (no conversion in this step's forward)
                self._x_bf16(X, ws)
            ws.xb_fresh = False
            if getattr(ws, "xb_ready", None) is not None:  # (converted on the side stream)
                torch.cuda.current_stream().wait_event(ws.xb_ready)
                ws.xb_ready = None
            if getattr(ws, "dGsumb", None) is None:
                ws.dGsumb = torch.empty((B, 4 * H), device=self.device, dtype=torch.bfloat16)
            _ops.cvt_bf16_batch_([ws.dGsum], [ws.dGsumb], [B, 4 * H, 4 * H, B, 4 * H, 4 * H, 0])
        # split-K 8 at B = 8192, partials summed through the workspace
        # (scripts/x1_sweep.py, us for 1/2/3/4/6/8 splits: 138/84/77/73/73/72;
        # with float atomics 77/76/81/88 from 3 splits)
        with self._timed("lstm_x_projection_grad", ("mfma", 2.0 * B * (m1 - m0) * 4 * H, "bf16")):
            ops.gemm_x3p_tn(ws.Xb.view(-1)[m0:], 0, ws.dGsumb, 0, gK[m0:m1], m1 - m0, 4 * H, B,
                            C2p, 4 * H, 4 * H, splitk=self._sk(max(1, min(B // 1024, 8))),
                            colsum=bias_out, npieces=1)
