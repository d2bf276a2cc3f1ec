"""Graph capture of the AIR train step (AIRModel mixes this in): the forward
+ backward replayed from one hipGraph (torch.cuda.CUDAGraph), bit-identical
to the eager step (tests/test_gpu_graph.py).  The reference's batch of 64
(training_air_original.py:22) is launch-bound without it."""
from __future__ import annotations

from typing import Optional

import torch

from . import ops


class GraphCapture:
    # A captured train step (hipGraph through torch.cuda.CUDAGraph): the whole
    # forward + backward -- ~80 launches, every one of them with arguments that
    # are the same from step to step -- replays as ONE graph launch.  What
    # changes per step stays outside the graph or is read from device memory:
    # the Philox noise fills (their counter offsets advance, eager launches
    # before the replay; eps_x is filled too instead of being generated inside
    # the VAE kernels), the annealed z_pres prior log-odds (a device scalar the
    # step kernels read, filled before the replay) and TF Adam (lr_t from the
    # fp32 beta powers, an eager launch after it).  The reference's batch of 64
    # (training_air_original.py:22) is launch-bound without it.
    _graph_noise = False  # eps_x filled into its buffer (graph mode)
    _graph_mode = False   # inside train_step_graphed (eager first step, capture, replay)
    _prior_dev = None     # device z_pres prior log-odds (graph mode only)
    _prior_dev_val = None  # the value last written there
    _graph = None
    _graph_ws = None      # the workspace the graph was captured on (its pointers)

    def _prior_arg(self):
        """The device prior log-odds the step kernels read instead of the host
        scalar: only in graph mode, where train_step_graphed refreshes it
        before every replay.  Eager steps pass the host value (None here), so a
        stale device value from an earlier graphed step is never read."""
        return self._prior_dev if self._graph_mode else None

    def _graph_ok(self):
        others = [k for k in self.annealing_schedules if k != "z_pres_prior_log_odds"]
        if others:
            raise NotImplementedError(f"graph mode: annealed {others} would be frozen at capture")
        if self.grad_reducer is not None or self.live_hook is not None:
            raise NotImplementedError("graph mode is the single-device train step")

    def train_step_graphed(self, images, targets=None, global_batch: Optional[int] = None) -> None:
        """train_step_async with the forward + backward replayed from a captured
        graph; bit-identical to it.  The first call at a batch shape runs the
        step eagerly and captures the graph (capture executes nothing); later
        calls copy the inputs into the graph's static buffers and replay."""
        if not self.train:
            raise RuntimeError("train_step on a model built with train=False")
        self._graph_ok()
        self._graph_mode = self._graph_noise = True
        try:
            self._train_step_graphed(images, targets, global_batch)
        finally:
            self._graph_mode = self._graph_noise = False

    def _train_step_graphed(self, images, targets, global_batch):
        X, tg = self._prep(images, targets)
        key = (tuple(X.shape), None if tg is None else tuple(tg.shape), global_batch)
        if self._graph is None or self._graph_key != key:
            self._graph = self._graph_ws = None
            if self._prior_dev is None:
                self._prior_dev = torch.zeros(1, device=self.device)
            self._prior_dev_val = float(self.hyper("z_pres_prior_log_odds"))
            self._prior_dev.fill_(self._prior_dev_val)
            self.train_step_async(X, tg, global_batch=global_batch)  # this call's step
            self._capture(X, tg, global_batch)
            self._graph_key = key
            return
        gX, gT = self._graph_io
        # the inputs into the graph's static buffers, both in one launch
        dst, src = [], []
        if X.data_ptr() != gX.data_ptr():
            dst.append(gX)
            src.append(X)
        if tg is not None and tg.data_ptr() != gT.data_ptr():
            dst.append(gT)
            src.append(tg)
        if dst:
            ops._ops.copy32_batch_(dst, src)
        # The graph holds raw pointers into the workspace it was captured on:
        # replay on that one (kept alive by _graph_ws), even when an infer /
        # step / compute_gradients at another batch has replaced self._ws since
        ws = self._ws = self._graph_ws
        self._fill_noise(ws, None)
        if ws.noise_side:  # the graph's first launch reads it
            torch.cuda.current_stream().wait_stream(self._side_stream())
            ws.noise_side = False
        lo = float(self.hyper("z_pres_prior_log_odds"))
        if lo != self._prior_dev_val:  # (a fill launch only when the value moves)
            self._prior_dev.fill_(lo)
            self._prior_dev_val = lo
        self._graph.replay()
        self.params.apply_adam(self.hyper("learning_rate"), self.gradient_clipping_norm)
        self.params.global_step += 1
        self._X = gX
        self._loss_inputs = (gX, gT)
        ws.materialized = False
        self._outputs_ready = True

    def _capture(self, X, tg, global_batch):
        ws = self._ws
        gX = X.clone()
        gT = tg.clone() if tg is not None else None
        self._graph_io = (gX, gT)
        # the weight packs are refreshed by a launch inside the graph on every
        # replay (the parameters change every step): force it to be recorded
        self._pack_version = self._pack32_version = self._w1cat_version = None
        self._w3_version = self._vae_wT_version = None
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        self._global_batch = global_batch
        with torch.cuda.graph(g):
            self._forward(gX, gT, ws, need_grad=True, outputs=False)
            self._backward(gX, ws)
        self._graph = g
        self._graph_ws = ws
        # capture executed nothing: the weight packs / copies recorded above
        # are not in their buffers yet, so the next eager use must refresh them
        self._pack_version = self._pack32_version = self._w1cat_version = None
        self._w3_version = self._vae_wT_version = None
