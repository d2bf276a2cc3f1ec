"""Data parallelism for the AIR train step.

Every image is independent in AIR, so the batch is sharded contiguously over
ranks (one process per GPU) and the only exchange is a SUM all-reduce of the
flat fp32 gradient buffer per step (4.01 M values = 16.05 MB).  Each rank
scales its loss gradient by 1/B_global (the model's ``_gscale``; B_global is
the step's global batch, so unequal shards weigh every image alike) and the
summed buffer is the global-batch mean.  NaN/Inf zeroing, per-tensor
clip_by_norm and Adam run after the all-reduce, on identical buffers on every
rank, as the single-process reference applies them to the batch-mean
gradient (air/air_model.py:966-972).

Bucketing and overlap (GradReducer): the AIR backward hands the buffer to the
collective in buckets as they become final -- first the heads + VAE block
(1.2 M values, final once the glimpse-path backward is done; its all-reduce
runs under the sequential LSTM chain), then the x-part of the LSTM kernel
gradient in 640-row chunks (each all-reduced while the next chunk's GEMM
runs), the recurrent rows + bias last.  Each launch is ``async_op``; on
MI355X the backend is "nccl" (= RCCL over xGMI), which orders the
collective after the producing kernels on the current stream and lets
``wait()`` make the stream (not the host) wait before clip + Adam.  The same
code runs with "gloo" (CPU tensors, or HIP tensors staged through the host)
for the multi-process tests.
"""
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def shard(batch: int, rank: int, world: int) -> Tuple[int, int]:
    """[start, stop) of this rank's contiguous shard of a global batch; ranks
    differ by at most one image."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} for world {world}")
    base, extra = divmod(batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def allreduce_grads(grad: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> None:
    """In-place SUM all-reduce of the flat gradient buffer (no-op at world 1)."""
    if not dist.is_available() or not dist.is_initialized():
        return
    if dist.get_world_size(group) == 1:
        return
    if not grad.is_contiguous():
        raise ValueError("gradient buffer must be contiguous (one collective per step)")
    dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)


class GradReducer:
    """Bucketed, asynchronous SUM all-reduce of views of the flat gradient
    buffer: ``launch(view)`` when a bucket is final, ``wait()`` once before
    the optimizer.  ``log`` (optional list) records (offset-free) bucket sizes
    for tests."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None):
        self.group = group
        self.pending: List = []
        self.log: Optional[List[int]] = None

    def launch(self, view: torch.Tensor) -> None:
        if view.numel() == 0:
            return
        if not view.is_contiguous():
            raise ValueError("gradient bucket must be a contiguous view")
        if self.log is not None:
            self.log.append(view.numel())
        self.pending.append(dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group,
                                            async_op=True))

    def wait(self) -> None:
        for w in self.pending:
            w.wait()
        self.pending.clear()


def attach(model, group: Optional[dist.ProcessGroup] = None,
           global_steps: Optional[bool] = None) -> GradReducer:
    """Make ``model`` (an AIRModel built with grad_world = world size)
    all-reduce its gradients across ``group`` (bucketed, overlapped with the
    backward) before clipping and the optimizer.

    ``global_steps``: all-reduce (MAX) each loop step's "any image still
    active" flag so every rank runs the data-dependent loop of the GLOBAL batch
    (air_model.py:428-432).  AIR-ASR always needs it (its losses cover every
    executed step, air_number_bbox_location.py:1017-1063); AIR needs it only
    with ``num_prior`` (``-ap``: the z_pres_kl_end term of :646-653 is added
    while the loop runs), which is the default (None); pass True to make the
    executed step count equal the full batch's in any case."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if getattr(model, "grad_world", 1) != world:
        raise ValueError(f"model.grad_world={model.grad_world} but the group has {world} ranks")
    reducer = GradReducer(group)
    model.grad_reducer = reducer if world > 1 else None
    if world > 1:
        asr = hasattr(model, "zsum_hook")
        if global_steps is None:
            global_steps = asr or getattr(model, "marginal", None) is not None
        if global_steps:
            model.live_hook = lambda live, t: dist.all_reduce(live[t + 1:t + 2],
                                                              op=dist.ReduceOp.MAX, group=group)
        if asr:
            # the margin / element losses use the batch-mean z_pres
            # probabilities (:982-998) -> SUM of the per-step partial sums
            model.zsum_hook = lambda zsum: dist.all_reduce(zsum, op=dist.ReduceOp.SUM,
                                                           group=group)
    return reducer
