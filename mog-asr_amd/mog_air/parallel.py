"""Data parallelism for the AIR train step.

Every image is independent in AIR, so the batch is sharded contiguously over
ranks (one process per GPU) and the only exchange is ONE all-reduce of the
flat fp32 gradient buffer per step (4.01 M values = 16.05 MB), SUM over ranks.
The 1/world factor is folded into the loss-mean gradient scale (``grad_world``
in the model: d(loss)/d(x) is scaled by 1/(B_local * world)), so the summed
buffer is already the global-batch mean.  NaN/Inf zeroing, per-tensor
clip_by_norm and Adam run after the all-reduce, on identical buffers on every
rank (training_air_original.py:84-88 applies them to the averaged gradient
of the single-process reference).

On MI355X the backend is "nccl" (= RCCL over xGMI); the same code runs with
"gloo" on CPU tensors for the host-side tests.  The buffer is contiguous
(ParamStore), so one collective moves it at ring bandwidth: 16 MB is large
enough that a single bucket is link-bound, not latency-bound, on 7 xGMI links.
"""
from typing import Optional, Tuple

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


def attach(model, group: Optional[dist.ProcessGroup] = None) -> None:
    """Make ``model`` (an AIRModel built with grad_world = world size) reduce
    its gradients across ``group`` before clipping and the optimizer."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if getattr(model, "grad_world", 1) != world:
        raise ValueError(f"model.grad_world={model.grad_world} but the group has {world} ranks")
    model.grad_hook = lambda g: allreduce_grads(g, group)
    if world > 1 and hasattr(model, "zsum_hook"):
        # AIR-ASR (air_number_bbox_location.py): the loop predicate is global
        # over the batch (:386-390) -> MAX of each step's live flag; the margin
        # loss uses the batch-mean z_pres probabilities (:982-998) -> SUM of
        # the per-step partial sums.  Both stay on the stream (no host sync).
        model.live_hook = lambda live, t: dist.all_reduce(live[t + 1:t + 2],
                                                          op=dist.ReduceOp.MAX, group=group)
        model.zsum_hook = lambda zsum: dist.all_reduce(zsum, op=dist.ReduceOp.SUM, group=group)
