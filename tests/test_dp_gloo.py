"""Row E (data parallelism) on CPU: world_size-2 gloo ranks (subprocesses
running tests/dp_worker.py), each running the CPU restatement on its
contiguous shard with the model's 1/(B_local*world) loss scaling, reduced
with the product's all-reduce helper (mog_air.parallel.allreduce_grads), must
reproduce the single-process full-batch gradient.  The MI355X path runs the
same helper over RCCL."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from mog_air import parallel

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dp_worker  # noqa: E402

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_partition():
    for batch in (1, 7, 8, 8192, 10001):
        for world in (1, 2, 3, 8):
            spans = [parallel.shard(batch, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == batch
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        parallel.shard(8, 2, 2)


def test_allreduce_is_noop_without_group():
    g = torch.arange(4.0)
    parallel.allreduce_grads(g)
    assert torch.equal(g, torch.arange(4.0))


@pytest.mark.timeout(300)
def test_dp_gloo_world2_matches_full_batch(tmp_path):
    out = str(tmp_path / "g.npy")
    port = _free_port()
    procs = []
    for r in range(WORLD):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE=str(WORLD), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), out],
                                      env=env))
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * WORLD
    reduced = np.load(out)
    P, nz, x, k = dp_worker.inputs()
    full = dp_worker.grads(P, nz, x, k, 0, dp_worker.B, 1.0)
    np.testing.assert_allclose(reduced, full.numpy(), rtol=1e-9, atol=1e-12)


def _run_world(args):
    port = _free_port()
    procs = []
    for r in range(WORLD):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE=str(WORLD), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py")] + args,
                                      env=env))
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * WORLD


@pytest.mark.timeout(300)
def test_dp_gloo_world2_asr_matches_full_batch(tmp_path):
    """AIR-ASR: with the hooks parallel.attach installs — MAX
    of each step's live flag, SUM of the per-step z_pres probability sums — the
    shards' summed gradient, summed loss and executed step count equal the
    full batch's (each rank's loss is its share of the mean plus the global
    margin, so the summed loss holds the margin world times).  The config is
    chosen so that the shards alone would exit after 3 and 2 steps."""
    out = str(tmp_path / "asr.npz")
    _run_world([out, "asr"])
    r = np.load(out)
    cfg, P, nz, x, G = dp_worker.asr_inputs()
    g_full, loss_full, T_full = dp_worker.asr_grads(cfg, P, nz, x, G, 0, cfg.batch)
    assert int(r["T"][0]) == T_full
    np.testing.assert_allclose(r["g"], g_full.numpy(), rtol=1e-9, atol=1e-12)
    # every rank adds the (global) margin once: sum = full loss + (world - 1) margin
    from oracle import asr_torch as st
    Pt = {n: torch.tensor(v, dtype=torch.float64) for n, v in P.items()}
    margin = float(st.asr_forward(cfg, Pt, nz, torch.tensor(x, dtype=torch.float64),
                                  canvas_cotangent=torch.tensor(G))["margin"])
    assert abs(float(r["loss"][0]) - (loss_full + (WORLD - 1) * margin)) < 1e-8 * max(1.0, abs(loss_full))
