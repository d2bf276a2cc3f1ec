"""Row E on the GPU: the HIP AIR and AIR-ASR models with world = 2
(tests/gpu_dp_worker.py ranks, gloo process group, both on cuda:0) against
the single-process full-batch HIP run.

Both batches are odd (13 and 11 images: shards 7 + 6 and 6 + 5), so the
1/B_global gradient scale is exercised.  The summed (all-reduced) gradient
equals the full-batch gradient within summation-order tolerance (the weight
gradients are split-K atomic sums either way); the executed loop steps are
equal (global live flag), counts and per-image losses are bit-exact (every
per-image quantity is independent of the rest of the batch), and the ASR
margin (batch-mean z_pres probabilities through the zsum hook) is the full
batch's on every rank.  The AIR case uses ``-ap`` (num_prior), whose
z_pres_kl_end term depends on the global loop exit."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gpu_dp_worker as W  # noqa: E402

WORLD = 2


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(prefix, kind, world=WORLD):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE=str(world), LOCAL_RANK="0", OMP_NUM_THREADS="1",
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "gpu_dp_worker.py"),
                                       prefix, kind], env=env))
    try:
        rcs = [p.wait(timeout=100) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * world
    return [dict(np.load(f"{prefix}_{r}.npz")) for r in range(world)]


def test_rccl_single_rank_bucketed_allreduce(tmp_path):
    """The data-parallel step over RCCL on the HIP device (one rank: RCCL
    refuses two ranks on one GPU): five bucketed async SUM all-reduces of the
    flat gradient overlapped with the backward and the MAX all-reduce of each
    step's live flag run through RCCL, and the gradient equals the run without
    a reducer bit for bit (a sum over one rank), batched T*B-row VAE path."""
    r = _launch(str(tmp_path / "rccl1"), "rccl1", world=1)[0]
    full = W.run("rccl1", 0, W.BATCH["rccl1"], 1, scope="dp_full_rccl1", attach=False)
    assert int(r["batched"][0]) and len(r["buckets"]) == 5
    np.testing.assert_array_equal(r["digits"], full["digits"])
    assert int(r["T"][0]) == int(full["T"][0])
    err = np.linalg.norm(r["g"] - full["g"]) / np.linalg.norm(full["g"])
    assert err < 1e-5, err  # (split-K atomic weight gradients: order only)


@pytest.mark.parametrize("kind", ["air", "asr", "air64", "air64b", "air1k", "asr1k"])
def test_world2_matches_full_batch(tmp_path, kind):
    """air64 / air64b: 64-row shards, so every rank takes the batched VAE
    (T*B rows; bf16: the fused step kernel), every launch on the main stream
    (below AIRModel.SIDE_MIN_BATCH).  air1k / asr1k: 1,024 images per rank
    (2,048 global), so each rank forks its VAE weight gradients to the side
    stream and joins them before the glimpse bucket's all-reduce
    (air_model.py _vae_weight_grads_async, _backward_body) -- the bench's
    data-parallel schedule (reference semantics: air/air_model.py:966-972,
    air_number_bbox_location.py:386-390)."""
    ranks = _launch(str(tmp_path / kind), kind)
    n = W.BATCH[kind]
    full = W.run(kind, 0, n, 1, scope=f"dp_full_{kind}", attach=False)
    if kind.startswith("air64") or kind == "air1k":
        assert all(int(r["batched"][0]) for r in ranks) and int(full["batched"][0])
    if kind.endswith("1k"):
        assert all(int(r["side"][0]) for r in ranks)
    # every rank holds the same reduced gradient
    np.testing.assert_array_equal(ranks[0]["g"], ranks[1]["g"])
    g, ref = ranks[0]["g"], full["g"]
    err = np.linalg.norm(g - ref) / np.linalg.norm(ref)
    assert err < 1e-5, err
    np.testing.assert_allclose(g, ref, rtol=2e-4, atol=2e-6 * np.abs(ref).max())
    for r in ranks:
        assert int(r["T"][0]) == int(full["T"][0])
        lo, hi = int(r["lo"][0]), int(r["hi"][0])
        np.testing.assert_array_equal(r["digits"], full["digits"][lo:hi])
        np.testing.assert_allclose(r["loss_b"], full["loss_b"][lo:hi], rtol=1e-6)
    # batch mean: the shards' local means weighted by their sizes
    sizes = [int(r["hi"][0] - r["lo"][0]) for r in ranks]
    if not kind.startswith("asr"):
        mean = sum(float(r["mean"][0]) * s for r, s in zip(ranks, sizes)) / n
        assert mean == pytest.approx(float(full["mean"][0]), rel=1e-5)
        # buckets: glimpse block, 3 x-grad chunks, the rest (5 launches)
        assert len(ranks[0]["buckets"]) == 5
    else:
        for r in ranks:
            np.testing.assert_allclose(r["margin"], full["margin"], rtol=1e-6)
