"""The fp32 output layer with its likelihood noise generated in the GEMM
epilogue (mog_gemm_f32_sigmoid_philox) is bit-identical to the same layer
reading a buffer that mog_rng_fill filled from the same Philox counters
(vae.py:44-46, air_model.py:548-550), alone and inside the train model."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


@pytest.mark.parametrize("M,N,K", [(300, 784, 512), (24576, 784, 512), (70, 16, 64)])
def test_gemm_sigmoid_philox_matches_filled_noise(M, N, K):
    from mog_air import ops
    g = torch.Generator().manual_seed(M + N)
    A = (torch.randn(M, K, generator=g) * 0.1).to(DEV)
    B = (torch.randn(K, N, generator=g) * 0.1).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    seed, off = 1235 + M, 77777 + 13 * M
    eps = torch.empty(M, N, device=DEV)
    ops.rng_fill(eps, seed, off, True)
    c_buf = torch.empty(M, N, device=DEV)
    c_gen = torch.empty(M, N, device=DEV)
    ops.gemm([A], [B], [c_buf], M, N, K, K, N, N, epi=ops.EPI_SIGMOID_NOISE, bias=[bias],
             aux=[eps], ldaux=N, aux_scale=0.3)
    ops.gemm_sigmoid_philox(A, B, c_gen, bias, M, N, K, K, N, N, 0.3, seed, off)
    assert torch.equal(c_buf, c_gen)


def test_train_model_epilogue_noise_matches_buffer_noise():
    from mog_air.air_model import AIRModel
    from oracle import air_oracle as ao
    B = 64  # the batched fp32 VAE (B % 64 == 0) generates eps_x in the epilogue
    m = AIRModel(max_steps=3, scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01,
                 learning_rate=1e-4, gradient_clipping_norm=1.0, cnn=False, train=True,
                 scope="philox_ep", device=DEV, noise_seed=4242)
    x, k = ao.synthetic_canvases(B, seed=31)
    assert m._eps_x_in_kernel(B)
    ctr = m._noise_ctr
    m.infer(x, k)
    loss_gen, canvas_gen = m.loss, m.canvas.clone()
    r_gen = m._ws.r.clone()
    m._noise_ctr = ctr
    m._eps_x_in_kernel = lambda b: False  # fill eps_x, read it as the aux operand
    m.infer(x, k)
    assert torch.equal(m._ws.r, r_gen)
    assert torch.equal(m.canvas, canvas_gen)
    assert m.loss == loss_gen
