"""The small-batch NT path of mog_gemm_f32 (csrc/gemm_f32.hip launch_auto:
an operand off the LDS-DMA alignment -- K = Z = 50, the latent layer's input
gradient at the reference's batch of 64 -- with fewer than 128 tiles of
64 x 64 runs on 32 x 32 x 32 register-staged tiles).  Every output element is
still ONE k-ordered fp32 fma chain (from +0, or continuing Cin), so the small
problem must equal, bit for bit, the same rows computed inside a tall
problem that takes the 64 x 64 x 16 path, and a float64 restatement within
fp32 rounding -- for the plain store, the softplus-backward epilogue
(acc * (1 - exp(-aux)), aux = the layer's softplus output) and Cin, with
ragged M / N."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


@pytest.mark.parametrize("M,N", [(64, 256), (45, 77), (192, 50)])
@pytest.mark.parametrize("epi,cin", [("store", False), ("softplus_bwd", False),
                                     ("softplus_bwd", True), ("store", True)])
def test_nt_small_tiles_equal_tall_path_and_float64(M, N, epi, cin):
    from mog_air import ops
    K, MB = 50, 4096  # MB rows: >= 128 tiles of 64 x 64 (the 64 x 64 x 16 path)
    rng = np.random.default_rng(M * 7 + N + (epi == "store") + 2 * cin)
    A = rng.standard_normal((MB, K)).astype(np.float32)
    W = rng.standard_normal((N, K)).astype(np.float32)          # B = W [N][K] (transB)
    aux = np.log1p(np.exp(rng.standard_normal((MB, N)) * 3)).astype(np.float32)
    Cin = rng.standard_normal((MB, N)).astype(np.float32)
    e = ops.EPI_SOFTPLUS_BWD if epi == "softplus_bwd" else ops.EPI_STORE
    d = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(DEV)  # noqa: E731

    def run(rows):
        C = torch.full((rows, N), float("nan"), device=DEV)
        ops.gemm([d(A[:rows])], [d(W)], [C], rows, N, K, K, K, N, transB=True, epi=e,
                 Cin=[d(Cin[:rows])] if cin else None,
                 aux=[d(aux[:rows])] if e == ops.EPI_SOFTPLUS_BWD else None,
                 ldaux=N if e == ops.EPI_SOFTPLUS_BWD else 0)
        torch.cuda.synchronize()
        return C.cpu()

    small, tall = run(M), run(MB)
    assert torch.equal(small, tall[:M])
    ref = A[:M].astype(np.float64) @ W.T.astype(np.float64)
    bound = np.abs(A[:M]).astype(np.float64) @ np.abs(W.T).astype(np.float64)
    if cin:
        ref, bound = ref + Cin[:M], bound + np.abs(Cin[:M])
    if e == ops.EPI_SOFTPLUS_BWD:
        sig = -np.expm1(-aux[:M].astype(np.float64))
        ref, bound = ref * sig, bound * sig
    err = np.abs(small.numpy().astype(np.float64) - ref)
    assert (err <= 1e-6 * bound + 1e-30).all(), float((err / (bound + 1e-30)).max())
