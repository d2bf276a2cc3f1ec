"""Generation and the result accessors of AIRModel (mixed in): the test
model's generated_samples (air/air_model.py:1001-1146, vae.py:51-86) and the
reference's result attributes (rec_num_digits, rec_scales, ..., sliced to the
executed loop steps)."""
from __future__ import annotations

from typing import Optional

import torch

from . import ops
from .ops import EPI_SIGMOID_NOISE, EPI_SOFTPLUS, gemm

_ops = ops._ops


class Results:
    def generate(self, num_steps: int, batch: Optional[int] = None, noise=None):
        """The test model's ``generated_samples`` (air_model.py:1001-1146):
        ``num_steps`` objects per canvas (``max_steps_generation_placeholder``),
        each with prior-sampled scale / shift / latent, decoded by the
        generative VAE (vae.py:51-86, sigmoid of mean + std * eps) and
        STN-written; the canvas sums every step's window.  Returns the canvas
        [G, C, C, 1]; ``generated_st_back`` [G, T, 2, 3] and
        ``generated_num_digits`` [G] hold the loop's other outputs.  ``noise``
        (optional) injects eps_scale [T,G], eps_shift [T,G,2], eps_z [T,G,Z],
        eps_x [T,G,784]; otherwise device Philox noise is drawn.  Runs the
        fp32 decoder GEMMs in either precision."""
        G = int(batch if batch is not None else self.generation_batch_size)
        T, C, W2, Z = int(num_steps), self.canvas_size, self.W2, self.vae_latent_dimensions
        G1, G2 = self.vae_generative_units
        dev = self.device
        e = lambda *sh: torch.empty(sh, device=dev, dtype=torch.float32)  # noqa: E731
        eps = {"eps_scale": e(T, G), "eps_shift": e(T, G, 2), "eps_z": e(T, G, Z),
               "eps_x": e(T, G, W2)}
        for k, buf in eps.items():
            if noise is not None:
                buf.copy_(torch.as_tensor(noise[k], dtype=torch.float32))
            else:
                ops.rng_fill(buf, self.noise_seed, self._noise_ctr, True)
                self._noise_ctr += (buf.numel() + 3) // 4
        canvas = torch.zeros((G, C * C), device=dev, dtype=torch.float32)
        st_back = e(T, G, 6)
        scale, shift, z = e(G), e(G, 2), e(G, Z)
        d1, d2, r = e(G, G1), e(G, G2), e(G, W2)
        ones = torch.ones(G, device=dev, dtype=torch.float32)
        vw = {n: self._P("vae/" + n + "/weights") for n in self._VAE}
        vb = {n: self._P("vae/" + n + "/biases") for n in self._VAE}
        lik_std = float(self.hyper("vae_likelihood_std"))
        for t in range(T):
            _ops.generation_prior_(G, Z, float(self.scale_prior_mean),
                                   self.scale_prior_log_variance, float(self.shift_prior_mean),
                                   self.shift_prior_log_variance, float(self.vae_prior_mean),
                                   self.vae_prior_log_variance, eps["eps_scale"][t],
                                   eps["eps_shift"][t], eps["eps_z"][t], st_back[t], scale, shift,
                                   z)
            gemm([z], [vw["generative_1"]], [d1], G, G1, Z, Z, G1, G1, epi=EPI_SOFTPLUS,
                 bias=[vb["generative_1"]])
            gemm([d1], [vw["generative_2"]], [d2], G, G2, G1, G1, G2, G2, epi=EPI_SOFTPLUS,
                 bias=[vb["generative_2"]])
            gemm([d2], [vw["gen_mean"]], [r], G, W2, G2, G2, W2, W2, epi=EPI_SIGMOID_NOISE,
                 bias=[vb["gen_mean"]], aux=[eps["eps_x"][t]], ldaux=W2, aux_scale=lik_std)
            # every step is written (the stopping sum stays 0 < threshold, :1085-1097)
            ops.stn_forward(r, st_back[t], (C, C), out=canvas, z=ones, mask=ones,
                            accumulate=True)
        self.generated_st_back = st_back.transpose(0, 1).reshape(G, T, 2, 3)
        self.generated_num_digits = torch.full((G,), T, device=dev, dtype=torch.int32)
        self.generated_samples = canvas.reshape(G, C, C, 1)
        return self.generated_samples

    # ------------------------------------------------------- outputs -------
    def _T(self) -> int:
        live = self._ws.live.detach().cpu().numpy()
        return int(live[: self.max_steps].sum())

    def _bt(self, t: torch.Tensor) -> torch.Tensor:
        T = self._T()
        return t[:T].transpose(0, 1)

    @property
    def executed_steps(self) -> int:
        return self._T()

    @property
    def loss(self):
        return float(self._ws.means[0])

    @property
    def accuracy(self):
        return float(self._ws.means[1])

    @property
    def mse_loss(self):
        return float(self._ws.means[2])

    @property
    def rec_num_digits(self):
        return self._ws.digits

    @property
    def accuracy_instance(self):
        return self._ws.acc_b

    @property
    def rec_scales(self):
        return self._bt(self._ws.scale).unsqueeze(-1)

    @property
    def rec_shifts(self):
        return self._bt(self._ws.shift)

    @property
    def rec_st_back(self):
        return self._bt(self._ws.th_b).reshape(self._ws.B, -1, 2, 3)

    @property
    def rec_windows(self):
        return self._bt(self._ws.r)

    @property
    def rec_latents(self):
        return self._bt(self._ws.z)

    @property
    def z_pres_probs(self):
        return self._bt(self._ws.zprob)

    @property
    def z_pres_kls(self):
        return self._bt(self._ws.zkl)

    @property
    def scale_kls(self):
        return self._bt(self._ws.skl)

    @property
    def shift_kls(self):
        return self._bt(self._ws.shkl)

    @property
    def vae_kls(self):
        return self._bt(self._ws.vkl)

    @property
    def reconstruction(self):
        self._materialize()
        return self._ws.recon

    @property
    def reconstruction_loss(self):
        return self._ws.bce

    @property
    def canvas(self):
        self._materialize()
        return self._ws.canvas

    @property
    def per_image_loss(self):
        return self._ws.loss_b
