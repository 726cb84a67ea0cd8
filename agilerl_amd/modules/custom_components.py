"""NoisyLinear and GumbelSoftmax (agilerl/modules/custom_components.py:10-131)."""

from __future__ import annotations

import math

import torch
from torch import nn
from torch.nn import functional as F


class GumbelSoftmax(nn.Module):
    """softmax(logits + Gumbel noise) over the last dim (custom_components.py:10-35)."""

    @staticmethod
    def gumbel_softmax(logits: torch.Tensor, tau: float = 1.0, eps: float = 1e-20) -> torch.Tensor:
        u = torch.rand_like(logits)
        return F.softmax((logits - torch.log(-torch.log(u + eps) + eps)) / tau, dim=-1)

    def forward(self, input: torch.Tensor) -> torch.Tensor:
        return self.gumbel_softmax(input)


@torch.no_grad()
def reset_noise_layers(layers: list) -> None:
    """NoisyLinear.reset_noise of each layer in order (custom_components.py:
    116-131).  Every layer's two torch.randn draws are made in the
    reference's order; on the GPU the transform sign(x) sqrt(|x|), the outer
    product and both epsilon writes of up to 16 layers are one agx_noisy_reset
    launch (bit-identical to the torch ops: one correctly rounded sqrt and
    one multiply per element)."""
    if not layers:
        return
    if layers[0].weight_mu.device.type != "cuda":
        for m in layers:
            eps_in, eps_out = m._scale_noise(m.in_features), m._scale_noise(m.out_features)
            m.weight_epsilon.copy_(eps_out.ger(eps_in))
            m.bias_epsilon.copy_(eps_out)
        return
    from .. import kernels as K

    for c in range(0, len(layers), 16):
        batch = []
        for m in layers[c:c + 16]:
            dev = m.weight_mu.device
            eps_in = torch.randn(m.in_features, device=dev)
            eps_out = torch.randn(m.out_features, device=dev)
            batch.append((eps_in, eps_out, m.weight_epsilon, m.bias_epsilon))
        K.noisy_reset_(batch)


# noisy weights formed once per update (noisy_scope): NoisyLinear -> (W, b)
_SCOPE: dict | None = None


class noisy_scope:
    """Within one update the parameters and noise of every NoisyLinear are
    fixed, and the reference's update runs the online network twice (on s'
    for a*, on s for the loss) and the target once: inside this scope each
    layer forms mu + sigma * eps once and reuses it (the same tensors the
    repeated forwards would compute, so results are bit-identical; the
    gradient path goes through _NoisyParam).  RainbowDQN._losses opens it."""

    def __enter__(self):
        global _SCOPE
        self._prev, _SCOPE = _SCOPE, {}
        return self

    def __exit__(self, *exc):
        global _SCOPE
        _SCOPE = self._prev
        return False


class _NoisyParam(torch.autograd.Function):
    """mu + sigma * eps already formed (``w``): forward returns it; backward is
    autograd's for the expression (d mu = g, d sigma = g * eps)."""

    @staticmethod
    def forward(ctx, mu, sigma, eps, w):
        ctx.save_for_backward(eps)
        return w.view_as(w)

    @staticmethod
    def backward(ctx, g):
        (eps,) = ctx.saved_tensors
        return g, g * eps, None, None


class NoisyLinear(nn.Module):
    """Factorised-Gaussian noisy linear layer (custom_components.py:38-131):
    mu ~ U(+-1/sqrt(in)), sigma = std_init/sqrt(in) (weights) and
    std_init/sqrt(out) (bias); eps = sign(x) sqrt(|x|), x ~ N(0,1); train mode
    uses mu + sigma * eps, eval mode mu."""

    def __init__(self, in_features: int, out_features: int, std_init: float = 0.5, device="cpu"):
        super().__init__()
        self.in_features, self.out_features, self.std_init = in_features, out_features, std_init
        self.weight_mu = nn.Parameter(torch.empty(out_features, in_features, device=device))
        self.weight_sigma = nn.Parameter(torch.empty(out_features, in_features, device=device))
        self.register_buffer("weight_epsilon", torch.empty(out_features, in_features, device=device))
        self.bias_mu = nn.Parameter(torch.empty(out_features, device=device))
        self.bias_sigma = nn.Parameter(torch.empty(out_features, device=device))
        self.register_buffer("bias_epsilon", torch.empty(out_features, device=device))
        self.reset_parameters()
        self.reset_noise()

    @torch.no_grad()
    def reset_parameters(self) -> None:
        mu_range = 1 / math.sqrt(self.in_features)
        self.weight_mu.uniform_(-mu_range, mu_range)
        self.weight_sigma.fill_(self.std_init / math.sqrt(self.in_features))
        self.bias_mu.uniform_(-mu_range, mu_range)
        self.bias_sigma.fill_(self.std_init / math.sqrt(self.out_features))

    def _scale_noise(self, size: int) -> torch.Tensor:
        x = torch.randn(size, device=self.weight_mu.device)
        return x.sign().mul_(x.abs().sqrt_())

    @torch.no_grad()
    def reset_noise(self) -> None:
        reset_noise_layers([self])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.training:
            if _SCOPE is None:
                return F.linear(x, self.weight_mu + self.weight_sigma * self.weight_epsilon,
                                self.bias_mu + self.bias_sigma * self.bias_epsilon)
            wb = _SCOPE.get(id(self))
            if wb is None:
                with torch.no_grad():
                    wb = _SCOPE[id(self)] = (self.weight_mu + self.weight_sigma * self.weight_epsilon,
                                             self.bias_mu + self.bias_sigma * self.bias_epsilon)
            if torch.is_grad_enabled():
                return F.linear(x, _NoisyParam.apply(self.weight_mu, self.weight_sigma, self.weight_epsilon, wb[0]),
                                _NoisyParam.apply(self.bias_mu, self.bias_sigma, self.bias_epsilon, wb[1]))
            return F.linear(x, wb[0], wb[1])
        return F.linear(x, self.weight_mu, self.bias_mu)
