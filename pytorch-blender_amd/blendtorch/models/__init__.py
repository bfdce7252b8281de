"""Consumer models used by the examples and the benchmark (random init).

* :class:`Discriminator` -- the DCGAN image discriminator of the densityopt
  example (reference: examples/densityopt/densityopt.py:139-190): 4x
  [conv4x4/s2 -> BN -> LeakyReLU(0.2)] then conv4x4 -> sigmoid, ndf=32, for
  64x64 inputs.  ``adaptive=True`` inserts a global pooling head so the same
  stack scores 640x480 Cube frames (used by ``bench.py --consumer disc``).
* :class:`ProbModel` -- LogNormal simulation-parameter model trained with the
  score-function gradient (densityopt.py:30-93).
* :class:`CartpolePolicy` -- the P-controller of examples/control/cartpole.py
  as a batched GPU module.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.distributions as D


def _weights_init(m):
    name = m.__class__.__name__
    if 'Conv' in name:
        nn.init.normal_(m.weight, 0.0, 0.02)
    elif 'BatchNorm' in name:
        nn.init.normal_(m.weight, 1.0, 0.02)
        nn.init.zeros_(m.bias)


class Discriminator(nn.Module):
    """DCGAN discriminator: N x nc x H x W -> N probabilities."""

    def __init__(self, nc=3, ndf=32, adaptive=False):
        super().__init__()
        layers = []
        cin = nc
        for i, mult in enumerate((1, 2, 4, 8)):
            layers += [nn.Conv2d(cin, ndf * mult, 4, 2, 1, bias=False), nn.BatchNorm2d(ndf * mult),
                       nn.LeakyReLU(0.2, inplace=True)]
            cin = ndf * mult
        if adaptive:
            layers += [nn.AdaptiveAvgPool2d(4)]
        layers += [nn.Conv2d(cin, 1, 4, 1, 0, bias=False), nn.Sigmoid()]
        self.features = nn.Sequential(*layers)
        self.apply(_weights_init)

    def forward(self, x):
        return self.features(x).view(-1, 1).squeeze(1)


class ProbModel(nn.Module):
    """Factorised LogNormal over simulation parameters (densityopt.py:30-93).

    ``sample(n)`` draws parameters; ``log_prob(samples)`` gives per-sample
    log-densities used by the REINFORCE estimator
    ``grad E[f(x)] = E[(f(x) - b) grad log p(x)]``.
    """

    def __init__(self, mu0, std0):
        super().__init__()
        mu0 = torch.as_tensor(mu0, dtype=torch.float32)
        std0 = torch.as_tensor(std0, dtype=torch.float32)
        self.log_mu = nn.Parameter(torch.log(mu0))
        self.log_std = nn.Parameter(torch.log(std0))

    @property
    def m(self):
        return torch.exp(self.log_mu)

    @property
    def s(self):
        return torch.exp(self.log_std)

    def dist(self):
        return D.LogNormal(self.log_mu, torch.exp(self.log_std))

    def sample(self, n):
        with torch.no_grad():
            return self.dist().sample((n,))

    def log_prob(self, samples):
        return self.dist().log_prob(samples).sum(-1)

    def readable_params(self):
        return self.dist().mean.detach()


class CartpolePolicy(nn.Module):
    """Proportional controller ``a = kappa * (pole_x - cart_x)`` for a batch
    of observations ``(cart_x, pole_x, pole_angle)`` (examples/control/
    cartpole.py:17-36), evaluated on the GPU for many envs at once."""

    def __init__(self, kappa=30.0):
        super().__init__()
        self.register_buffer('kappa', torch.tensor(float(kappa)))

    def forward(self, obs):
        return self.kappa * (obs[..., 1] - obs[..., 0])
