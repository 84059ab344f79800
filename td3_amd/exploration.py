"""Exploration noise for the acting loop.

The reference perturbs ``select_action`` with an Ornstein-Uhlenbeck process
(``utils/noise.py:4-22``, used at ``main.py:240,251-253``): per environment step

    X <- X + (theta * (mu - X) + sigma * n),   n ~ N(0, I) from numpy's global RNG,

and ``reset()`` at episode ends returns X to mu.  It is a few flops per step, so it stays on the
host beside ``env.step``.  The update below keeps the reference's rounding order (drift first,
then the diffusion term, then the add), so a seeded numpy RNG gives the same float64 sequence.
"""
from __future__ import annotations

import numpy as np

__all__ = ["OrnsteinUhlenbeckActionNoise"]


class OrnsteinUhlenbeckActionNoise:
    """Drop-in for the reference class: ``(action_dim, mu=0, theta=0.1, sigma=0.2)``,
    ``sample() -> float64 [action_dim]``, ``reset()``; the state is exposed as ``X``."""

    def __init__(self, action_dim, mu=0, theta=0.1, sigma=0.2):
        self.action_dim = int(action_dim)
        self.mu, self.theta, self.sigma = mu, theta, sigma
        self.reset()

    def reset(self):
        self.X = np.full(self.action_dim, self.mu, dtype=np.float64)

    def sample(self):
        drift = self.theta * (self.mu - self.X)
        step = drift + self.sigma * np.random.randn(self.action_dim)
        self.X = self.X + step
        return self.X
