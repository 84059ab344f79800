"""Hyper-parameters, iteration counter and checkpoint I/O (TD3_base.py:6-50).

``save`` / ``load`` write and read the reference's six files (``critic``,
``critic_target``, ``critic_optimizer``, ``actor``, ``actor_target``,
``actor_optimizer``) as torch state_dicts with the reference key layout, so a
checkpoint moves between the reference and this build in both directions.
Loads use ``torch.load(..., weights_only=True)``.
"""
from __future__ import annotations

import os


class TD3_base(object):
    def __init__(self, max_action=1, discount=0.99, tau=0.005, policy_noise=0.2,
                 noise_clip=0.5, policy_freq=2):
        self.max_action = max_action
        self.discount = discount
        self.tau = tau
        self.policy_noise = policy_noise
        self.noise_clip = noise_clip
        self.policy_freq = policy_freq

    def save(self, folder):                                               # TD3_base.py:26-34
        import torch
        os.makedirs(folder, exist_ok=True)
        torch.save(self.critic.state_dict(), os.path.join(folder, "critic"))
        torch.save(self.critic_target.state_dict(), os.path.join(folder, "critic_target"))
        torch.save(self.critic_optimizer.state_dict(), os.path.join(folder, "critic_optimizer"))
        torch.save(self.actor.state_dict(), os.path.join(folder, "actor"))
        torch.save(self.actor_target.state_dict(), os.path.join(folder, "actor_target"))
        torch.save(self.actor_optimizer.state_dict(), os.path.join(folder, "actor_optimizer"))

    def load(self, folder):                                               # TD3_base.py:37-50
        import torch

        def _ld(name):
            return torch.load(os.path.join(folder, name), map_location="cpu", weights_only=True)

        self.critic.load_state_dict(_ld("critic"))
        self.critic_optimizer.load_state_dict(_ld("critic_optimizer"))
        if os.path.isfile(os.path.join(folder, "critic_target")):
            self.critic_target.load_state_dict(_ld("critic_target"))
        else:
            self.critic_target.load_state_dict(self.critic.state_dict())
        self.actor.load_state_dict(_ld("actor"))
        self.actor_optimizer.load_state_dict(_ld("actor_optimizer"))
        if os.path.isfile(os.path.join(folder, "actor_target")):
            self.actor_target.load_state_dict(_ld("actor_target"))
        else:
            self.actor_target.load_state_dict(self.actor.state_dict())
