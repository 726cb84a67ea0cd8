"""CPU restatement of the reference's PPO population iteration (TEST
INFRASTRUCTURE ONLY — the timed CPU baseline in bench.py).

Mirrors what the reference runs for config 2 on a CPU device, one agent after
another (agilerl/training/train_on_policy.py:210-243):
  * networks as ``create_mlp`` builds them (agilerl/utils/evolvable_networks.py
    :527-644): Linear -> LayerNorm -> ReLU blocks, encoder output LayerNorm
    without affine, heads with x0.1 output init; shared encoder (ppo.py:487-491);
  * rollout: per vector step ``get_action`` (softmax + multinomial,
    agilerl/utils/torch_utils.py:130-139), env step, buffer write
    (agilerl/rollouts/on_policy.py:82-172);
  * GAE with the numpy restatement (rollout_buffer.py:413-481);
  * learn (ppo.py:814-921): normalise, E epochs x shuffled minibatches, loss,
    backward, clip_grad_norm_ x2, Adam.
"""

from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn

from . import gae as ogae


def _mlp(fin, hidden, fout, out_ln_plain=False, out_act=False, vanish=True):
    layers = []
    dims = [fin, *hidden]
    for i in range(1, len(dims)):
        lin = nn.Linear(dims[i - 1], dims[i])
        nn.init.orthogonal_(lin.weight, math.sqrt(2))
        nn.init.zeros_(lin.bias)
        layers += [lin, nn.LayerNorm(dims[i]), nn.ReLU()]
    out = nn.Linear(dims[-1], fout)
    nn.init.orthogonal_(out.weight, math.sqrt(2))
    nn.init.zeros_(out.bias)
    if vanish:
        out.weight.data.mul_(0.1)
        out.bias.data.mul_(0.1)
    layers.append(out)
    if out_ln_plain:
        layers.append(nn.LayerNorm(fout, elementwise_affine=False))
    if out_act:
        layers.append(nn.ReLU())
    return nn.Sequential(*layers)


class CpuPPOAgent:
    def __init__(self, obs_dim=8, n_actions=4, num_envs=128, learn_step=2048, batch_size=128, lr=1e-3,
                 hidden=64, latent=64, update_epochs=4, seed=0):
        torch.manual_seed(seed)
        self.encoder = _mlp(obs_dim, [hidden], latent, out_ln_plain=True, out_act=True, vanish=False)
        self.actor = _mlp(latent, [hidden], n_actions)
        self.critic = _mlp(latent, [hidden], 1)
        self.opt = torch.optim.Adam(
            list(self.encoder.parameters()) + list(self.actor.parameters()) + list(self.critic.parameters()), lr=lr)
        self.N, self.T = num_envs, -(learn_step // -num_envs)
        self.b, self.E = batch_size, update_epochs
        self.obs_dim = obs_dim

    @torch.no_grad()
    def get_action(self, obs):
        lat = self.encoder(torch.from_numpy(obs))
        logits = self.actor(lat)
        p = torch.softmax(logits, -1)
        a = torch.multinomial(p, 1).squeeze(-1)
        logp = torch.log_softmax(logits, -1).gather(-1, a[:, None]).squeeze(-1)
        v = self.critic(lat).squeeze(-1)
        return a.numpy(), logp.numpy(), v.numpy()

    def iteration(self, env):
        T, N, D = self.T, self.N, self.obs_dim
        obs_buf = np.zeros((T, N, D), np.float32)
        act_buf = np.zeros((T, N), np.int64)
        rew_buf = np.zeros((T, N), np.float32)
        done_buf = np.zeros((T, N), bool)
        val_buf = np.zeros((T, N), np.float32)
        lp_buf = np.zeros((T, N), np.float32)
        # the env is reset once, on the first collect (rollouts/on_policy.py:50-56);
        # later rollouts continue from the last observation
        if getattr(self, "_obs", None) is None:
            obs, _ = env.reset()
            self._obs = np.array(obs)
        obs = self._obs
        term = np.zeros(N, bool)
        for t in range(T):
            a, lp, v = self.get_action(obs)
            nobs, r, term, trunc, _ = env.step(a)
            obs_buf[t], act_buf[t], rew_buf[t], done_buf[t], val_buf[t], lp_buf[t] = obs, a, r, term | trunc, v, lp
            obs = np.array(nobs)
        self._obs = obs
        _, _, lv = self.get_action(obs)
        adv, ret = ogae.gae(rew_buf, val_buf, done_buf, lv, term)
        S = T * N
        ob = torch.from_numpy(obs_buf.reshape(S, D))
        ac = torch.from_numpy(act_buf.reshape(S))
        olp = torch.from_numpy(lp_buf.reshape(S))
        ov = torch.from_numpy(val_buf.reshape(S))
        A = torch.from_numpy(adv.reshape(S))
        A = (A - A.mean()) / (A.std() + 1e-8)
        R = torch.from_numpy(ret.reshape(S))
        idx = np.arange(S)
        actor_params = list(self.encoder.parameters()) + list(self.actor.parameters())
        for _ in range(self.E):
            np.random.shuffle(idx)
            for s in range(0, S, self.b):
                mb = idx[s: s + self.b]
                lat = self.encoder(ob[mb])
                logits = self.actor(lat)
                value = self.critic(lat).squeeze(-1)
                logp_all = torch.log_softmax(logits, -1)
                p = torch.softmax(logits, -1)
                ent = -(p * torch.log(p + 1e-8)).sum(-1)
                logp = logp_all.gather(-1, ac[mb][:, None]).squeeze(-1)
                ratio = torch.exp(logp - olp[mb])
                pl = torch.max(-A[mb] * ratio, -A[mb] * torch.clamp(ratio, 0.8, 1.2)).mean()
                vc = ov[mb] + torch.clamp(value - ov[mb], -0.2, 0.2)
                vl = 0.5 * torch.max((value - R[mb]) ** 2, (vc - R[mb]) ** 2).mean()
                loss = pl + 0.5 * vl - 0.01 * ent.mean()
                self.opt.zero_grad()
                loss.backward()
                nn.utils.clip_grad_norm_(actor_params, 0.5)
                nn.utils.clip_grad_norm_(self.critic.parameters(), 0.5)
                self.opt.step()
        return S
