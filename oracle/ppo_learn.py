"""Pure-PyTorch fp32 restatement of one PPO learn() (TEST INFRASTRUCTURE ONLY:
the checker for the fused HIP learner, never imported by the product path).

Follows agilerl/algorithms/ppo.py:814-921 (``_learn_from_rollout_buffer_flat``)
line by line for ONE agent, on the shared-encoder MLP actor-critic the
reference builds (agilerl/utils/evolvable_networks.py:527-644 ``create_mlp``;
networks/base.py:541-561; ppo.py:487-491):

  * advantages normalised once, ``(a - a.mean()) / (a.std() + 1e-8)`` (:829-834);
  * per epoch the cumulative shuffle ``perms[e]`` (the caller supplies the
    np.random.shuffle stream, :836-842), contiguous minibatches, the last one
    short (:843-845);
  * evaluate_actions: latent = encoder(obs); logits = actor head; masked logits
    -> -1e8 (distributions.py:16-28); log_prob = log_softmax gather, entropy =
    -sum p log(p + 1e-8) (torch_utils.py:142-199); value = critic head on the
    SAME latent (gradient flows into the shared encoder);
  * clipped surrogate + clipped value loss - entropy (:868-896), approx_kl
    (:899-902), zero_grad, backward, clip_grad_norm_(actor) then (critic)
    (:910-911), torch.optim.Adam step (optimizer_wrapper.py:444-452),
    mean_loss += loss.item();
  * target-KL early stop on the mean of every minibatch's approx_kl so far
    (:917-918); mean_loss / (num_samples * update_epochs) (:920).

Nothing here calls agilerl_amd: modules are plain nn.Linear / nn.LayerNorm /
nn.ReLU with the reference's module names, loaded from a reference-named
state dict (``actor.encoder.model.encoder_linear_layer_1.weight`` ...).
"""

from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn
from torch.nn.utils import clip_grad_norm_


def _mlp(name: str, fin: int, hidden: list[int], fout: int, *, out_ln: bool, out_act: bool) -> nn.Sequential:
    """create_mlp(..., layer_norm=True, output_layernorm=out_ln) module layout."""
    d: "OrderedDict[str, nn.Module]" = OrderedDict()
    dims = [fin, *hidden]
    for i in range(1, len(dims)):
        d[f"{name}_linear_layer_{i}"] = nn.Linear(dims[i - 1], dims[i])
        d[f"{name}_layer_norm_{i}"] = nn.LayerNorm(dims[i])
        d[f"{name}_activation_{i}"] = nn.ReLU()
    d[f"{name}_linear_layer_output"] = nn.Linear(dims[-1], fout)
    if out_ln:
        d[f"{name}_layer_norm_output"] = nn.LayerNorm(fout, elementwise_affine=False)
    d[f"{name}_activation_output"] = nn.ReLU() if out_act else nn.Identity()
    return nn.Sequential(d)


def reference_names(sd: dict) -> dict:
    """Key names as the reference's PPO state dict has them: the golden
    generator (tests/golden/gen_golden.py) names the actor's head MLP
    ``actor.head_net.model.*``; the reference wraps it (``head_net._wrapped``)."""
    return {(k.replace("actor.head_net.model.", "actor.head_net._wrapped.model.", 1)
             if k.startswith("actor.head_net.model.") else k): v for k, v in sd.items()}


class ActorCritic(nn.Module):
    """encoder [Linear-LN-ReLU]* -> Linear -> LN(plain) -> ReLU; actor head and
    critic ("value") head [Linear-LN-ReLU]* -> Linear."""

    def __init__(self, obs_dim: int, n_actions: int, enc_hidden: list[int], latent: int, actor_hidden: list[int],
                 critic_hidden: list[int]):
        super().__init__()
        self.encoder = _mlp("encoder", obs_dim, enc_hidden, latent, out_ln=True, out_act=True)
        self.actor_head = _mlp("actor", latent, actor_hidden, n_actions, out_ln=False, out_act=False)
        self.critic_head = _mlp("value", latent, critic_hidden, 1, out_ln=False, out_act=False)

    # reference state-dict prefixes of the three parts (the actor's head is an
    # EvolvableDistribution wrapping the MLP: head_net._wrapped, actors.py:330-336)
    PREFIX = {"encoder": "actor.encoder.model.", "actor_head": "actor.head_net._wrapped.model.",
              "critic_head": "critic.head_net.model."}

    def load_reference(self, sd: dict) -> None:
        sd = reference_names(sd)
        with torch.no_grad():
            for part, pre in self.PREFIX.items():
                mod = getattr(self, part)
                for k, t in mod.state_dict().items():
                    t.copy_(torch.as_tensor(np.asarray(sd[pre + k])))

    def reference_state(self) -> dict:
        out = {}
        for part, pre in self.PREFIX.items():
            for k, t in getattr(self, part).state_dict().items():
                out[pre + k] = t.detach().clone()
        return out

    def named_reference_params(self):
        for part, pre in self.PREFIX.items():
            for k, t in getattr(self, part).named_parameters():
                yield pre + k, t

    def evaluate(self, obs, actions, mask=None):
        lat = self.encoder(obs)
        logits = self.actor_head(lat)
        if mask is not None:
            logits = torch.where(mask, logits, torch.full_like(logits, -1e8))
        logp_all = torch.log_softmax(logits, dim=-1)
        logp = logp_all.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
        p = torch.softmax(logits, dim=-1)
        ent = -(p * torch.log(p + 1e-8)).sum(-1)
        value = self.critic_head(lat).squeeze(-1)
        return logp, ent, value


class _Norm(nn.Module):
    """preprocess_observation's image normalisation (algo_utils.py:1134-1183)."""

    def __init__(self, bounds):
        super().__init__()
        self.bounds = bounds

    def forward(self, x):
        x = x.float()
        if self.bounds is None:
            return x
        lo, hi = self.bounds
        return (x - lo) / (hi - lo)


class ImageActorCritic(ActorCritic):
    """The shared-encoder actor-critic for image spaces (ppo.py:286-320,
    base.py:521-530): EvolvableCNN encoder (cnn.py:224-552: Conv2d -> ReLU per
    layer, flatten, Linear -> ReLU) and create_mlp heads (layer_norm as given,
    output x0.1).  Plain nn.Conv2d modules with the reference's names
    (``{encoder}_conv_layer_{i}``, ``{encoder}_linear_output``)."""

    def __init__(self, obs_shape, n_actions: int, channels: list[int], kernels: list[int], strides: list[int],
                 latent: int, actor_hidden: list[int], critic_hidden: list[int], head_ln: bool = False,
                 norm=(0.0, 255.0), encoder_name: str = "shared_encoder"):
        nn.Module.__init__(self)
        c, h, w = obs_shape
        d: "OrderedDict[str, nn.Module]" = OrderedDict()
        for i, (co, k, st) in enumerate(zip(channels, kernels, strides), 1):
            d[f"{encoder_name}_conv_layer_{i}"] = nn.Conv2d(c, co, k, stride=st)
            d[f"{encoder_name}_activation_{i}"] = nn.ReLU()
            c, h, w = co, (h - k) // st + 1, (w - k) // st + 1
        d[f"{encoder_name}_flatten"] = nn.Flatten()
        d[f"{encoder_name}_linear_output"] = nn.Linear(c * h * w, latent)
        d[f"{encoder_name}_output_activation"] = nn.ReLU()
        self.encoder = nn.Sequential(d)
        self.norm = _Norm(norm)
        self.obs_shape = tuple(obs_shape)
        self.actor_head = _head_mlp("actor", latent, actor_hidden, n_actions, head_ln)
        self.critic_head = _head_mlp("value", latent, critic_hidden, 1, head_ln)

    def evaluate(self, obs, actions, mask=None):
        x = self.norm(obs.reshape(-1, *self.obs_shape))
        lat = self.encoder(x)
        logits = self.actor_head(lat)
        if mask is not None:
            logits = torch.where(mask, logits, torch.full_like(logits, -1e8))
        logp_all = torch.log_softmax(logits, dim=-1)
        logp = logp_all.gather(-1, actions.long().unsqueeze(-1)).squeeze(-1)
        p = torch.softmax(logits, dim=-1)
        ent = -(p * torch.log(p + 1e-8)).sum(-1)
        value = self.critic_head(lat).squeeze(-1)
        return logp, ent, value


def _head_mlp(name: str, fin: int, hidden: list[int], fout: int, ln: bool) -> nn.Sequential:
    d: "OrderedDict[str, nn.Module]" = OrderedDict()
    dims = [fin, *hidden]
    for i in range(1, len(dims)):
        d[f"{name}_linear_layer_{i}"] = nn.Linear(dims[i - 1], dims[i])
        if ln:
            d[f"{name}_layer_norm_{i}"] = nn.LayerNorm(dims[i])
        d[f"{name}_activation_{i}"] = nn.ReLU()
    d[f"{name}_linear_layer_output"] = nn.Linear(dims[-1], fout)
    d[f"{name}_activation_output"] = nn.Identity()
    return nn.Sequential(d)


def reference_learn(net: ActorCritic, adam_state: dict | None, obs, actions, old_logp, adv, ret, old_v,
                    perms, *, batch_size: int, epochs: int, clip: float = 0.2, vf: float = 0.5, ent: float = 0.01,
                    max_norm: float = 0.5, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                    target_kl: float | None = None, masks=None, dtype=torch.float32, on_update=None) -> dict:
    """One learn() of one agent.  ``adam_state``: {reference name: (exp_avg,
    exp_avg_sq)} plus "step" (None: a fresh optimizer).  Arrays are the
    flattened rollout [S, ...] in get_tensor_batch order; ``perms`` [E][S].
    Returns {"mean_loss", "approx_kl" (list), "epochs", "state", "exp_avg",
    "exp_avg_sq", "step"} (state dicts by reference name).  ``dtype``
    float64 runs the same algorithm in double precision (the network must be
    converted first): a measure of how far fp32 rounding alone moves the
    result, never a parity target.  ``on_update(k, snapshot)`` is called
    before update k with the state the update starts from (params,
    exp_avg, exp_avg_sq by reference name, step, the minibatch indices and
    the normalised advantages)."""
    names, params = zip(*net.named_reference_params())
    opt = torch.optim.Adam(list(params), lr=lr, betas=betas, eps=eps, foreach=False)
    if adam_state is not None and int(adam_state["step"]) > 0:
        for n_, p_ in zip(names, params):
            m, v = adam_state[n_]
            opt.state[p_] = {"step": torch.tensor(float(adam_state["step"])),
                             "exp_avg": torch.as_tensor(np.asarray(m)).clone().reshape(p_.shape),
                             "exp_avg_sq": torch.as_tensor(np.asarray(v)).clone().reshape(p_.shape)}
    actor_params = list(net.encoder.parameters()) + list(net.actor_head.parameters())
    critic_params = list(net.critic_head.parameters())
    t = lambda a: torch.as_tensor(np.asarray(a))  # noqa: E731
    obs, actions = t(obs), t(actions)
    if not isinstance(net, ImageActorCritic):  # image frames stay uint8 until the net normalises them
        obs = obs.to(dtype)
    old_logp, ret, old_v, adv = (t(x).to(dtype) for x in (old_logp, ret, old_v, adv))
    mask_t = None if masks is None else t(masks).bool()
    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    S = obs.shape[0]
    mean_loss = 0.0
    kls: list[float] = []
    ran = 0
    for e in range(epochs):
        idx_all = np.asarray(perms[e])
        for s0 in range(0, S, batch_size):
            idx = torch.as_tensor(idx_all[s0:min(s0 + batch_size, S)])
            if on_update is not None:
                on_update(len(kls), _snapshot(names, params, opt, idx, adv))
            logp, entropy, value = net.evaluate(obs[idx], actions[idx], None if mask_t is None else mask_t[idx])
            mb_adv, mb_old = adv[idx], old_logp[idx]
            ratio = torch.exp(logp - mb_old)
            pg = torch.max(-mb_adv * ratio, -mb_adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
            v_unc = (value - ret[idx]) ** 2
            v_clip = old_v[idx] + torch.clamp(value - old_v[idx], -clip, clip)
            v_loss = 0.5 * torch.max(v_unc, (v_clip - ret[idx]) ** 2).mean()
            loss = pg + vf * v_loss + ent * (-entropy.mean())
            with torch.no_grad():
                kls.append(((ratio - 1) - (logp - mb_old)).mean().item())
            opt.zero_grad()
            loss.backward()
            clip_grad_norm_(actor_params, max_norm)
            clip_grad_norm_(critic_params, max_norm)
            opt.step()
            mean_loss += loss.item()
        ran += 1
        if target_kl is not None and np.mean(kls) > target_kl:
            break
    mean_loss /= S * epochs
    state = net.reference_state()
    m_out, v_out = {}, {}
    step = 0
    for n_, p_ in zip(names, params):
        st = opt.state.get(p_, {})
        m_out[n_] = st["exp_avg"].clone() if st else torch.zeros_like(p_)
        v_out[n_] = st["exp_avg_sq"].clone() if st else torch.zeros_like(p_)
        step = int(st["step"]) if st else 0
    return {"mean_loss": mean_loss, "approx_kl": kls, "epochs": ran, "state": state, "exp_avg": m_out,
            "exp_avg_sq": v_out, "step": step}


def _snapshot(names, params, opt, idx, adv) -> dict:
    snap = {"state": {}, "exp_avg": {}, "exp_avg_sq": {}, "step": 0, "idx": idx.numpy().copy(),
            "adv_norm": adv.detach().numpy().copy()}
    for n_, p_ in zip(names, params):
        st = opt.state.get(p_, {})
        snap["state"][n_] = p_.detach().clone()
        snap["exp_avg"][n_] = st["exp_avg"].clone() if st else torch.zeros_like(p_)
        snap["exp_avg_sq"][n_] = st["exp_avg_sq"].clone() if st else torch.zeros_like(p_)
        snap["step"] = int(st["step"]) if st else 0
    return snap


def orthogonal_init_(net: ActorCritic, seed: int) -> None:
    """layer_init (evolvable_networks.py:410-441): orthogonal gain sqrt(2),
    zero bias; output layers x0.1 (output_vanish) — encoder output excluded."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for mod in (net.encoder, net.actor_head, net.critic_head):
            for name, m in mod.named_children():
                if isinstance(m, nn.Linear):
                    nn.init.orthogonal_(m.weight, math.sqrt(2), generator=g)
                    nn.init.zeros_(m.bias)
                    if name.endswith("linear_layer_output") and mod is not net.encoder:
                        m.weight.mul_(0.1)
