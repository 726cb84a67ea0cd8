"""Checkpoints in the layout of ``get_checkpoint_dict`` (agilerl/algorithms/
core/base.py:168-224, 939-1072): hyper-parameter attributes at the top level
plus ``network_info = {network_names, modules: {<net>_state_dict},
optimizer_names, optimizers: {<opt>_state_dict}}``, with the reference's
state-dict key names.

Differences of form: classes and spaces are not pickled (the file holds only
tensors, numbers, strings, lists and dicts), so it is written by
``torch.save`` and read back with ``torch.load(weights_only=True)`` — nothing
in a checkpoint is executed on load.  Spaces are stored as
``{"obs_shape", "n_actions"}`` for ``load``.

Checkpoints the reference itself wrote (dill-pickled agents, spaces and
registries) are read by ``refckpt.read_reference`` — the same weights-only
unpickler with inert stand-ins for the classes they name — and converted to
this layout, so ``load_checkpoint`` / ``load`` accept either file.
"""

from __future__ import annotations

import pickle
from typing import Any

import torch

HP_NAMES = ("index", "batch_size", "lr", "learn_step", "gamma", "tau", "double", "beta", "prior_eps", "num_atoms",
            "v_min", "v_max", "noise_std", "n_step", "combined_reward", "gae_lambda", "clip_coef", "ent_coef",
            "vf_coef", "max_grad_norm", "target_kl", "update_epochs", "num_envs", "net_config", "scores", "fitness",
            "steps", "mut", "normalize_images")


def _plain(v: Any) -> Any:
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().clone()
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    if hasattr(v, "item") and callable(v.item) and not isinstance(v, (str, bytes)):
        return v.item()
    return v


def checkpoint_dict(agent, modules: dict[str, dict[str, torch.Tensor]], optimizers: dict[str, Any],
                    spaces: bool = True) -> dict:
    out = {k: _plain(getattr(agent, k)) for k in HP_NAMES if hasattr(agent, k)}
    out["algo"] = agent.algo
    out["agilerl_version"] = "agx"
    if spaces:
        out["spaces"] = {"obs_shape": list(agent.observation_space.shape), "n_actions": int(agent.action_space.n)}
    out["network_info"] = {
        "network_names": list(modules),
        "modules": {f"{k}_state_dict": _plain(v) for k, v in modules.items()},
        "optimizer_names": list(optimizers),
        "optimizers": {f"{k}_state_dict": _plain(v) for k, v in optimizers.items()},
    }
    return out


def load_file(path: str, adam_networks: tuple[str, ...] | None = None) -> dict:
    """An agx checkpoint as written, or a reference one converted to the agx
    layout (refckpt.to_agx; ``adam_networks`` as there)."""
    from . import refckpt

    try:
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
    except pickle.UnpicklingError:
        ckpt = refckpt.read_reference(path)
    if isinstance(ckpt, dict) and ckpt.get("agilerl_version") == "agx":
        return ckpt
    if not refckpt.is_reference_checkpoint(ckpt):
        raise ValueError(f"{path}: not an agent checkpoint of agilerl >= 2.0 (no network_info)")
    return refckpt.to_agx(ckpt, adam_networks)


def read(path: str, algo: str, adam_networks: tuple[str, ...] | None = None) -> dict:
    ckpt = load_file(path, adam_networks)
    if ckpt.get("algo") != algo:
        raise ValueError("Loaded registry does not match the algorithm's registry. Please make sure you are "
                         "loading the checkpoint with the correct algorithm.")
    return ckpt


def restore_attributes(agent, ckpt: dict) -> None:
    for k in HP_NAMES:
        if k in ckpt:
            setattr(agent, k, ckpt[k])


def spaces(ckpt: dict):
    from ..envs import Box, Discrete

    s = ckpt["spaces"]
    return Box(-float("inf"), float("inf"), tuple(s["obs_shape"])), Discrete(s["n_actions"])


class TorchCheckpointMixin:
    """save_checkpoint / load_checkpoint / load for algorithms whose networks
    are torch modules ``actor`` / ``actor_target`` with one ``optimizer``."""

    def save_checkpoint(self, path: str) -> None:
        torch.save(checkpoint_dict(self, {"actor": self.actor.state_dict(),
                                          "actor_target": self.actor_target.state_dict()},
                                   {"optimizer": self.optimizer.state_dict()}), path)

    @torch.no_grad()
    def load_checkpoint(self, path: str) -> None:
        ck = read(path, self.algo)
        info = ck["network_info"]
        for name in ("actor", "actor_target"):
            sd = info["modules"].get(f"{name}_state_dict")
            if sd:  # an empty state dict is skipped, as the reference (core/base.py:1010)
                getattr(self, name).load_state_dict(sd)
        self.optimizer.load_state_dict(info["optimizers"]["optimizer_state_dict"])
        restore_attributes(self, ck)

    @classmethod
    def load(cls, path: str, device="cuda", accelerator=None):
        ck = load_file(path)
        obs_space, act_space = spaces(ck)
        code = cls.__init__.__code__
        names = set(code.co_varnames[1:code.co_argcount])
        agent = cls(obs_space, act_space, device=device, **{k: ck[k] for k in names if k in ck})
        agent.load_checkpoint(path)
        return agent
