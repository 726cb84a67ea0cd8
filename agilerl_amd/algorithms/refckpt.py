"""Reading checkpoints the reference wrote, without executing anything from
the file.

The reference saves ``get_checkpoint_dict`` (agilerl/algorithms/core/
base.py:168-224) with ``torch.save(..., pickle_module=dill)`` (base.py:939-949)
and reads it back with ``torch.load(weights_only=False, pickle_module=dill)``
(base.py:951-960), which calls whatever classes and functions the pickle
names.  Here the file goes through torch's weights-only unpickler instead.
The globals a checkpoint names are listed first by
``torch.serialization.get_unsafe_globals_in_checkpoint`` (a static opcode
scan), and each one the unpickler does not already allow is bound to an
*inert stand-in*: a class with no behaviour that records the arguments and
state it is rebuilt with.  agilerl classes, gymnasium spaces, torch loss
modules, dill's type/function helpers all come back as stand-ins.  The real
callables added to the allow-list are numpy's array / scalar / dtype
reconstructors, so spaces' bounds and numpy scalars come back as numpy
values, and ``dill._dill._create_array`` is replaced by a function that
accepts only numpy's own array reconstructor.

``read_reference`` returns the checkpoint dict; ``to_agx`` turns it into the
layout ``algorithms/checkpoint.py`` reads (spaces as shapes, the
hyper-parameter attributes, ``network_info`` with the state dicts), so
``load_checkpoint`` / ``load`` take either file.
"""

from __future__ import annotations

import pickle
from typing import Any

import numpy as np
import torch


class Inert:
    """Stand-in for a class or function named in a checkpoint: built, never run."""

    qualname = "?"
    args: tuple = ()
    kwargs: dict = {}
    state: Any = None

    def __init__(self, *args, **kwargs) -> None:
        self.args, self.kwargs = args, kwargs

    def __setstate__(self, state) -> None:
        self.state = state

    def __repr__(self) -> str:
        return f"<inert {self.qualname}>"

    def attr(self, name: str, default=None):
        """An attribute of the object the stand-in replaces (its pickled state)."""
        st = self.state
        if isinstance(st, tuple) and len(st) == 2:  # (dict, slots)
            st = {**(st[0] or {}), **(st[1] or {})}
        return st.get(name, default) if isinstance(st, dict) else default


_STANDINS: dict[str, type] = {}


def _standin(name: str) -> type:
    cls = _STANDINS.get(name)
    if cls is None:
        mod, _, short = name.rpartition(".")
        cls = type(short or name, (Inert,), {"qualname": name, "__module__": "agx_inert." + mod})
        _STANDINS[name] = cls
    return cls


def _np_reconstruct_fn():
    core = getattr(np, "_core", None) or np.core
    return core.multiarray._reconstruct, core.multiarray.scalar


def _safe_create_array(f, args, state, npdict=None):
    """dill._dill._create_array (an ndarray subclass rebuild) restricted to
    numpy's own reconstructor; anything else stays inert."""
    reconstruct, _ = _np_reconstruct_fn()
    if f is not reconstruct:
        out = _standin("dill._dill._create_array")(f, args, state, npdict)
        return out
    arr = reconstruct(*args)
    arr.__setstate__(state)
    return arr


def _safe_load_type(name: str):
    """dill._dill._load_type (a builtin type by name, then called through
    REDUCE): an inert stand-in class, allow-listed for the rest of this load
    (the enclosing ``safe_globals`` context restores the list afterwards)."""
    cls = _standin(f"dill._dill.{name}")
    torch.serialization.add_safe_globals([(cls, cls.qualname)])
    return cls


def _numpy_globals() -> list:
    reconstruct, scalar = _np_reconstruct_fn()
    out = [np.dtype, np.ndarray]
    for mod in ("numpy.core.multiarray", "numpy._core.multiarray"):
        out += [(reconstruct, f"{mod}._reconstruct"), (scalar, f"{mod}.scalar")]
    out += [getattr(np.dtypes, n) for n in dir(np.dtypes) if n.endswith("DType")]
    out.append((_safe_create_array, "dill._dill._create_array"))
    out.append((_safe_load_type, "dill._dill._load_type"))
    return out


def read_reference(path: str) -> dict:
    """torch.load(weights_only=True) of a reference checkpoint with every
    unknown global bound to an inert stand-in."""
    allowed = _numpy_globals()
    known = {name for item in allowed if isinstance(item, tuple) for name in [item[1]]}
    known |= {f"{c.__module__}.{c.__qualname__}" for c in allowed if isinstance(c, type)}
    extra = [(_standin(n), n) for n in torch.serialization.get_unsafe_globals_in_checkpoint(path) if n not in known]
    before = list(torch.serialization.get_safe_globals())
    try:
        for _ in range(64):  # names the static scan could not see surface as UnpicklingError
            with torch.serialization.safe_globals(allowed + extra):
                try:
                    return torch.load(path, map_location="cpu", weights_only=True)
                except pickle.UnpicklingError as err:
                    name = _unsupported_global(str(err))
                    if name is None or name in {n for _, n in extra}:
                        raise
                    extra.append((_standin(name), name))
        raise pickle.UnpicklingError(f"{path}: too many unknown globals")
    finally:
        # the stand-ins _safe_load_type allow-listed during the load go again
        if set(torch.serialization.get_safe_globals()) != set(before):
            torch.serialization.clear_safe_globals()
            torch.serialization.add_safe_globals(before)


def _unsupported_global(msg: str) -> str | None:
    import re

    m = re.search(r"GLOBAL ([\w\.]+) was not an allowed global", msg)
    return m.group(1) if m else None


def is_reference_checkpoint(ck: dict) -> bool:
    return isinstance(ck, dict) and ck.get("agilerl_version") != "agx" and "network_info" in ck


def _space_shapes(ck: dict) -> dict | None:
    obs, act = ck.get("observation_space"), ck.get("action_space")
    if not isinstance(obs, Inert) or not isinstance(act, Inert):
        return None
    shape = obs.attr("_shape")
    n = act.attr("n")
    if shape is None or n is None:
        return None
    return {"obs_shape": [int(s) for s in shape], "n_actions": int(n)}


def _plain(v):
    if isinstance(v, np.generic):
        return v.item()
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    return v


def _adam_rows(opt_sd: dict, module_sds: list[dict]) -> dict:
    """A torch Adam state_dict over ``module_sds``' parameters in order (the
    reference's OptimizerWrapper, one param group per network,
    optimizer_wrapper.py:45-53) -> {"exp_avg": {name: t}, "exp_avg_sq":
    {name: t}, "step": int} keyed by each network's state-dict names."""
    state = opt_sd.get("state", {})
    ids = [i for g in opt_sd.get("param_groups", []) for i in g["params"]]
    names = [(net, k) for net, sd in module_sds for k in sd
             if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))]
    if len(ids) != len(names):
        raise ValueError(f"reference optimizer holds {len(ids)} parameters, the networks {len(names)}")
    m, v, step = {}, {}, 0
    for i, (net, k) in zip(ids, names):
        s = state.get(i)
        if not s:
            continue
        m[f"{net}.{k}"], v[f"{net}.{k}"] = s["exp_avg"], s["exp_avg_sq"]
        step = max(step, int(torch.as_tensor(s["step"]).item()))
    return {"exp_avg": m, "exp_avg_sq": v, "step": step}


def to_agx(ck: dict, adam_networks: tuple[str, ...] | None = None) -> dict:
    """The reference checkpoint in the layout algorithms/checkpoint.py
    reads.  ``adam_networks``: the networks one reference Adam covers, in
    its param-group order (PPO's ("actor", "critic"), ppo.py:329-333); its
    moments are re-keyed ``<net>.<param>`` as the agx PPO checkpoint holds
    them.  Other optimizers keep the reference's torch state_dict."""
    from .checkpoint import HP_NAMES

    out = {k: _plain(ck[k]) for k in HP_NAMES if k in ck and not isinstance(ck[k], Inert)}
    out["algo"] = ck.get("algo")
    out["agilerl_version"] = ck.get("agilerl_version")
    sp = _space_shapes(ck)
    if sp is not None:
        out["spaces"] = sp
    info = ck["network_info"]
    mods = {k: v for k, v in info["modules"].items() if k.endswith("_state_dict")}
    opts = {k: v for k, v in info["optimizers"].items() if k.endswith("_state_dict")}
    if adam_networks is not None and "optimizer_state_dict" in opts:
        sds = [(n, info["modules"][f"{n}_state_dict"]) for n in adam_networks]
        opts["optimizer_state_dict"] = _adam_rows(opts["optimizer_state_dict"], sds)
    out["network_info"] = {"network_names": list(info["network_names"]), "modules": mods,
                           "optimizer_names": list(info["optimizer_names"]), "optimizers": opts}
    for k in ("lr_actor", "lr_critic", "agent_ids"):
        if k in ck:
            out[k] = _plain(ck[k])
    return out
