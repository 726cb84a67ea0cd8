"""HPO mutations (agilerl_amd.hpo.mutation) against the reference's own
Mutations run (tests/golden/mut*.npz): the per-agent mutation choices, the
RL-hyperparameter values (shared HyperparameterConfig, torch-drawn sample and
grow / shrink), the optimizer re-initialisations, and the parameter-mutated
policy weights — bit for bit."""

import types

import numpy as np
import pytest
import torch

from agilerl_amd.hpo.mutation import Mutations
from agilerl_amd.hpo.registry import HyperparameterConfig, MutationRegistry, RLParameter


class _Agent:
    def __init__(self, i, weights, hp):
        self.index, self.batch_size, self.ent_coef, self.update_epochs = i, 128, 0.01, 4
        self.lr = 1e-3
        self.registry = MutationRegistry(hp)
        self.w = {k: torch.tensor(v) for k, v in weights.items()}
        self.mut, self.reinits = None, 0

    def get_lr_names(self):
        return ["lr"]

    def reinit_optimizers(self, optimizer=None):
        self.reinits += 1

    def policy_weights(self):
        return self.w

    def mutation_hook(self):
        pass


@pytest.mark.parametrize("case", ["mut0", "mut1"])
def test_mutations_match_reference(golden, case):
    g = golden(case)
    P = int(g["P"])
    hp = HyperparameterConfig(lr=RLParameter(min=1e-4, max=1e-2), batch_size=RLParameter(min=8, max=1024, dtype=int),
                              ent_coef=RLParameter(min=0.001, max=0.1),
                              update_epochs=RLParameter(min=1, max=10, dtype=int))
    pop = []
    for i in range(P):
        pre = f"init.a{i}."
        pop.append(_Agent(i, {k[len(pre):]: g[k] for k in g if k.startswith(pre)}, hp))
    no, arch, par, act, rlhp = (float(x) for x in g["probs"])
    m = Mutations(no_mutation=no, architecture=arch, new_layer_prob=0.2, parameters=par, activation=act,
                  rl_hp=rlhp, mutation_sd=0.1, mutate_elite=bool(g["mutate_elite"]), rand_seed=int(g["seed"]))
    for gen in range(int(g["generations"])):
        pop = m.mutation(pop)
        assert [a.mut for a in pop] == list(g["muts"][gen]), gen
        got = np.array([[a.lr, a.batch_size, a.ent_coef, a.update_epochs, a.reinits] for a in pop], np.float64)
        np.testing.assert_array_equal(got, g["hps"][gen])
    for i, a in enumerate(pop):
        pre = f"final.a{i}."
        for k in (k for k in g if k.startswith(pre)):
            assert np.array_equal(a.w[k[len(pre):]].numpy(), g[k]), (i, k)


def test_rlparameter_bounds_and_dtype():
    torch.manual_seed(0)
    p = RLParameter(min=8, max=16, dtype=int)
    p.value = 15
    seen = {p.mutate() for _ in range(40)}
    assert all(isinstance(v, int) and 8 <= v <= 16 for v in seen)
    assert not HyperparameterConfig()
    with pytest.raises(TypeError):
        HyperparameterConfig(lr=1e-3)


def test_no_hp_config_is_no_mutation():
    a = types.SimpleNamespace(registry=MutationRegistry(None), mut=None)
    m = Mutations(0, 0, 0, 0, 0, 1, rand_seed=1)
    assert m.rl_hyperparam_mutation(a).mut == "None"
