"""Drop-in ``Mutations`` (agilerl/hpo/mutation.py:80-827) for populations
whose networks live in HBM.

What runs, with the reference's draws from the reference's generators:

* ``mutation(population)`` (:311-365): one choice per agent from
  ``self.rng.choice(options, len(population), p=proba)`` (numpy PCG64 seeded
  by ``rand_seed``); ``mutate_elite=False`` forces no mutation on the first
  (elite) slot;
* ``rl_hyperparam_mutation`` (:413-453): ``hp_config.sample()`` and
  ``RLParameter.mutate()`` (global torch generator, hpo/registry.py), the new
  value set on the agent; a mutated learning rate re-initialises that agent's
  optimizer (fresh Adam).  On a PPO population the value lands in the
  population's per-agent hyperparameter table, so the fused learner trains
  every agent with its own lr / batch size / epochs / entropy coefficient;
* ``parameter_mutation`` (:515-565 -> _gaussian_parameter_mutation
  :733-827): on the policy's 2-D weight matrices, the chosen keys, entries and
  the normal / super / reset noise drawn exactly as the reference draws them
  (self.rng, then torch.normal on the CPU generator); each chosen matrix
  (a few KB) is updated on the host with the reference's CPU indexing
  semantics and copied back to its HBM row.

* ``architecture_mutate`` (:373-411, :829-885) on PPO agents: the method
  sampled from the actor's mutation table with ``self.rng``, applied to the
  actor, the applied method to the critic, shared encoder, fresh optimizer
  (population/arch.py, bit-exact against the reference's own networks); the
  population engine regroups agents by network shape;
* ``learn_step`` as an RL hyperparameter: the agent's rollout length, applied
  by the engine at the next generation (agents grouped by learn_step).

* ``activation_mutation`` (:457-513, _permutate_activation :710-731) on DQN /
  Rainbow agents: the new activation drawn with ``self.rng`` from
  ``activation_selection`` minus the current one, every evolvable module of
  the Q network recreated with it (the encoder's output activation too), the
  target network re-made from the mutated network (reinit_shared_networks,
  :104-160) and fresh optimizers.  Policy-gradient algorithms (PPO, MADDPG)
  keep their activations, as the reference's :469-479.

* ``architecture_mutate`` on PPO agents with CNN encoders (config 5):
  population/image_arch.py on the flat rows, the CNN table (encoder channel /
  kernel methods; its LAYER methods disabled), bit-exact against the
  reference's own networks; the engine regroups them as the MLP agents.

* ``architecture_mutate`` on DQN / Rainbow agents with MLP or CNN encoders:
  the method from the network's table (head layer / node, latent node, and
  the encoder's node methods: MLP nodes or CNN channels / kernels), applied
  to the Q network with the network's generator, the target network re-made
  from it, fresh optimizers (modules/cnn.py bit-exact per method).

* ``architecture_mutate`` on MADDPG (config 4): _architecture_mutate_multi
  (:887-1011) in algorithms/maddpg.py — the actors' ModuleDict table, the
  applied method on every actor that has it, the analogous method on every
  critic, targets re-made; bit-exact against the reference's own networks.

Not applied: architecture / activation mutations of DQN / Rainbow / MADDPG
agents in a population sharded over ranks (the modules' draws are not
replayed on the other ranks; recorded as no mutation with a warning, on
every rank alike).
"""

from __future__ import annotations

import random
import warnings

import numpy as np
import torch


def set_global_seed(seed: int | None) -> None:
    """mutation.py:41-54.  The reference also seeds fastrand there; fastrand
    is not installed, and nothing on this path draws from it (the reference
    only seeds it: the architecture mutations draw from Mutations.rng, the
    modules' numpy generators and torch's global generator, all seeded or
    replayed here)."""
    if seed is None:
        return
    np.random.seed(seed)
    torch.manual_seed(seed)
    random.seed(seed)


class Mutations:
    def __init__(self, no_mutation: float, architecture: float, new_layer_prob: float, parameters: float,
                 activation: float, rl_hp: float, mutation_sd: float = 0.1, activation_selection=None,
                 mutate_elite: bool = True, rand_seed: int | None = None, device="cpu", accelerator=None) -> None:
        for name, v in (("no mutation", no_mutation), ("architecture mutation", architecture),
                        ("parameters mutation", parameters), ("activation mutation", activation),
                        ("reinforcement learning hyperparameter mutation", rl_hp)):
            assert isinstance(v, (float, int)), f"Probability of {name} must be a float or integer."
            assert v >= 0, f"Probability of {name} must be greater than or equal to zero."
        assert 1 >= new_layer_prob >= 0, \
            "Probability of new layer architecture mutation must be between zero and one (inclusive)."
        assert mutation_sd >= 0, "Mutation strength must be greater than or equal to zero."
        assert isinstance(mutate_elite, bool), "Mutate elite must be boolean value True or False."
        assert isinstance(rand_seed, int) or rand_seed is None, "Random seed must be an integer or None."
        set_global_seed(rand_seed)
        self.rng = np.random.default_rng(rand_seed)
        self.no_mut, self.architecture_mut, self.new_layer_prob = no_mutation, architecture, new_layer_prob
        self.parameters_mut, self.activation_mut, self.rl_hp_mut = parameters, activation, rl_hp
        self.activation_selection = activation_selection or ["ReLU", "ELU", "GELU"]
        self.mutation_sd, self.mutate_elite, self.device = mutation_sd, mutate_elite, device
        self.pretraining_mut_options, self.pretraining_mut_proba = self._get_mutations_options(pretraining=True)
        self.mut_options, self.mut_proba = self._get_mutations_options()

    def _get_mutations_options(self, pretraining: bool = False):
        """mutation.py:572-606."""
        opts = [(self.no_mutation, self.no_mut), (self.architecture_mutate, self.architecture_mut),
                (self.parameter_mutation, self.parameters_mut), (self.activation_mutation, self.activation_mut),
                (self.rl_hyperparam_mutation, self.rl_hp_mut)]
        if pretraining:
            opts[0] = (self.no_mutation, 0)
        opts = [(f, p) for f, p in opts if p > 0]
        if not opts:
            opts = [(self.no_mutation, 1)]
        funcs, proba = zip(*opts)
        proba = np.array(proba) / np.sum(proba)
        return funcs, proba

    # ------------------------------------------------------------------ #
    def mutation(self, population, pre_training_mut: bool = False):
        """mutation.py:311-365."""
        options = self.pretraining_mut_options if pre_training_mut else self.mut_options
        proba = self.pretraining_mut_proba if pre_training_mut else self.mut_proba
        choice = self.rng.choice(options, len(population), p=proba)
        if not self.mutate_elite:
            choice[0] = self.no_mutation
        out = []
        for fn, individual in zip(choice, population):
            individual = fn(individual)
            hook = getattr(individual, "mutation_hook", None)
            if hook is not None:
                hook()
            out.append(individual)
        return out

    def no_mutation(self, individual):
        individual.mut = "None"
        return individual

    def _not_applied(self, individual, what: str):
        warnings.warn(f"agx Mutations: {what} mutations are not applied to this agent (a population sharded "
                      "over ranks, or a network without evolvable modules); recorded as no mutation", stacklevel=3)
        individual.mut = "None"
        return individual

    def architecture_mutate(self, individual):
        """mutation.py:373-411 -> _architecture_mutate_single (:829-885) for
        individuals that can change shape (PPO views: population/arch.py — the
        method sampled from the actor's table with self.rng, applied to the
        actor, the applied method to the critic, the shared encoder, then
        mutation_hook and a fresh optimizer; CNN-encoder PPO agents:
        population/image_arch.py; DQN / Rainbow with MLP or CNN encoders:
        algorithms/evolvable.py, the target re-made from the mutated network;
        MADDPG: _architecture_mutate_multi in algorithms/maddpg.py).  Sharded
        object-level populations: not applied."""
        fn = getattr(individual, "architecture_mutation", None)
        if fn is None or not getattr(individual, "can_mutate_architecture", False):
            return self._not_applied(individual, "architecture")
        applied = fn(self.new_layer_prob, self.rng)
        individual.mutation_hook()
        individual.reinit_optimizers()
        individual.mut = applied or "None"
        return individual

    def activation_mutation(self, individual):
        if getattr(individual, "algo", None) in ("PPO", "DDPG", "TD3", "IPPO", "MADDPG", "MATD3", "GRPO"):
            # mutation.py:469-479: policy-gradient algorithms keep their activations
            warnings.warn(f"Activation mutations are not supported for {individual.algo}.", stacklevel=2)
            individual.mut = "None"
            return individual
        net = getattr(individual, "actor", None)
        if net is None or not hasattr(net, "change_activation") or getattr(individual, "sharded", False):
            # populations sharded over ranks: the recreated modules' draws are not
            # replayed on the other ranks (hpo/shard.py), so no rank applies it
            return self._not_applied(individual, "activation")
        if net.activation is None:  # :489-499
            warnings.warn("Found no activation mutation capabilities. We advise setting the probability to "
                          "0.0 to disable activation mutations.", stacklevel=2)
            individual.mut = "None"
            return individual
        options = list(self.activation_selection)  # _permutate_activation (:710-731)
        if len(options) > 1 and net.activation in options:
            options.remove(net.activation)
        net.change_activation(str(self.rng.choice(options, size=1)[0]), output=False)
        individual.reinit_optimizers()
        individual.mut = "act"
        # reinit_shared_networks (:104-160): the target network re-made from the
        # mutated evaluation network (its modules and weights)
        if hasattr(individual, "actor_target"):
            import copy

            individual.actor_target = copy.deepcopy(individual.actor)
        return individual

    def rl_hyperparam_mutation(self, individual):
        """mutation.py:413-453."""
        registry = getattr(individual, "registry", None)
        hp_config = getattr(registry, "hp_config", None)
        if not hp_config:
            individual.mut = "None"
            return individual
        attr, spec = hp_config.sample()
        if spec.value is None:
            spec.value = getattr(individual, attr)
        new_value = spec.mutate()
        try:
            setattr(individual, attr, new_value)
        except NotImplementedError as err:
            warnings.warn(f"agx Mutations: {attr} not applied ({err})", stacklevel=2)
            individual.mut = "None"
            return individual
        if attr in individual.get_lr_names():  # a new lr: fresh optimizer for it (:440-450)
            individual.reinit_optimizers(attr)
        individual.mut = attr
        return individual

    def parameter_mutation(self, individual):
        """mutation.py:515-570: _gaussian_parameter_mutation (:733-827) on the
        policy's 2-D weight matrices — one network, or each agent's network of
        a ModuleDict policy in turn (``policy_weight_groups``); then the policy
        group's shared networks load the mutated policy and the optimizers are
        re-initialised."""
        groups = individual.policy_weight_groups() if hasattr(individual, "policy_weight_groups") \
            else [individual.policy_weights()]
        for weights in groups:
            self._gaussian_parameter_mutation(weights)
        if hasattr(individual, "sync_shared_networks"):
            individual.sync_shared_networks()
        individual.reinit_optimizers()  # :567
        individual.mut = "param"
        return individual

    def _gaussian_parameter_mutation(self, weights: dict) -> None:
        """mutation.py:733-827 on ``weights`` (reference state-dict name ->
        device tensor, in state-dict order): the chosen keys, entries and the
        normal / super / reset noise drawn as a CPU-device reference agent
        draws them (self.rng, then torch.normal on the global CPU generator);
        each chosen matrix is updated on the host with the reference's CPU
        indexing semantics and copied back in place."""
        potential = [k for k, w in weights.items() if w.dim() == 2 and "lstm" not in k and "norm" not in k]
        if not potential:
            return
        mut_strength, frac, super_strength, super_prob = self.mutation_sd, 0.1, 10, 0.05
        reset_prob, mag_limit = super_prob + 0.05, 1000000
        how_many = int(self.rng.integers(1, len(potential) + 1))
        chosen = self.rng.choice(potential, how_many, replace=False)
        with torch.no_grad():
            for key in chosen:
                W_dev = weights[key]
                W = W_dev.cpu()  # one small matrix: the update runs with CPU index semantics, as the reference's
                n = W.shape[0] * W.shape[1]
                num = int(np.ceil(frac * n))
                if num < 1:
                    continue
                rows = self.rng.integers(0, W.shape[0], size=num)
                cols = self.rng.integers(0, W.shape[1], size=num)
                rand_vals = self.rng.uniform(0, 1, size=num)
                r_t, c_t = torch.tensor(rows, dtype=torch.long), torch.tensor(cols, dtype=torch.long)
                rv = torch.tensor(rand_vals, dtype=W.dtype)
                cur = W[r_t, c_t]
                new = cur.clone()
                m_super = rv < super_prob
                m_reset = (rv >= super_prob) & (rv < reset_prob)
                m_norm = rv >= reset_prob
                if m_super.sum() > 0:
                    std = (super_strength * cur[m_super]).abs()
                    new[m_super] = cur[m_super] + torch.normal(mean=torch.zeros_like(std), std=std)
                if m_reset.sum() > 0:
                    k = int(m_reset.sum())
                    new[m_reset] = torch.normal(mean=torch.zeros(k), std=torch.ones(k))
                if m_norm.sum() > 0:
                    std = (mut_strength * cur[m_norm]).abs()
                    new[m_norm] = cur[m_norm] + torch.normal(mean=torch.zeros_like(std), std=std)
                new = new.clamp(min=-mag_limit, max=mag_limit)
                W[r_t, c_t] = new
                W_dev.copy_(W)
