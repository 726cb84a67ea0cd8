"""The EvolvableAlgorithm hooks the reference's Mutations call
(agilerl/algorithms/core/base.py:744-775, hpo/mutation.py:413-453, 515-570)
for the object-level agents (DQN, RainbowDQN, MADDPG):

* ``registry``            the agent's HyperparameterConfig (hpo/registry.py);
* ``get_lr_names``        the attributes that are learning rates;
* ``reinit_optimizers``   a fresh Adam at the current learning rate — all of
                          them, or only the one whose lr was mutated
                          (mutation.py:440-450 ``to_reinit``);
* ``policy_weight_groups``the eval network's state dict(s) (one per agent id
                          for a ModuleDict policy, mutation.py:543-547), whose
                          2-D entries parameter mutations perturb in place;
* ``sync_shared_networks``the policy group's shared networks load the mutated
                          policy (mutation.py:554-561: the target networks);
* ``mutation_hook``       registered hooks (none for these algorithms)."""

from __future__ import annotations

import torch

from ..modules.mlp import EvolvableMLP


class EvolvableAgentMixin:
    sharded = False  # set by create_population when the agent is one shard of a global population

    #: learning-rate attribute -> the optimizer attribute it drives
    _lr_optimizers: dict[str, str] = {"lr": "optimizer"}
    #: (eval network attribute, shared network attribute) of the policy group
    _policy_group: tuple[str, str] = ("actor", "actor_target")

    def _init_registry(self, hp_config) -> None:
        from ..hpo.registry import MutationRegistry

        self.hp_config = hp_config
        self.registry = MutationRegistry(hp_config)

    def get_lr_names(self) -> list[str]:
        return list(self._lr_optimizers)

    def _fresh_optimizer(self, lr_name: str):
        raise NotImplementedError

    @property
    def can_mutate_architecture(self) -> bool:
        """MLP-encoder Q networks (the encoder's and head's node / layer
        mutations and the latent's); CNN encoders and multi-agent ModuleDicts
        are not mutated."""
        if getattr(self, "sharded", False):
            # a population sharded over ranks replays every global agent's draws
            # on every rank (hpo/shard.py RemoteAgent); the module and init draws
            # of a Q-network mutation are not replayed: not applied anywhere.
            # The flag is set by create_population and, for agents built any
            # other way, by the entry points' sharded mutation / selection
            # steps (hpo/shard.py mark_sharded): the off-policy loops treat
            # every multi-rank run as one population split over the ranks.
            return False
        from ..modules.cnn import EvolvableCNN

        net = getattr(self, self._policy_group[0])
        return isinstance(getattr(net, "encoder", None), (EvolvableMLP, EvolvableCNN)) and \
            isinstance(getattr(net, "head_net", None), EvolvableMLP)

    def architecture_mutation(self, new_layer_prob: float, rng) -> str:
        """mutation.py:829-885 on the policy network: the method sampled from
        its mutation table with ``rng`` (Mutations.rng; the table of an
        EvolvableNetwork with an MLP encoder, population/arch.py, or a CNN
        encoder, population/image_arch.py), applied
        with the modules' own generators; the shared (target) network re-made
        from the mutated one (reinit_shared_networks, mutation.py:104-160)."""
        import copy

        net = getattr(self, self._policy_group[0])
        applied = net.apply_mutation(net.sample_mutation_method(new_layer_prob, rng))
        setattr(self, self._policy_group[1], copy.deepcopy(net))
        return applied

    def reinit_optimizers(self, optimizer=None) -> None:
        names = self.get_lr_names() if optimizer is None else [optimizer]
        for lr_name in names:
            setattr(self, self._lr_optimizers[lr_name], self._fresh_optimizer(lr_name))

    def policy_weight_groups(self) -> list[dict[str, torch.Tensor]]:
        net = getattr(self, self._policy_group[0])
        if isinstance(net, torch.nn.ModuleDict):
            return [m.state_dict() for m in net.values()]
        return [net.state_dict()]

    @torch.no_grad()
    def sync_shared_networks(self) -> None:
        net, shared = getattr(self, self._policy_group[0]), getattr(self, self._policy_group[1])
        if isinstance(net, torch.nn.ModuleDict):
            for k in net:
                shared[k].load_state_dict(net[k].state_dict(), strict=False)
        else:
            shared.load_state_dict(net.state_dict(), strict=False)

    def mutation_hook(self) -> None:
        pass
