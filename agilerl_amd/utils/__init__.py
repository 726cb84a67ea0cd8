"""create_population (agilerl/utils/utils.py:347-): P agents of one algorithm.

For PPO the agents are views of ONE HBM-resident PPOPopulation (stacked
parameters / Adam state / rollout SoA), so a whole population is trained with
one launch per kernel; the INIT_HP keys and defaults follow the reference
(utils.py:502-537).

Sharding.  Under an initialised torch.distributed group of G > 1 ranks
(``shard=None``, the default, or ``shard=True``) ``population_size`` is the
GLOBAL population and each rank gets its slice: rank r holds global agents
r*P .. r*P + P - 1 with P = population_size / G (their global indices, init
seeds and sampling streams), so the same script trains the same population
on 1 or G GPUs.  Object-level agents (DQN / Rainbow / MADDPG) are built for
the whole population in order and the slice is kept, which leaves the
torch generators where the unsharded build leaves them.  ``shard=False``
keeps ``population_size`` agents per rank."""

from __future__ import annotations

from typing import Any

import torch


def create_population(algo: str, net_config: dict[str, Any] | None, INIT_HP: dict[str, Any], observation_space=None,
                      action_space=None, hp_config=None, actor_network=None, critic_network=None,
                      agent_wrapper=None, wrapper_kwargs=None, population_size: int = 1, num_envs: int = 1,
                      device="cuda", accelerator=None, torch_compiler=None, algo_kwargs=None, shard=None, **_unused):
    algo_kwargs = dict(algo_kwargs or {})
    import torch.distributed as dist

    world, rank = (dist.get_world_size(), dist.get_rank()) if dist.is_initialized() else (1, 0)
    if shard is None:
        shard = world > 1
    from ..hpo.shard import mark_shared

    mark_shared(hp_config)  # one config object for every agent, as the reference hands it out
    lo, P = 0, int(population_size)
    if shard and world > 1:
        if population_size % world:
            raise ValueError(f"population_size {population_size} is not divisible by the {world} ranks")
        P = population_size // world
        lo = rank * P
    if algo == "PPO":
        from ..algorithms.ppo import PPO, spec_from_net_config
        from ..population.ppo_pop import PPOPopulation

        if actor_network is not None or critic_network is not None:
            raise NotImplementedError("custom actor/critic modules: use net_config (MLP) networks")
        hp = dict(batch_size=INIT_HP.get("BATCH_SIZE", 64), lr=INIT_HP.get("LR", 0.0001),
                  learn_step=INIT_HP.get("LEARN_STEP", 2048), gamma=INIT_HP.get("GAMMA", 0.99),
                  gae_lambda=INIT_HP.get("GAE_LAMBDA", 0.95), clip_coef=INIT_HP.get("CLIP_COEF", 0.2),
                  ent_coef=INIT_HP.get("ENT_COEF", 0.01), vf_coef=INIT_HP.get("VF_COEF", 0.5),
                  max_grad_norm=INIT_HP.get("MAX_GRAD_NORM", 0.5), target_kl=INIT_HP.get("TARGET_KL"),
                  update_epochs=INIT_HP.get("UPDATE_EPOCHS", 4))
        if INIT_HP.get("RECURRENT", False):
            raise NotImplementedError("recurrent PPO is outside the agx hot path")
        spec = spec_from_net_config(observation_space, action_space, net_config,
                                    share_encoders=bool(algo_kwargs.get("share_encoders", True)))
        G = population_size if shard and world > 1 else P
        pop = PPOPopulation(spec, P, num_envs, seeds=list(range(lo, lo + P)), device=torch.device(device),
                            agent_offset=lo, global_pop_size=G, seed_base=0, **hp)
        return [PPO(observation_space, action_space, index=lo + i, hp_config=hp_config, net_config=net_config,
                    num_envs=num_envs, device=device, _population=pop, _row=i, **hp, **algo_kwargs)
                for i in range(P)]
    if algo in ("DQN", "Rainbow DQN", "RainbowDQN"):
        from ..algorithms.dqn import DQN, RainbowDQN

        cls = DQN if algo == "DQN" else RainbowDQN
        agents = [cls.from_init_hp(observation_space, action_space, net_config, INIT_HP, index=i, device=device,
                                   hp_config=hp_config, **algo_kwargs)
                  for i in range(population_size if shard else P)]
        for a in agents:
            a.sharded = bool(shard and world > 1)
        return agents[lo:lo + P]
    if algo == "MADDPG":  # utils/utils.py:590-618
        from ..algorithms.maddpg import MADDPG

        hp = dict(batch_size=INIT_HP.get("BATCH_SIZE", 64), lr_actor=INIT_HP.get("LR_ACTOR", 0.0001),
                  lr_critic=INIT_HP.get("LR_CRITIC", 0.001), learn_step=INIT_HP.get("LEARN_STEP", 5),
                  gamma=INIT_HP.get("GAMMA", 0.95), tau=INIT_HP.get("TAU", 0.01),
                  O_U_noise=INIT_HP.get("O_U_NOISE", True), expl_noise=INIT_HP.get("EXPL_NOISE", 0.1),
                  vect_noise_dim=num_envs, mean_noise=INIT_HP.get("MEAN_NOISE", 0.0),
                  theta=INIT_HP.get("THETA", 0.15), dt=INIT_HP.get("DT", 0.01))
        agents = [MADDPG(observation_space, action_space, agent_ids=INIT_HP["AGENT_IDS"], index=i,
                         net_config=net_config, device=device, hp_config=hp_config, **hp, **algo_kwargs)
                  for i in range(population_size if shard else P)]
        for a in agents:
            a.sharded = bool(shard and world > 1)
        return agents[lo:lo + P]
    raise NotImplementedError(f"algorithm {algo!r} is outside the agx hot path (PPO, DQN, Rainbow DQN, MADDPG)")


__all__ = ["create_population"]
