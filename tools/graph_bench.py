"""Time one learn() of the runtime-shape learner (agx_ppo_learn_graph) against
the compiled fused learner (same shape) and the PyTorch learner (mutated
shapes), config-2 sizes: P agents x 16 envs x learn_step 128 (S = 2048),
batch 128, 4 epochs.  Prints one JSON line."""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agilerl_amd.population.learner import FusedLearner, GraphLearner  # noqa: E402
from agilerl_amd.population.nets import ActorCriticSpec  # noqa: E402
from agilerl_amd.population.ppo_pop import PPOPopulation  # noqa: E402

DEV = torch.device("cuda:0")
P = int(os.environ.get("P", "8"))
REPS = int(os.environ.get("REPS", "5"))


def make(**kw):
    spec = ActorCriticSpec(obs_dim=8, n_actions=4, **kw)
    pop = PPOPopulation(spec, P, 16, learn_step=2048, batch_size=128, update_epochs=4, device=DEV, fused=True,
                        seeds=list(range(P)), perm_source="device")
    g = torch.Generator(device=DEV).manual_seed(0)
    pop.obs.copy_(torch.randn(pop.obs.shape, device=DEV, generator=g))
    pop.actions.copy_(torch.randint(0, 4, pop.actions.shape, device=DEV, generator=g))
    pop.rewards.copy_(torch.randn(pop.rewards.shape, device=DEV, generator=g))
    pop.values.copy_(torch.randn(pop.values.shape, device=DEV, generator=g))
    pop.log_probs.copy_(-torch.rand(pop.log_probs.shape, device=DEV, generator=g) - 0.5)
    pop.finish_rollout(torch.randn(P, 16, 8, device=DEV, generator=g), torch.zeros(P, 16, dtype=torch.uint8,
                                                                                   device=DEV))
    return pop


def timed(fn, reps=REPS):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / reps * 1e3, 3)


def main():
    out = {"P": P, "S": 2048, "batch": 128, "epochs": 4}
    pop = make()
    perms = pop.permutations()
    fl, gl = FusedLearner(pop), GraphLearner(pop)
    out["config2_fused_ms"] = timed(lambda: fl.learn(pop, perms))
    out["config2_graph_ms"] = timed(lambda: gl.learn(pop, perms))
    for name, kw in {"mutated_enc80_lat56_head2": dict(encoder_hidden=[80], latent_dim=56, actor_hidden=[64, 64]),
                     "mutated_wide": dict(encoder_hidden=[192], latent_dim=96, actor_hidden=[128], critic_hidden=[128])
                     }.items():
        pop = make(**kw)
        perms = pop.permutations()
        gl = GraphLearner(pop)
        out[name + "_graph_ms"] = timed(lambda: gl.learn(pop, perms))
        out[name + "_torch_ms"] = timed(lambda: pop._learn_torch(perms), reps=1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
