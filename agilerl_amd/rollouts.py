"""Drop-in ``collect_rollouts`` (agilerl/rollouts/on_policy.py:23-203) for an
agx PPO agent: fills the agent's HBM rollout from ``env`` (num_envs envs, or
num_envs x population_size for a population view) and computes the bootstrap
value + GAE, ready for ``agent.learn()``."""

from __future__ import annotations

from .population.runner import PopulationRunner


def collect_rollouts(agent, env, n_steps: int | None = None, last_obs=None, last_done=None, last_scores=None,
                     last_info=None, **_kwargs):
    """-> (completed episode scores, last_obs, last_done, last_scores,
    last_info) as the reference (episode scores of the envs that finished
    during this rollout; the runner carries the env state between calls, so
    the last_* values are returned for the caller's loop and not needed back)."""
    pop = agent.population
    if n_steps is not None and n_steps != pop.T:
        raise ValueError(f"n_steps must equal the rollout capacity ceil(learn_step / num_envs) = {pop.T}")
    runner = getattr(pop, "_runner", None)
    if runner is None or runner.env is not env:
        runner = PopulationRunner(pop, env)
        pop._runner = runner
    runner.reset_episode_stats()
    runner.collect()
    pop.finish_rollout(runner.last_obs, runner.last_done, runner.last_value if runner.last_value_valid else None)
    s = float(runner.episode_return_sum[agent.row].item())
    c = int(runner.episodes[agent.row].item())
    scores = [s / c] * c if c else []
    return scores, runner.last_obs, runner.last_done, None, None
