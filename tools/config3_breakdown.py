"""Where the per-agent config-3 iteration (sample -> RainbowDQN.learn ->
update_priorities, bench.config3_leg's per_agent) spends its time: each
phase bracketed by synchronize, plus the whole iteration unbracketed.
Diagnostic only; MODE=trace runs just the unbracketed loop (for
rocprofv3 --kernel-trace: kernel launches and GPU time per iteration)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from agilerl_amd.algorithms import RainbowDQN  # noqa: E402
from agilerl_amd.algorithms.flat_state import flat_state  # noqa: E402
from agilerl_amd.components import PrioritizedReplayBuffer  # noqa: E402
from agilerl_amd.envs import Box, Discrete  # noqa: E402


def main():
    P, B, fill = 8, 64, 1 << 15
    dev = torch.device("cuda")
    obs_space, act_space = Box(0, 255, (4, 84, 84), dtype=np.uint8), Discrete(6)
    torch.manual_seed(0)
    agents = [RainbowDQN(obs_space, act_space, net_config=bench.CONFIG3_NET, batch_size=B, lr=1e-4, gamma=0.99,
                         tau=1e-3, v_min=-200.0, v_max=200.0, num_atoms=51) for _ in range(P)]
    memory = PrioritizedReplayBuffer(1_000_000, alpha=0.6)
    g = torch.Generator(device=dev).manual_seed(1)
    for c in range(0, fill, 4096):
        n = min(4096, fill - c)
        memory.add({"obs": torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g),
                    "action": torch.randint(0, 6, (n,), device=dev, generator=g),
                    "reward": torch.randn(n, device=dev, generator=g),
                    "next_obs": torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g),
                    "done": (torch.rand(n, device=dev, generator=g) < 0.02).float()})

    def iteration():
        for a in agents:
            s = memory.sample(B, beta=0.4)
            _, idxs, pri = a.learn(s, per=True)
            memory.update_priorities(idxs, pri)

    for _ in range(3):
        iteration()
    torch.cuda.synchronize()
    iters = int(os.environ.get("ITERS", 10))
    t0 = time.perf_counter()
    for _ in range(iters):
        iteration()
    torch.cuda.synchronize()
    whole = (time.perf_counter() - t0) / iters / P * 1e3
    print(f"whole: {whole:.3f} ms per agent-iteration", flush=True)
    if os.environ.get("MODE") == "trace":
        return

    sync = torch.cuda.synchronize
    acc = {}

    def tick(name, t):
        sync()
        now = time.perf_counter()
        acc[name] = acc.get(name, 0.0) + now - t
        return now

    a = agents[0]
    for _ in range(iters * P):
        t = time.perf_counter()
        s = memory.sample(B, beta=0.4)
        t = tick("sample", t)
        ex = [a._obs(s["obs"]), s["action"], s["reward"], a._obs(s["next_obs"]), s["done"]]
        t = tick("obs_norm", t)
        el = a._dqn_loss(*ex, a.gamma)
        t = tick("loss_fwd", t)
        loss = torch.mean(el * s["weights"])
        a.optimizer.zero_grad()
        loss.backward()
        t = tick("backward", t)
        fs = flat_state(a)
        t = tick("flat_state_check", t)
        fs.step(10.0)
        t = tick("clip_adam", t)
        fs.polyak(a.tau)
        t = tick("polyak", t)
        a.actor.reset_noise()
        a.actor_target.reset_noise()
        t = tick("reset_noise", t)
        pri = el.detach().cpu().numpy() + a.prior_eps
        loss.item()
        t = tick("to_host", t)
        memory.update_priorities(s["idxs"], pri)
        t = tick("update_priorities", t)
    n = iters * P
    tot = sum(acc.values())
    for k, v in acc.items():
        print(f"{k:18s} {v / n * 1e3:7.3f} ms", flush=True)
    print(f"{'sum (bracketed)':18s} {tot / n * 1e3:7.3f} ms", flush=True)
    print("params per agent:", len(list(a.actor.parameters())), flush=True)


if __name__ == "__main__":
    main()
