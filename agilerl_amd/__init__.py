"""agilerl_amd — MI355X-native (gfx950) hot path of a population-based RL
trainer, drop-in for the mcx/AgileRL hot path (GAE + PPO clipped loss,
prioritized-replay segment trees, DQN TD target, Rainbow C51 projection,
tournament selection with an RCCL fitness exchange).

The compute lives in libagx.so (HIP, C ABI: include/agx.h); this package is
the host side mirroring the reference's Python interfaces.
"""

import os as _os

__version__ = "0.1.0"

# Hardware queues per process.  The population engine gives every group of
# agents (network shape x learn_step) a stream of its own and paces their
# persistent rollouts together (population/engine.py); HIP maps streams onto
# GPU_MAX_HW_QUEUES hardware queues (HIP's default: 4), and a persistent
# launch holds its queue until it ends, so groups that share a queue run one
# after another.  8 queues: the 4-group train phase of a mutated ppo.yaml
# population took 24 instead of 31 ms per generation.  Read
# when the HIP runtime initialises, so this takes effect only when the
# package is imported before the first device call; AGX_HW_QUEUES overrides
# (0: leave the environment alone).
_q = int(_os.environ.get("AGX_HW_QUEUES", "8"))
if _q > 0 and int(_os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _q:
    _os.environ["GPU_MAX_HW_QUEUES"] = str(min(_q, 32))
