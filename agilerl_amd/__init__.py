"""agilerl_amd — MI355X-native (gfx950) hot path of a population-based RL
trainer, drop-in for the mcx/AgileRL hot path (GAE + PPO clipped loss,
prioritized-replay segment trees, DQN TD target, Rainbow C51 projection,
tournament selection with an RCCL fitness exchange).

The compute lives in libagx.so (HIP, C ABI: include/agx.h); this package is
the host side mirroring the reference's Python interfaces.
"""

__version__ = "0.1.0"
