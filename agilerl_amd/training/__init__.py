from .train_multi_agent_off_policy import train_multi_agent_off_policy
from .train_off_policy import train_off_policy
from .train_on_policy import train_on_policy

__all__ = ["train_on_policy", "train_off_policy", "train_multi_agent_off_policy"]
