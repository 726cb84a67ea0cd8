from .train_on_policy import train_on_policy

__all__ = ["train_on_policy"]
