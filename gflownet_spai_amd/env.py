"""Environment plugin interface (mirror of gflownet/env.py:3-38)."""
from abc import ABC, abstractmethod


class Env(ABC):
    """Signatures GFlowNet is generic over: ``update`` (state, actions) -> rewards,
    ``mask`` (state) -> allowed actions, ``reward`` (state) -> reward."""

    @abstractmethod
    def update(self, s, actions):
        ...

    @abstractmethod
    def mask(self, s):
        ...

    @abstractmethod
    def reward(self, s):
        ...
