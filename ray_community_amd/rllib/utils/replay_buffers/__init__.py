"""Replay buffers (reference: ``rllib/utils/replay_buffers``): uniform ring and prioritized
(sum-tree) transition buffers, and the episode buffer of the new API stack."""
from .episode_replay_buffer import EpisodeReplayBuffer
from .replay_buffer import PrioritizedReplayBuffer, ReplayBuffer

__all__ = ["ReplayBuffer", "PrioritizedReplayBuffer", "EpisodeReplayBuffer"]
