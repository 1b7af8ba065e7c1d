"""Replay buffers (reference: ``rllib/utils/replay_buffers``): uniform ring, prioritized
(sum-tree), FIFO and reservoir transition buffers, their multi-agent wrappers (independent /
lockstep, prioritized, mix-in), and the episode buffers of the new API stack."""
from . import utils
from .episode_replay_buffer import EpisodeReplayBuffer
from .multi_agent import (FifoReplayBuffer, MultiAgentMixInReplayBuffer, MultiAgentPrioritizedReplayBuffer,
                          MultiAgentReplayBuffer, PrioritizedEpisodeReplayBuffer, ReplayMode, ReservoirReplayBuffer,
                          StorageUnit)
from .replay_buffer import PrioritizedReplayBuffer, ReplayBuffer

__all__ = ["ReplayBuffer", "PrioritizedReplayBuffer", "EpisodeReplayBuffer", "FifoReplayBuffer",
           "ReservoirReplayBuffer", "MultiAgentReplayBuffer", "MultiAgentPrioritizedReplayBuffer",
           "MultiAgentMixInReplayBuffer", "PrioritizedEpisodeReplayBuffer", "ReplayMode", "StorageUnit", "utils"]
