"""``GroupAgentsWrapper`` (reference: ``rllib/env/wrappers/group_agents_wrapper.py``): agents of a
MultiAgentEnv grouped into super-agents that observe / act with tuples of their members' values
and receive the sum of their rewards -- the class behind ``MultiAgentEnv.with_agent_groups``."""
from ..multi_agent_env import _GroupedAgents as GroupAgentsWrapper

__all__ = ["GroupAgentsWrapper"]
