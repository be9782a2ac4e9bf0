from swarmrl_amd.agents import dummy_models
from swarmrl_amd.agents.actor_critic import ActorCriticAgent
from swarmrl_amd.agents.agent import Agent
from swarmrl_amd.agents.classical_agent import ClassicalAgent

__all__ = ["Agent", "ActorCriticAgent", "ClassicalAgent", "dummy_models"]
