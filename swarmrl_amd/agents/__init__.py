from swarmrl_amd.agents import bechinger_models, dummy_models, lymburn_model
from swarmrl_amd.agents.actor_critic import ActorCriticAgent
from swarmrl_amd.agents.agent import Agent
from swarmrl_amd.agents.classical_agent import ClassicalAgent

__all__ = ["Agent", "ActorCriticAgent", "ClassicalAgent", "dummy_models", "bechinger_models",
           "lymburn_model"]
