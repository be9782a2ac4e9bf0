from swarmrl_amd.agents import bechinger_models, dummy_models, lymburn_model
from swarmrl_amd.agents.actor_critic import ActorCriticAgent
from swarmrl_amd.agents.agent import Agent
from swarmrl_amd.agents.classical_agent import ClassicalAgent
from swarmrl_amd.agents.find_point import FindPoint

__all__ = ["Agent", "ActorCriticAgent", "ClassicalAgent", "FindPoint", "dummy_models",
           "bechinger_models", "lymburn_model"]
