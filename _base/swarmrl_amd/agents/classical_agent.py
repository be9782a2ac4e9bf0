"""
Classical (non-learning) agents (reference: swarmrl/agents/classical_agent.py).

Deviation, documented in DESIGN.md: ``calc_reward`` is a no-op here.  The
reference inherits Agent.calc_reward, which raises NotImplementedError, yet
its own engine test drives ConstForce through integrate(), which calls
calc_reward after every chunk (espresso.py:1307); a no-op is the only
behaviour under which that test can run.
"""

from swarmrl_amd.agents.agent import Agent


class ClassicalAgent(Agent):
    def __init__(self, particle_type: int, actions: dict, task=None, observable=None):
        self.particle_type = particle_type
        self.task = task
        self.observable = observable
        self.actions = actions

    def calc_action(self, colloids):
        raise NotImplementedError("Implement in subclass")

    def calc_reward(self, colloids, external_reward: float = 0.0):
        return None
