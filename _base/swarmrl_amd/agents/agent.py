"""
Parent class for agents (reference: swarmrl/agents/agent.py).
"""


class Agent:
    """Parent class for a SwarmRL agent."""

    _killed = False

    @property
    def kill_switch(self):
        return self._killed

    @kill_switch.setter
    def kill_switch(self, value):
        self._killed = value

    def supports_device(self) -> bool:
        return False

    def calc_action(self, colloids):
        raise NotImplementedError("Implemented in Child class.")

    def calc_reward(self, colloids, external_reward: float = 0.0) -> None:
        raise NotImplementedError("Implemented in Child class.")
