from swarmrl_amd.value_functions.expected_returns import ExpectedReturns
from swarmrl_amd.value_functions.generalized_advantage_estimate import GAE

__all__ = ["GAE", "ExpectedReturns"]
