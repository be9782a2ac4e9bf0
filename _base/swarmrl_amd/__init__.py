"""
swarmrl_amd -- MI355X-native engine for SwarmRL's rollout hot path.

Drop-in for swarmrl.engine.espresso (EspressoMD / MDParams) and the Colloid,
Action, ForceFunction, observable and task APIs on the path; the physics and
the observable reductions run in hand-written HIP (csrc/), the policy in
PyTorch-ROCm.  See DESIGN.md.
"""

import logging

from swarmrl_amd import (  # noqa: F401
    actions,
    agents,
    components,
    exploration_policies,
    force_functions,
    losses,
    networks,
    observables,
    sampling_strategies,
    tasks,
    trainers,
    units,
    utils,
    value_functions,
)
from swarmrl_amd.engine import swarm_engine as espresso  # noqa: F401
from swarmrl_amd.engine import EspressoMD, MDParams, SwarmEngine  # noqa: F401

_logger = logging.getLogger(__name__)
_logger.setLevel(logging.NOTSET)
