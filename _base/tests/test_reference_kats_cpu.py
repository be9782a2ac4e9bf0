"""
Known-answer tests of the reference's unit suite for host-only components
(list path, no GPU): Director / PositionObservable observables
(CI/unit_tests/observables/test_director.py, test_position.py), FindPoint
(CI/unit_tests/agents/test_find_point.py), MultiTasking and the object-array
layout of MultiSensing.
"""

import numpy as np
from numpy.testing import assert_array_equal

from swarmrl_amd.components import Colloid


def _three():
    return [Colloid(np.array([0.0, 0.0, 0.0]), np.array([0.0, 1.0, 0]), 0, 0),
            Colloid(np.array([0.0, 1.0, 0.0]), np.array([0.0, 1.0, 0]), 1, 0),
            Colloid(np.array([1.0, 1.0, 0.0]), np.array([0.0, 1.0, 0]), 2, 0)]


def test_director_kat():
    from swarmrl_amd.observables import Director

    ob = Director(particle_type=0)
    cols = _three()
    assert_array_equal(ob.compute_single_observable(0, cols), np.array([0.0, 1.0, 0.0]))
    assert_array_equal(ob.compute_observable(cols), np.array([[0.0, 1.0, 0.0]] * 3))


def test_position_kat():
    from swarmrl_amd.observables import PositionObservable

    ob = PositionObservable(box_length=np.array([1.0, 1.0, 1.0]), particle_type=0)
    cols = _three()
    assert_array_equal(ob.compute_observable(cols),
                       np.array([[0.0, 0.0, 0.0], [0.0, 1.0, 0.0], [1.0, 1.0, 0.0]]))
    assert_array_equal(ob.compute_single_observable(0, cols), np.array([0.0, 0.0, 0.0]))


def test_find_point_kat():
    from swarmrl_amd.agents import FindPoint

    fm = FindPoint(act_force=1.234, act_torque=1.234, point=np.array([1, 0, 0]))
    orientation = np.array([1, 0, 0])
    cols = [Colloid(pos=np.array([2, 0, 0]), director=orientation, id=1)]
    assert fm.calc_action(cols)[0].force == 0
    cols.append(Colloid(pos=np.array([0, 0, 0]), director=orientation, id=5))
    assert fm.calc_action(cols)[-1].force == 1.234


def test_multi_tasking_sums_tasks():
    from swarmrl_amd.tasks import MultiTasking, Task

    class Const(Task):
        def __init__(self, v):
            super().__init__(0)
            self.v = v

        def __call__(self, colloids):
            return np.full(len(self.get_colloid_indices(colloids)), self.v)

    mt = MultiTasking(particle_type=0, tasks=[Const(1.5), Const(-0.25)])
    assert_array_equal(mt(_three()), np.full(3, 1.25, np.float32))


def test_multi_sensing_object_layout():
    from swarmrl_amd.observables import Director, MultiSensing, PositionObservable

    ms = MultiSensing([PositionObservable(np.array([2.0, 2.0, 2.0])), Director()])
    out = ms.compute_observable(_three())
    assert out.dtype == object and out.shape[:2] == (3, 2)
    assert_array_equal(np.asarray(out[2, 0], dtype=float), [0.5, 0.5, 0.0])
    assert_array_equal(np.asarray(out[1, 1], dtype=float), [0.0, 1.0, 0.0])
