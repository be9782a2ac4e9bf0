"""swarmrl_amd.trainers on CPU (the HIP backend replaced by the recording fake
of test_engine_host): the reference trainers' loop contracts
(swarmrl/trainers/trainer.py:76-101, continuous_trainer.py:22-89,
episodic_trainer.py:26-130) -- episodes of integrate(episode_length), every
ActorCriticAgent updated after each, classical agents skipped, the kill
switch ending a continuous run, engines rebuilt with h5_group_tag per cycle.
"""

import numpy as np
import pytest

from swarmrl_amd.agents import dummy_models
from swarmrl_amd.agents.actor_critic import ActorCriticAgent
from swarmrl_amd.trainers import ContinuousTrainer, EpisodicTrainer, Trainer
from test_engine_host import _engine, fake_backend  # noqa: F401 (fixture)


class _Learner(ActorCriticAgent):
    """An ActorCriticAgent whose update is recorded instead of run."""

    def __init__(self, particle_type=0, rewards=(1.0, 3.0), kill_at=None):
        self.particle_type = particle_type
        self.updates = 0
        self.resets = 0
        self._rewards = list(rewards)
        self._kill_at = kill_at
        self.kill_switch = False

    def calc_action(self, colloids):
        return [dummy_models.ConstForce(1.0).calc_action([c])[0] for c in colloids]

    def calc_reward(self, colloids, external_reward=0.0):
        return np.zeros(len(colloids))

    def reset_agent(self, colloids):
        self.resets += 1

    def update_agent(self):
        self.updates += 1
        return [np.array([r]) for r in self._rewards], self.updates == self._kill_at


def test_update_rl_updates_learners_only():
    learner, const = _Learner(0), dummy_models.ConstForce(1.0)
    const.particle_type = 1
    t = Trainer([learner, const])
    ff, reward, stop = t.update_rl()
    assert learner.updates == 1 and float(reward) == 2.0 and stop is False
    assert set(ff.agents) == {"0", "1"}


def test_continuous_trainer_episodes_and_kill_switch(fake_backend, tmp_path):  # noqa: F811
    eng = _engine(tmp_path, 2, 2)
    learner = _Learner(kill_at=3)
    rewards = ContinuousTrainer([learner]).perform_rl_training(eng, n_episodes=5,
                                                                episode_length=4, load_bar=False)
    # episodes 1, 2 recorded; episode 3 raised the kill switch (not recorded)
    assert np.array_equal(rewards, [0.0, 2.0, 2.0])
    assert learner.updates == 3 and learner.resets == 1
    native = fake_backend.instances[-1]
    assert sum(native.runs()) == 3 * 4 * eng.params.steps_per_slice


def test_episodic_trainer_resets_and_group_tags(fake_backend, tmp_path):  # noqa: F811
    tags = []

    def get_engine(system, tag):
        tags.append(tag)
        return _engine(tmp_path / tag, 2, 2)

    learner = _Learner()
    rewards = EpisodicTrainer([learner]).perform_rl_training(
        get_engine, None, n_episodes=5, episode_length=3, reset_frequency=2, load_bar=False)
    assert tags == ["0", "1", "2"]          # episodes 0, 2, 4
    assert learner.resets == 3 and learner.updates == 5
    assert rewards.shape == (6,) and np.all(rewards[1:] == 2.0)


def test_episodic_trainer_engine_without_group_tag(fake_backend, tmp_path):  # noqa: F811
    def get_engine(system):
        return _engine(tmp_path, 2, 2)

    with pytest.raises(ValueError, match="h5_group_tag"):
        EpisodicTrainer([_Learner()]).perform_rl_training(get_engine, None, 1, 2, load_bar=False)
    r = EpisodicTrainer([_Learner()]).perform_rl_training(
        get_engine, None, 2, 2, load_bar=False, save_episodic_data=False)
    assert r.shape == (3,)
