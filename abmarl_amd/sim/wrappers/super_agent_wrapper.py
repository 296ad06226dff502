"""Super agents: one policy id controlling several agents (reference:
abmarl/sim/wrappers/super_agent_wrapper.py:11-292).

A super agent's observation is {covered id: obs, 'mask': {covered id: [live]}},
its action a dict over its covered agents, its reward the sum over covered
agents (a done agent's last reward counted once), and it is done when all of
its covered agents are.  A covered agent that is done reports its last real
observation once, then its null observation (with a one-time warning when it
has none).

`BatchedSuperAgents` is the same reduction over the engine's lane tensors for
the batched env: rewards summed per super agent with one index_add on the
device (a lane that finished earlier carries reward 0, so the "counted once"
rule holds by construction), done = all covered done, mask = covered live.
"""
import warnings

import numpy as np

from abmarl_amd.spaces import Dict, MultiBinary, make_dict
from abmarl_amd.sim.agent_based_simulation import Agent
from abmarl_amd.sim.wrappers.sar_wrapper import Wrapper


class SuperAgentWrapper(Wrapper):
    def __init__(self, sim, super_agent_mapping=None, **kwargs):
        self.sim = sim
        self._warned = False
        self.super_agent_mapping = super_agent_mapping

    @property
    def super_agent_mapping(self):
        return self._mapping

    @super_agent_mapping.setter
    def super_agent_mapping(self, value):
        assert type(value) is dict, "super agent mapping must be a dictionary."
        covered = set()
        for sup, members in value.items():
            assert type(sup) is str, "The keys super agent mapping must be the super agent's id."
            assert sup not in self.sim.agents, \
                "A super agent cannot have the same id as an agent from the underlying sim."
            assert type(members) is list, \
                "The values in super agent mapping must be lists of agent ids."
            for aid in members:
                assert type(aid) is str, "The covered agents list must be agent ids."
                assert aid in self.sim.agents, \
                    "The covered agent must be an agent in the underlying sim."
                assert aid not in covered, "The agent is already covered by another super agent."
                assert isinstance(self.sim.agents[aid], Agent), \
                    "Covered agents must be learning Agents."
                covered.add(aid)
        self._covered_agents = covered
        self._uncovered_agents = self.sim.agents.keys() - covered
        self._mapping = value
        self._build_agents()

    def _build_agents(self):
        agents = {}
        for sup, members in self._mapping.items():
            obs = {aid: self.sim.agents[aid].observation_space for aid in members}
            obs['mask'] = {aid: MultiBinary(1) for aid in members}
            agents[sup] = Agent(id=sup, observation_space=make_dict(obs),
                                action_space=Dict({aid: self.sim.agents[aid].action_space
                                                   for aid in members}))
        for aid in self._uncovered_agents:
            agents[aid] = self.sim.agents[aid]
        self.agents = agents

    def _not_covered(self, agent_id, what):
        assert agent_id not in self._covered_agents, \
            f"We cannot {what} an agent that is covered by a super agent."

    def reset(self, **kwargs):
        self._obs_reported = dict.fromkeys(self._covered_agents, False)
        self._reward_reported = dict.fromkeys(self._covered_agents, False)
        self.sim.reset(**kwargs)

    def step(self, action_dict, **kwargs):
        flat = {}
        for aid, action in action_dict.items():
            self._not_covered(aid, "receive actions from")
            if aid in self._mapping:
                # actions for covered agents that are already done are dropped
                flat.update({cid: a for cid, a in action.items() if not self.sim.get_done(cid)})
            else:
                flat[aid] = action
        self.sim.step(flat, **kwargs)

    def get_obs(self, agent_id, **kwargs):
        self._not_covered(agent_id, "produce observations for")
        if agent_id not in self._mapping:
            return self.sim.get_obs(agent_id, **kwargs)
        out = {'mask': {}}
        for cid in self._mapping[agent_id]:
            done = self.sim.get_done(cid, **kwargs)
            if done and self._obs_reported[cid]:
                out[cid] = self._null_obs(cid, **kwargs)
            else:
                out[cid] = self.sim.get_obs(cid, **kwargs)
                if done:
                    self._obs_reported[cid] = True
            out['mask'][cid] = [not done]
        return out

    def get_reward(self, agent_id, **kwargs):
        self._not_covered(agent_id, "get rewards for")
        if agent_id not in self._mapping:
            return self.sim.get_reward(agent_id, **kwargs)
        total = 0
        for cid in self._mapping[agent_id]:
            if not self.sim.get_done(cid, **kwargs):
                total += self.sim.get_reward(cid, **kwargs)
            elif not self._reward_reported[cid]:
                total += self.sim.get_reward(cid, **kwargs)
                self._reward_reported[cid] = True
        return total

    def get_done(self, agent_id, **kwargs):
        self._not_covered(agent_id, "get done for")
        if agent_id not in self._mapping:
            return self.sim.get_done(agent_id, **kwargs)
        return all(self.sim.get_done(cid) for cid in self._mapping[agent_id])

    def get_info(self, agent_id, **kwargs):
        self._not_covered(agent_id, "get info for")
        if agent_id not in self._mapping:
            return self.sim.get_info(agent_id, **kwargs)
        return {cid: self.sim.get_info(cid, **kwargs) for cid in self._mapping[agent_id]}

    def _null_obs(self, agent_id, **kwargs):
        null = getattr(self.sim.agents[agent_id], 'null_observation', None)
        if null is not None and (not isinstance(null, (dict, list)) or len(null)):
            return null
        if not self._warned:
            self._warned = True
            warnings.warn("Some covered agents in the SuperAgentWrapper do not specify "
                          "a null observation. This may corrupt the learning data.")
        return self.sim.get_obs(agent_id, **kwargs)


class BatchedSuperAgents:
    """Super-agent reduction over a BatchedMultiAgentEnv's lane tensors.

    mapping: {super id: [covered agent ids]}; every covered id must be a lane.
    """

    def __init__(self, env, mapping):
        import torch
        lane = {aid: i for i, aid in enumerate(env.agent_ids)}
        self.ids = list(mapping)
        width = max(len(v) for v in mapping.values())
        members = np.full((len(self.ids), width), -1, np.int64)
        owner = np.full(len(env.agent_ids), -1, np.int64)
        for s, sup in enumerate(self.ids):
            for j, aid in enumerate(mapping[sup]):
                assert aid in lane, f"{aid} is not an engine lane"
                assert owner[lane[aid]] < 0, f"{aid} is already covered"
                members[s, j] = lane[aid]
                owner[lane[aid]] = s
        dev = env.engine.device
        self.members = torch.as_tensor(members, device=dev)       # [S][K], -1 = padding
        self.covered = torch.as_tensor(np.nonzero(owner >= 0)[0], device=dev)
        self.owner = torch.as_tensor(owner[owner >= 0], device=dev)

    def reduce(self, reward, done, live):
        """reward f64[E][A], done u8[E][A], live bool[E][A] ->
        (reward f64[E][S], done bool[E][S], mask bool[E][S][K])."""
        import torch
        E, S = reward.shape[0], len(self.ids)
        r = torch.zeros((E, S), dtype=reward.dtype, device=reward.device)
        r.index_add_(1, self.owner, reward.index_select(1, self.covered))
        pad = self.members < 0
        idx = self.members.clamp(min=0)
        d = done.bool()[:, idx] | pad                               # padding counts as done
        mask = live[:, idx] & ~pad
        return r, d.all(dim=2), mask
