"""Dict-API runtime: one SmartGridWorldSimulation on a one-env engine.

Every reset/step:
  1. uploads the global numpy legacy RNG state (np.random.get_state()) into
     the env's MT19937 slot,
  2. runs the fused HIP reset / step,
  3. reads the RNG state back into np.random (np.random.set_state), and
     mirrors positions / health / active onto the agent objects.
So ``np.random.seed(s); manager.reset(); manager.step(...)`` consumes and
produces exactly what the reference does for the same seed.
"""
import random

import numpy as np
import torch

from abmarl_amd import _abi
from abmarl_amd.engine import GridWorldEngine
from abmarl_amd.sim.gridworld.agent import HealthAgent, GridObservingAgent, OrientationAgent, AmmoAgent


class DictRuntime:
    """For the Pacman program the manager's protocol stays in Python (the
    engine's simulation-only entry points): step runs sim.step alone, rewards
    accumulate on the device until get_reward consumes them, and get_obs draws
    the observation when it is called, in call order — so the same runtime
    serves AllStepManager and TurnBasedManager exactly."""

    def __init__(self, sim, compiled, device=None):
        self.sim = sim
        self.cc = compiled
        self.ids = list(sim.agents.keys())
        self.index = {aid: i for i, aid in enumerate(self.ids)}
        self.eng = GridWorldEngine(compiled, 1, device=device, seeds=[0])
        self.dev = self.eng.device
        # engine arrays are per lane; static entities (walls: never move, act
        # or die, overlap nothing) have no lane (gw_engine.h "Entities and lanes")
        self.lanes = self.eng.lane_entities
        self.lane_of = np.full(len(self.ids), -1, np.int64)
        self.lane_of[self.lanes] = np.arange(len(self.lanes))
        A = len(self.lanes)
        self.obs = np.full((A, self.cc.obs_side, self.cc.obs_side), -2, np.int32)
        self.reward = np.zeros(A)
        self.done = np.ones(A, np.uint8)
        self.all_done = False
        self.live = np.zeros(A, bool)
        self.key = 'position_centered_encoding'
        self.observes = [isinstance(a, GridObservingAgent) for a in sim.agents.values()]
        self.sides = [2 * a.view_range + 1 if isinstance(a, GridObservingAgent) else 0
                      for a in sim.agents.values()]
        self.lazy = compiled.cfg.sim_kind == _abi.GW_SIM_PACMAN
        self.has_ammo = any(isinstance(a, AmmoAgent) for a in sim.agents.values())
        # PositionState(randomize_placement_order=True): the component's own
        # agents dict, reshuffled in place at every reset (state.py:97-101)
        self.place_items = list(range(len(self.ids))) if compiled.randomize_placement_order else None
        if self.lazy:
            self.key = 'absolute_encoding'
            specs = compiled.specs
            # passive (food) entities, in entity order = passive index order
            self.passive = [i for i, s in enumerate(specs) if s.kind & _abi.GW_K_FOOD]
            self.racc = np.zeros(A)
            self._racc_dirty = False

    # -------------------------------------------------------------- RNG sync
    def _push_rng(self):
        st = np.random.get_state()
        assert st[0] == 'MT19937'
        mt = self.eng.get_state()['mt']
        host = mt.cpu().numpy().view(np.uint32).copy()
        host[0, :624] = st[1]
        host[0, 624] = st[2]
        self._gauss = st[3:]
        self.eng.set_state(mt=torch.as_tensor(host.view(np.int32), device=self.dev))

    def _pull(self):
        st = self.eng.get_state()
        if self.lazy:
            aux = self.eng.get_aux_state()
        if self.has_ammo:
            st['ammo'] = self.eng.get_ammo()
        torch.cuda.synchronize(self.dev)
        host = {k: v.cpu().numpy() for k, v in st.items()}
        pbits = aux['passive'].cpu().numpy().view(np.uint32)[0] if self.lazy else None
        food = {}
        if self.lazy:
            for k, i in enumerate(self.passive):
                food[i] = bool((pbits[k >> 5] >> (k & 31)) & 1)
        mt = host['mt'].view(np.uint32)[0]
        np.random.set_state(('MT19937', mt[:624].copy(), int(mt[624])) + tuple(self._gauss))
        flags = host['flags'][0]
        self.live = (flags & _abi.FLAG_LIVE) != 0
        for i, agent in enumerate(self.sim.agents.values()):
            k = self.lane_of[i]
            if i in food:                  # passive food: on the grid until eaten
                agent.position = np.array(agent.initial_position, dtype=int)
                agent._health = 1.0 if food[i] else 0.0
                agent._active = food[i]
                continue
            if k < 0:                      # static entity: at its initial position
                agent.position = np.array(agent.initial_position, dtype=int)
                agent._active = True
                continue
            if isinstance(agent, OrientationAgent):
                agent._orientation = int((flags[k] >> 3) & 7) or None
            agent.position = host['pos'][0, k].astype(int)
            if isinstance(agent, HealthAgent):
                agent._health = float(host['health'][0, k])
            if isinstance(agent, AmmoAgent):
                agent._ammo = int(host['ammo'][0, k])
            agent._active = bool(flags[k] & _abi.FLAG_ACTIVE)

    # ------------------------------------------------- lazy (Pacman) protocol
    def _push_racc(self):
        if self._racc_dirty:
            self.eng.set_aux_state(racc=torch.as_tensor(self.racc[None], device=self.dev))
            self._racc_dirty = False

    def _shuffle_placement(self):
        """random.shuffle of the PositionState's agents dict, as the reference
        does it (Python's own random: the same draws), then the lanes in that
        order to the engine (static entities overlap nothing: left out)."""
        if self.place_items is None:
            return
        random.shuffle(self.place_items)
        self.eng.set_placement_order([int(self.lane_of[i]) for i in self.place_items if self.lane_of[i] >= 0])

    def _lazy_reset(self):
        self._shuffle_placement()
        self._push_rng()
        self.eng.err.zero_()
        self.eng.sim_reset()
        self.eng.check_errors()
        self.racc[:] = 0.0
        self._racc_dirty = False
        self.all_done = False
        self._pull()

    def _lazy_step(self, action_dict):
        act = np.zeros((1, len(self.lanes), self.eng.act_dim), np.int32)
        act[0, :, 2] = -1                      # not in action_dict
        for aid, a in action_dict.items():
            k = self.lane_of[self.index[aid]]
            assert k >= 0, f"{aid} does not act"
            a = a if isinstance(a, dict) else {}
            act[0, k, 0] = int(np.asarray(a.get('move', 0)).reshape(-1)[0])
            act[0, k, 2] = 0
        self._push_rng()
        self._push_racc()
        self.eng.err.zero_()
        rew, done, all_done = self.eng.sim_step(torch.as_tensor(act, device=self.dev))
        self.racc = rew[0].cpu().numpy().copy()
        self.done = done[0].cpu().numpy().copy()
        self.all_done = bool(all_done[0].item())
        self._pull()
        self.eng.check_errors()

    def _lazy_obs(self, i):
        self._push_rng()
        self._push_racc()
        o = self.eng.observe(self.lane_of[i])[0].cpu().numpy()
        self._pull()
        return {self.key: o.astype(int)}

    # -------------------------------------------------------------- protocol
    def reset(self):
        if self.lazy:
            return self._lazy_reset()
        self._shuffle_placement()
        self._push_rng()
        self.eng.err.zero_()
        obs = self.eng.reset()
        self.eng.check_errors()
        self.obs = obs[0].cpu().numpy()
        self.reward[:] = 0
        self.done[:] = 0
        self.all_done = False
        self._pull()

    def step(self, action_dict):
        ids = [a for a in action_dict]
        order = [self.index[a] for a in ids]
        shuffled = order != sorted(order)
        if shuffled and self.cc.cfg.sim_kind not in (
                _abi.GW_SIM_TEAM_BATTLE, _abi.GW_SIM_REACH_TARGET, _abi.GW_SIM_TRAFFIC,
                _abi.GW_SIM_PACMAN):
            raise NotImplementedError(
                "an action dict in another order than the agents dict (randomize_action_input) "
                "runs with the TeamBattle, ReachTheTarget, TrafficCorridor and Pacman programs only")
        # AllStepManager(randomize_action_input=True): the shuffled dict's order
        if shuffled:
            first = [int(self.lane_of[i]) for i in order if self.lane_of[i] >= 0]
            rest = [k for k in range(len(self.lanes)) if k not in set(first)]
            self.eng.set_action_order(first + rest)
            self._act_order_set = True
        elif getattr(self, '_act_order_set', False):
            self.eng.set_action_order(None)
            self._act_order_set = False
        if self.lazy:
            return self._lazy_step(action_dict)
        act = np.zeros((1, len(self.lanes), self.eng.act_dim), np.int32)
        act[0, :, 2] = -1                      # not in action_dict: does not act
        for aid, a in action_dict.items():
            k = self.lane_of[self.index[aid]]
            assert k >= 0 and self.live[k], "Received an action for an agent that is already done."
            a = a if isinstance(a, dict) else {}
            act[0, k, 0:2] = np.asarray(a.get('move', (0, 0)), dtype=np.int64)
            at = np.asarray(a.get('attack', 0), dtype=np.int64).reshape(-1)
            act[0, k, 2] = 0
            act[0, k, 2:2 + at.size] = at      # binary: one int; selective: (2r+1)^2 cells
        self._push_rng()
        self.eng.err.zero_()
        obs, rew, done, all_done = self.eng.step(torch.as_tensor(act, device=self.dev))
        self.obs = obs[0].cpu().numpy()
        self.reward = rew[0].cpu().numpy().copy()
        self.done = done[0].cpu().numpy().copy()
        self.all_done = bool(all_done[0].item())
        self._pull()
        self.eng.check_errors()                # e.g. ReachTheTarget's double remove -> KeyError

    def get_obs(self, agent_id):
        i = self.index[agent_id]
        if not self.observes[i]:
            return {}
        if self.lazy:
            return self._lazy_obs(i)
        s = self.sides[i]
        return {self.key: self.obs[self.lane_of[i], :s, :s].astype(int)}

    def get_reward(self, agent_id):
        k = self.lane_of[self.index[agent_id]]
        if k < 0:
            return 0.0
        if self.lazy:                          # smart.py:101-104: consume the accumulator
            r = float(self.racc[k])
            self.racc[k] = 0.0
            self._racc_dirty = True
            return r
        r = float(self.reward[k])
        self.reward[k] = 0.0
        return r

    def get_done(self, agent_id):
        k = self.lane_of[self.index[agent_id]]
        return False if k < 0 else bool(self.done[k])

    def get_all_done(self):
        return self.all_done

    def done_agents(self):
        out = {self.ids[i] for i in range(len(self.ids)) if self.lane_of[i] < 0}
        out.update(self.ids[e] for e, lv in zip(self.lanes, self.live) if not lv)
        return out
