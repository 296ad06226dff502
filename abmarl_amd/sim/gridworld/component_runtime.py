"""The component plugin API on the engine (gw_component).

The reference composes a simulation's step() from component calls
(PositionState.reset, MoveActor.process_action, BinaryAttackActor /
SelectiveAttackActor.process_action, PositionCenteredEncodingObserver.get_obs;
state.py:13-22, actor.py:13-52, observer.py:13-52).  Here each such call is
one device operation on a one-env engine: a wave loads the env, runs the
component's body exactly as the fused programs do (same MT19937 stream
consumption), and stores it back.

The Python objects stay the reference's: the agents' position / health /
active, the Grid's insertion-ordered cells (grid.py) and the global numpy
legacy RNG.  Before every operation the runtime uploads them (in-cell order
becomes the engine's per-entity placement sequence), after it the engine's
results are mirrored back, so user code may read or edit either between
calls, and a user-written step() runs its component calls on the GPU in its
own order.  The done components are plain reads of that state and run on the
host (components.py).

One runtime per (grid, agents dict); it is rebuilt when the agents'
attributes or the grid's overlapping change.  The components' own parameters
(no_overlap_at_reset, stacked_attacks, attack_mapping, observe_self) travel
with each call, so several actors / observers may share a grid, as in the
reference's tests.  Up to 64 entities run on the one-wave engine, up to
GW_MAX_LANES (256) on the workgroup-per-env engine (wg_comp_kernel; the
BASELINE config-4 grid of 256 entities).

Host <-> device traffic per call is kept small: the state is uploaded only
when the host changed it since the last call (agent / Grid setters bump
sim/host_version.py; the numpy stream is compared word for word, and the
lane agents' position / active / health / ammo values against what the last
call left, which catches in-place array edits), in-cell
order goes up as per-cell ranks, and the download rewrites only the Grid
cells whose occupants moved.
"""
import numpy as np
import torch

from abmarl_amd import _abi
from abmarl_amd.sim import host_version
from abmarl_amd.sim.gridworld.agent import HealthAgent, GridObservingAgent, OrientationAgent, AmmoAgent


class ComponentError(RuntimeError):
    pass


def _registry(grid):
    return grid.__dict__.setdefault('_components', [])


def register_component(component):
    """Called by the engine-backed components at construction."""
    reg = _registry(component.grid)
    if component not in reg:
        reg.append(component)


class ComponentRuntime:
    # run the component ops on the workgroup-per-env engine even for <= 64
    # entities (tests: both kernels on the reference's component tests)
    force_workgroup = False

    @staticmethod
    def of(component):
        grid, agents = component.grid, component.agents
        rts = grid.__dict__.setdefault('_component_runtimes', {})
        sig = ComponentRuntime._signature(grid, agents)
        rt = rts.get(id(agents))
        if rt is not None and rt.agents is agents and rt.sig == sig and rt.statics and \
                (rt._synced is None or rt._synced[0] != host_version.VERSION[0]) and not rt._statics_intact():
            # the host moved, removed or replaced a static entity (they live in
            # the engine's cell template, not in lanes): every entity a lane
            # from now on, so the device sees the host's grid as it is
            grid.__dict__['_component_all_lanes'] = True
            sig = ComponentRuntime._signature(grid, agents)
        if rt is None or rt.agents is not agents or rt.sig != sig:
            rt = rts[id(agents)] = ComponentRuntime(grid, agents, sig)
        return rt

    @staticmethod
    def _signature(grid, agents):
        from abmarl_amd.sim.gridworld.components import (
            SelectiveAttackActor, PositionCenteredEncodingObserver, AttackActorBaseComponent,
            _TargetPlacementState)
        mine = [c for c in _registry(grid) if c.agents is agents]
        # encodings any registered attack actor may attack (never static)
        attacked = {}
        for c in mine:
            if isinstance(c, AttackActorBaseComponent):
                for k, v in c.attack_mapping.items():
                    if 1 <= k <= _abi.GW_MAX_ENC:
                        attacked[k] = attacked.get(k, 0) | sum(1 << e for e in v if 1 <= e <= _abi.GW_MAX_ENC)
        sig = [tuple(agents), tuple(sorted(grid.overlap_bits().items())),
               any(isinstance(c, SelectiveAttackActor) for c in mine),
               ComponentRuntime.force_workgroup,
               any(isinstance(c, PositionCenteredEncodingObserver) for c in mine),
               # the maze placements place every entity: no static entities
               any(isinstance(c, _TargetPlacementState) for c in mine) or
               grid.__dict__.get('_component_all_lanes', False),
               tuple(sorted(attacked.items()))]
        sig.append(tuple((a.encoding, getattr(a, 'view_range', None), getattr(a, 'move_range', None),
                          getattr(a, 'attack_range', None), getattr(a, 'attack_strength', None),
                          getattr(a, 'attack_accuracy', None), getattr(a, 'simultaneous_attacks', None),
                          getattr(a, 'initial_health', None), getattr(a, 'initial_orientation', None),
                          getattr(a, 'initial_ammo', None),
                          None if a.initial_position is None else tuple(a.initial_position), a.blocking)
                         for a in agents.values()))
        return tuple(sig)

    def __init__(self, grid, agents, sig):
        from abmarl_amd.engine import GridWorldEngine
        from abmarl_amd.sim.gridworld.compile import agent_spec
        self.grid, self.agents, self.sig = grid, agents, sig
        self.ids = list(agents)
        # selective actions need the (2r+1)^2 action row; binary uses args[2] only
        kind = _abi.GW_ATTACK_SELECTIVE if sig[2] else _abi.GW_ATTACK_BINARY
        # the position-centred window is capped at GW_MAX_RANGE (ranges above
        # GW_FIXED_RANGE: the one-wave kernel's generic window path); without a
        # position-centred observer the window is not used at all, and the
        # absolute observer takes its view range with each call (any range)
        cap = _abi.GW_MAX_RANGE if sig[4] else _abi.GW_FIXED_RANGE
        views = [min(a.view_range, cap) for a in agents.values()
                 if isinstance(a, GridObservingAgent)]
        specs = [agent_spec(a) for a in agents.values()]
        for s_, a in zip(specs, agents.values()):
            s_.view_range = min(s_.view_range, cap)
            if not sig[4] and s_.kind & _abi.GW_K_GRID_OBSERVER:
                # no position-centred window on this grid: one view range
                # (the absolute observer takes its own with each call)
                s_.view_range = max(views)
            if a.blocking or isinstance(a, OrientationAgent):
                # the absolute observer's masks and the orientation ops take lanes
                s_.kind |= _abi.GW_K_LANE
        # static entities (walls: no mixin, an initial position, an encoding
        # nothing overlaps or attacks) stay in the engine's cell template; every
        # other entity is a lane (one wave up to 64, a workgroup up to 256)
        cc = _abi.CompiledConfig(
            grid.rows, grid.cols, specs, _abi.GW_SIM_TEAM_BATTLE,
            grid.overlap_bits(), dict(sig[6]), done_kind=_abi.GW_DONE_ACTIVE,
            obs_range=max(views) if views else 0, attack_kind=kind,
            force_workgroup=ComponentRuntime.force_workgroup)
        cc.cfg.component_api = 1
        # every entity a lane: the maze placements place every entity, and a
        # grid of static entities only has no lane to run on
        static = [self._static(a, s_, grid, sig) for a, s_ in zip(agents.values(), specs)]
        # a static entity whose initial cell another entity's initial position
        # also names: the reference's reset raises (Grid.place refuses), which
        # the lanes reproduce -- the cell template cannot hold both
        cells = {}
        for a in agents.values():
            if a.initial_position is not None:
                rc = (int(a.initial_position[0]), int(a.initial_position[1]))
                cells[rc] = cells.get(rc, 0) + 1
        clash = any(st and cells[(int(a.initial_position[0]), int(a.initial_position[1]))] > 1
                    for st, a in zip(static, agents.values()))
        cc.cfg.all_lanes = 1 if sig[5] or clash or not any(not st for st in static) else 0
        self.cc = cc
        try:
            self.eng = GridWorldEngine(cc, 1, seeds=[0])
        except RuntimeError as err:
            raise ComponentError(f"the component runtime cannot hold this grid: {err}") from err
        self.dev = self.eng.device
        # lane <-> entity: self.index maps an agent id to its lane
        ents = list(self.eng.lane_entities)
        all_agents = list(agents.values())
        self.lane_agents = [all_agents[i] for i in ents]
        self.lane_ids = [self.ids[i] for i in ents]
        self.index = {aid: k for k, aid in enumerate(self.lane_ids)}
        lanes = set(ents)
        self.statics = [all_agents[i] for i in range(len(all_agents)) if i not in lanes]
        A = len(ents)
        self.result = torch.zeros((1, 2 + A), dtype=torch.int32, device=self.dev)
        self.args = torch.zeros((1, self.eng.act_dim), dtype=torch.int32, device=self.dev)
        self.obs = torch.full((1, A) + self.eng.obs_shape, -2, dtype=torch.int32, device=self.dev)
        self._healthy = np.array([isinstance(a, HealthAgent) for a in self.lane_agents])
        self._ammo = np.array([isinstance(a, AmmoAgent) for a in self.lane_agents])
        # what the device holds after the last call: host version, numpy
        # stream, and the entities' (in grid, row, col, seq) for the mirror
        self._synced = None
        self._where = None
        self._fp = None

    @staticmethod
    def _static(agent, spec, grid, sig):
        """gw_create's static-entity rule (an initial position, no mixin that
        moves / acts / observes / has health, an encoding nothing overlaps or
        attacks, not GW_K_LANE)."""
        dyn = (_abi.GW_K_OBSERVING | _abi.GW_K_ACTING | _abi.GW_K_GRID_OBSERVER | _abi.GW_K_MOVING |
               _abi.GW_K_ATTACKING | _abi.GW_K_HEALTH | _abi.GW_K_LANE)
        ov = grid.overlap_bits()
        touched = 0
        for v in ov.values():
            touched |= v
        for v in dict(sig[6]).values():
            touched |= v
        e = agent.encoding
        return (not (spec.kind & dyn) and agent.initial_position is not None and not ov.get(e, 0)
                and not (touched >> e) & 1)

    # ------------------------------------------------------------- sync
    def _statics_intact(self):
        """Every static entity alone in its cell at its initial position (as
        the engine's cell template holds it), or the grid never reset."""
        cells = self.grid._internal
        if cells[0, 0] is None:
            return True
        for a in self.statics:
            r, c = (int(x) for x in a.initial_position)
            cell = cells[r, c]
            if not cell or len(cell) != 1 or cell.get(a.id) is not a:
                return False
            if a.position is None or int(a.position[0]) != r or int(a.position[1]) != c:
                return False
        return True

    def _rng_matches(self):
        st = np.random.get_state()
        s = self._synced
        return (st[2] == s[1] and st[3] == s[3] and st[4] == s[4] and np.array_equal(st[1], s[2]))

    def _upload(self):
        A = len(self.lane_ids)
        pos = np.zeros((1, A, 2), np.int32)
        health = np.zeros((1, A), np.float64)
        flags = np.zeros((1, A), np.uint8)
        seq = np.zeros((1, A), np.int32)
        cells = self.grid._internal
        for i, (aid, a) in enumerate(zip(self.lane_ids, self.lane_agents)):
            f = _abi.FLAG_LIVE
            p = a.position
            if p is not None:
                pos[0, i] = p
                cell = cells[int(p[0]), int(p[1])] if 0 <= p[0] < self.grid.rows and 0 <= p[1] < self.grid.cols \
                    else None
                if cell and aid in cell:
                    # in-cell insertion order as the rank inside the cell
                    seq[0, i] = list(cell).index(aid)
                    f |= _abi.FLAG_IN_GRID
            if a.active:
                f |= _abi.FLAG_ACTIVE
            flags[0, i] = f
            if self._healthy[i] and a.health is not None:
                health[0, i] = a.health
        st = np.random.get_state()
        assert st[0] == 'MT19937'
        self._gauss = st[3:]
        mt = np.zeros((1, _abi.GW_MT_STRIDE), np.uint32)
        mt[0, :624] = st[1]
        mt[0, 624] = st[2]
        mt[0, 625] = A                      # next placement sequence number (> every rank)
        d = self.dev
        self.eng.set_state(pos=torch.as_tensor(pos, device=d), health=torch.as_tensor(health, device=d),
                           flags=torch.as_tensor(flags, device=d), seq=torch.as_tensor(seq, device=d),
                           mt=torch.as_tensor(mt.view(np.int32), device=d))
        if self._ammo.any():
            ammo = np.zeros((1, A), np.int32)
            for i, a in enumerate(self.lane_agents):
                if self._ammo[i]:
                    ammo[0, i] = getattr(a, '_ammo', 0)
            self.eng.set_ammo(ammo)
        self._where = (flags[0] & _abi.FLAG_IN_GRID != 0, pos[0].copy(), seq[0].copy())

    def _download(self, op):
        st = {k: v.cpu().numpy() for k, v in self.eng.get_state().items()}
        if op == _abi.GW_OP_ATTACK and self._ammo.any():
            ammo = self.eng.get_ammo().cpu().numpy()[0]
            for i, a in enumerate(self.lane_agents):
                if self._ammo[i]:
                    a._ammo = int(ammo[i])
        mt = st['mt'].view(np.uint32)[0]
        np.random.set_state(('MT19937', mt[:624].copy(), int(mt[624])) + tuple(self._gauss))
        flags = st['flags'][0]
        inside = (flags & _abi.FLAG_IN_GRID) != 0
        pos, seq, health = st['pos'][0], st['seq'][0], st['health'][0]
        agents = self.lane_agents
        for i, a in enumerate(agents):
            if inside[i] or a.position is not None:
                a._position = pos[i].astype(int)
            if self._healthy[i] and (a.health is not None or op == _abi.GW_OP_HEALTH_RESET):
                a._health = float(health[i])
            a._active = bool(flags[i] & _abi.FLAG_ACTIVE)
        cells = self.grid._internal
        old_in, old_pos, old_seq = self._where
        moved = (inside != old_in) | (inside & ((pos != old_pos).any(1) | (seq != old_seq)))
        if op in (_abi.GW_OP_POSITION_RESET, _abi.GW_OP_MAZE_RESET) or cells[0, 0] is None:
            for r in range(self.grid.rows):
                for c in range(self.grid.cols):
                    cells[r, c] = {}
            if op == _abi.GW_OP_POSITION_RESET:
                # static entities: at their initial positions, alone in their cells
                for a in self.statics:
                    a._position = np.array(a.initial_position, dtype=int)
                    cells[tuple(int(x) for x in a.initial_position)] = {a.id: a}
            touched = {(int(p[0]), int(p[1])) for p in pos[inside]}
        else:
            touched = {(int(p[0]), int(p[1])) for p in old_pos[moved & old_in]} | \
                      {(int(p[0]), int(p[1])) for p in pos[moved & inside]}
        # each touched cell: its occupants in insertion (seq) order
        for rc in touched:
            here = np.nonzero(inside & (pos[:, 0] == rc[0]) & (pos[:, 1] == rc[1]))[0]
            cells[rc] = {self.lane_ids[i]: agents[i] for i in here[np.argsort(seq[here], kind='stable')]}
        self._where = (inside, pos.copy(), seq.copy())
        s = np.random.get_state()
        self._synced = (host_version.VERSION[0], s[2], s[1].copy(), s[3], s[4])
        self._fp = self._fingerprint()

    def _fingerprint(self):
        """The lane agents' position / active / health / ammo values as the
        host holds them: an in-place edit (an element of a position or health
        array) bumps no version, so op() compares this too."""
        out = []
        for a in self.lane_agents:
            p = a.position
            out.append((None if p is None else (int(p[0]), int(p[1])), bool(a.active),
                        getattr(a, '_health', None), getattr(a, '_ammo', None)))
        return out

    # ----------------------------------------------------------- operations
    def op(self, op, agent=None, args=None):
        """Run one component operation; returns (status, attacked agents, err)
        (the raw result row stays in self.last_result)."""
        lane = -1 if agent is None else self.index[agent.id]
        if self._synced is None or self._synced[0] != host_version.VERSION[0] or not self._rng_matches() or \
                self._fingerprint() != self._fp:
            self._upload()
        if args is not None:
            a = np.zeros((1, self.eng.act_dim), np.int32)
            flat = np.asarray(args, dtype=np.int64).reshape(-1)
            a[0, :flat.size] = flat
            self.args.copy_(torch.as_tensor(a, device=self.dev))
        self.eng.err.zero_()
        obs = self.obs if op == _abi.GW_OP_OBSERVE else (self._abs_obs() if op == _abi.GW_OP_OBSERVE_ABS else None)
        self.eng.component(op, lane, self.args if args is not None else None, self.result, obs)
        res = self.last_result = self.result[0].cpu().numpy()
        err = int(self.eng.err[0].item())
        self._download(op)
        attacked = [self.lane_agents[int(x)] for x in res[2:2 + int(res[1])]] \
            if op == _abi.GW_OP_ATTACK else []
        return int(res[0]), attacked, err

    def _abs_obs(self):
        if getattr(self, 'abs_obs', None) is None:
            self.abs_obs = torch.full((1, len(self.lane_ids), self.grid.rows, self.grid.cols), -2,
                                      dtype=torch.int32, device=self.dev)
        return self.abs_obs

    def observe_absolute(self, agent):
        """AbsoluteEncodingObserver.get_obs(agent): the (rows, cols) grid."""
        self.op(_abi.GW_OP_OBSERVE_ABS, agent, [int(agent.view_range)])
        return self.abs_obs[0, self.index[agent.id]].cpu().numpy().astype(int)

    def observe(self, agent, observe_self=True):
        if agent.view_range > _abi.GW_MAX_RANGE:
            raise ComponentError(f"PositionCenteredEncodingObserver: view_range {agent.view_range} > "
                                 f"{_abi.GW_MAX_RANGE} has no device window")
        self.op(_abi.GW_OP_OBSERVE, agent, [int(observe_self)])
        d = 2 * agent.view_range + 1
        return self.obs[0, self.index[agent.id], :d, :d].cpu().numpy().astype(int)
