"""Batched tensor API over the HIP engine (one handle = E environments).

All buffers are torch tensors on the engine's device; the C-ABI receives raw
device pointers and the current HIP stream.  This is the vectorised-env
surface (RLlib VectorEnv-style): ``reset`` / ``step`` advance every env in
one kernel launch each, with optional on-device auto-reset.
"""
import ctypes as C

import numpy as np
import torch

from abmarl_amd import _abi, _native


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def env_seeds(n_envs, run=0, first_env=0):
    """Per-env MT19937 seeds, keyed by the GLOBAL env id:
    seed_e = 1_000_003 * run + e  (mod 2^32)."""
    e = np.arange(first_env, first_env + n_envs, dtype=np.uint64)
    return ((np.uint64(1_000_003) * np.uint64(run) + e) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


class GridWorldEngine:
    def __init__(self, compiled, n_envs, device=None, seeds=None):
        if not torch.cuda.is_available():
            raise RuntimeError("GridWorldEngine needs a ROCm GPU (no CPU fallback).")
        self.L = _native.lib()
        self.cc = compiled
        self.device = torch.device(device if device is not None else 'cuda')
        if self.device.index is None:
            self.device = torch.device('cuda', torch.cuda.current_device())
        self.E, self.S = int(n_envs), compiled.obs_side
        h = C.c_void_p()
        # the engine passes its own obs buffer to every call: rows that hold
        # -2 and stay -2 are not rewritten (gw_config.persistent_obs)
        cfg = _abi.Config.from_buffer_copy(compiled.cfg)
        cfg.persistent_obs = 1
        self._cfg = cfg
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_create(C.cast(C.byref(cfg), C.c_void_p), self.E,
                                           self.device.index, C.byref(h)), 'gw_create')
        self.h = h
        # per-env arrays are per lane; static entities (never move / act /
        # die, overlap nothing) live in the engine's cell template
        self.A = int(self.L.gw_num_lanes(h))
        # ReachTheTarget beyond 64 lanes runs on a workgroup per env (gw_rtt.inc)
        # GW_KERNEL_*: MazeNavigation runs one env per lane (gw_lane.inc)
        self.kernel = int(self.L.gw_env_kernel(h))
        self.wg = self.kernel == _abi.GW_KERNEL_WORKGROUP
        ents = (C.c_int32 * self.A)()
        _native.check(self.L.gw_lane_entities(h, ents), 'gw_lane_entities')
        self.lane_entities = np.array(ents[:], dtype=np.int64)
        dev = self.device
        E, A = self.E, self.A
        rows, cols = C.c_int32(), C.c_int32()
        _native.check(self.L.gw_obs_shape(h, C.byref(rows), C.byref(cols)), 'gw_obs_shape')
        self.obs_shape = (rows.value, cols.value)   # per lane: (S, S) or (rows, cols) absolute
        self.n_passive = int(self.L.gw_num_passive(h))
        self.pacman = compiled.cfg.sim_kind == _abi.GW_SIM_PACMAN
        self.obs = torch.full((E, A) + self.obs_shape, -2, dtype=torch.int32, device=dev)
        self.reward = torch.zeros((E, A), dtype=torch.float64, device=dev)
        self.done = torch.ones((E, A), dtype=torch.uint8, device=dev)
        self.all_done = torch.zeros((E,), dtype=torch.uint8, device=dev)
        self.err = torch.zeros((E,), dtype=torch.int32, device=dev)
        self.acting = torch.zeros((E,), dtype=torch.int64, device=dev)
        self.act_dim = int(self.L.gw_act_dim(self.h))
        self.actions = torch.zeros((E, A, self.act_dim), dtype=torch.int32, device=dev)
        self._dbg = None
        self.stamps = None
        if _native.VARIANT == 'stamps':
            # per-env s_memtime per phase (diagnostic build, tools/stamps.py)
            self.stamps = torch.zeros((E, 64), dtype=torch.int64, device=dev)
            self.L.gw_debug_set_stamps.argtypes = [C.c_void_p, C.c_void_p]
            self.L.gw_debug_set_stamps(self.h, _ptr(self.stamps))
        if _native.VARIANT == 'checks':
            self._dbg = torch.zeros(256, dtype=torch.int32, device=dev)   # [0..15] checks; the rest diagnostic builds
            self.L.gw_debug_set_checks.argtypes = [C.c_void_p, C.c_void_p]
            self.L.gw_debug_set_checks(self.h, _ptr(self._dbg))
        self.seed(env_seeds(E) if seeds is None else seeds)

    def _check_debug(self, what):
        if self._dbg is None:
            return
        d = self._dbg.cpu().numpy().view(np.uint32)
        if d[0]:
            raise AssertionError(
                f"GW_CHECKS violation after {what}: mask={d[0]:#x} first code={d[1]} v0={int(np.int32(d[2]))} "
                f"v1={int(np.int32(d[3]))} env={d[4]} lane={d[5]} more={d[6]}")

    def __del__(self):
        h = getattr(self, 'h', None)
        if h is not None and h.value:
            try:
                torch.cuda.synchronize(self.device)
                self.L.gw_destroy(h)
            except Exception:
                pass
            self.h = None

    def step_occupancy(self):
        """(resident workgroups per CU, threads per workgroup, dynamic LDS
        bytes) of this engine's step launch (gw_step_occupancy)."""
        nb, bt, lds = C.c_int32(), C.c_int32(), C.c_int64()
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_step_occupancy(self.h, C.byref(nb), C.byref(bt), C.byref(lds)),
                          'gw_step_occupancy')
        return nb.value, bt.value, lds.value

    # ------------------------------------------------------------ control
    def seed(self, seeds):
        s = torch.as_tensor(np.asarray(seeds, dtype=np.uint32).view(np.int32),
                            device=self.device)
        assert s.numel() == self.E
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_seed(self.h, _ptr(s), _stream()), 'gw_seed')
            torch.cuda.current_stream().synchronize()

    def reset(self, mask=None, all_done=None, horizon=0):
        """Reset selected envs (all of them by default); returns the obs buffer."""
        out = self.obs
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_reset(self.h, _ptr(mask), _ptr(all_done), int(horizon),
                                          _ptr(out), _ptr(self.err), _stream()), 'gw_reset')
        self._check_debug('gw_reset')
        return out

    def step(self, actions=None):
        """One AllStepManager.step on every env; returns (obs, reward, done, all_done)."""
        a = self.actions if actions is None else actions
        assert a.dtype == torch.int32 and a.is_contiguous() and a.shape == self.actions.shape
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_step(self.h, _ptr(a), _ptr(self.obs), _ptr(self.reward),
                                         _ptr(self.done), _ptr(self.all_done), _ptr(self.acting),
                                         _ptr(self.err), _stream()), 'gw_step')
        self._check_debug('gw_step')
        return self.obs, self.reward, self.done, self.all_done

    def step_autoreset(self, actions=None, horizon=0):
        """step() + in-launch reset of the envs whose '__all__' is set or that
        reached `horizon`: their obs is the next episode's first observation,
        reward/done/all_done the terminal step's."""
        a = self.actions if actions is None else actions
        assert a.dtype == torch.int32 and a.is_contiguous() and a.shape == self.actions.shape
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_step_autoreset(
                self.h, _ptr(a), _ptr(self.obs), _ptr(self.reward), _ptr(self.done),
                _ptr(self.all_done), _ptr(self.acting), int(horizon), _ptr(self.err), _stream()),
                'gw_step_autoreset')
        self._check_debug('gw_step_autoreset')
        return self.obs, self.reward, self.done, self.all_done

    def step_autoreset_next(self, actions=None, horizon=0):
        """NEXT_STEP auto-reset (gymnasium convention): envs whose episode
        ended in the previous call (all_done set, or at the horizon) are reset
        by this call — obs is their first observation, reward 0, actions
        ignored — and every other env takes one step."""
        a = self.actions if actions is None else actions
        assert a.dtype == torch.int32 and a.is_contiguous() and a.shape == self.actions.shape
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_step_autoreset_next(
                self.h, _ptr(a), _ptr(self.obs), _ptr(self.reward), _ptr(self.done),
                _ptr(self.all_done), _ptr(self.acting), int(horizon), _ptr(self.err), _stream()),
                'gw_step_autoreset_next')
        self._check_debug('gw_step_autoreset_next')
        return self.obs, self.reward, self.done, self.all_done

    # ------------------------------------------------- Pacman program protocols
    def _turn_bufs(self):
        if not hasattr(self, 'returned'):
            self.returned = torch.zeros((self.E, self.A), dtype=torch.uint8, device=self.device)
            self.turn = torch.full((self.E,), -1, dtype=torch.int32, device=self.device)
        return self.returned, self.turn

    def turn_reset(self, mask=None):
        """TurnBasedManager.reset of the selected envs (all by default):
        returns (obs, returned, turn)."""
        ret, turn = self._turn_bufs()
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_turn_reset(self.h, _ptr(mask), _ptr(self.obs), _ptr(ret),
                                               _ptr(turn), _ptr(self.err), _stream()),
                          'gw_turn_reset')
        return self.obs, ret, turn

    def turn_step(self, actions=None, horizon=0):
        """TurnBasedManager.step with next-step auto-reset: the lane turn[e]
        acts; returns (obs, reward, done, all_done, returned, turn)."""
        a = self.actions if actions is None else actions
        assert a.dtype == torch.int32 and a.is_contiguous() and a.shape == self.actions.shape
        ret, turn = self._turn_bufs()
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_turn_step(
                self.h, _ptr(a), _ptr(self.obs), _ptr(self.reward), _ptr(self.done),
                _ptr(self.all_done), _ptr(ret), _ptr(turn), _ptr(self.acting), int(horizon),
                _ptr(self.err), _stream()), 'gw_turn_step')
        return self.obs, self.reward, self.done, self.all_done, ret, turn

    def turn_rollout_buffers(self, n_steps):
        """Per-turn output slabs for turn_rollout(): rollout_buffers plus
        returned[n][E][A] and turn[n][E]."""
        out = self.rollout_buffers(n_steps)
        out['returned'] = torch.empty((n_steps, self.E, self.A), dtype=torch.uint8, device=self.device)
        out['turn'] = torch.empty((n_steps, self.E), dtype=torch.int32, device=self.device)
        return out

    def turn_rollout(self, actions, horizon=0, out=None):
        """K = actions.shape[0] consecutive turn_step calls in ONE launch
        (gw_turn_rollout): turn t's outputs in slab t of `out`
        (turn_rollout_buffers).  The '__all__' before turn 0 is self.all_done
        (the previous call's); afterwards it holds the last turn's.  obs rows
        of lanes not returned in a turn are left unwritten (mask: returned)."""
        K = int(actions.shape[0])
        assert actions.dtype == torch.int32 and actions.is_contiguous()
        assert tuple(actions.shape[1:]) == tuple(self.actions.shape), actions.shape
        assert actions.device == self.device, (actions.device, self.device)
        out = self.turn_rollout_buffers(K) if out is None else out
        self._check_rollout_buffers(K, out)
        for k, shape, dt in (('returned', (self.E, self.A), torch.uint8), ('turn', (self.E,), torch.int32)):
            t = out[k]
            assert t.dtype == dt and t.is_contiguous() and t.device == self.device, k
            assert tuple(t.shape[1:]) == shape and t.shape[0] >= K, (k, tuple(t.shape))
        self._turn_bufs()
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_turn_rollout(
                self.h, K, _ptr(actions), _ptr(out['obs']), _ptr(out['reward']), _ptr(out['done']),
                _ptr(out['all_done']), _ptr(self.all_done), _ptr(out['returned']), _ptr(out['turn']),
                _ptr(self.acting), int(horizon), _ptr(self.err), _stream()), 'gw_turn_rollout')
        # the single-call buffers follow the last turn
        self.turn.copy_(out['turn'][K - 1])
        self._check_debug('gw_turn_rollout')
        return out

    def _event_setter(self, events):
        """events = (start, stop) torch.cuda.Events already recorded once (so
        their hipEvents exist): a callable that hands them to the next kernel
        launch (gw_set_launch_events), which records them as part of its own
        dispatch instead of two event records around the launch."""
        if events is None:
            return None
        a, b = events
        ha, hb = int(a.cuda_event), int(b.cuda_event)
        assert ha and hb, "launch events must have been recorded once (created)"
        fn, h, pa, pb = self.L.gw_set_launch_events, self.h, C.c_void_p(ha), C.c_void_p(hb)

        def arm():
            st = fn(h, pa, pb)
            if st != 0:
                _native.check(st, 'gw_set_launch_events')
        return arm

    def turn_rollout_launcher(self, actions, horizon=0, out=None, events=None):
        """A prepared gw_turn_rollout launch (see rollout_launcher); the
        single-call turn buffer is not refreshed by it."""
        K = int(actions.shape[0])
        assert actions.dtype == torch.int32 and actions.is_contiguous()
        assert tuple(actions.shape[1:]) == tuple(self.actions.shape), actions.shape
        assert torch.cuda.current_device() == self.device.index, "launcher: the engine's device must be current"
        out = self.turn_rollout_buffers(K) if out is None else out
        self._check_rollout_buffers(K, out)
        fn = self.L.gw_turn_rollout
        args = (self.h, K, _ptr(actions), _ptr(out['obs']), _ptr(out['reward']), _ptr(out['done']),
                _ptr(out['all_done']), _ptr(self.all_done), _ptr(out['returned']), _ptr(out['turn']),
                _ptr(self.acting), int(horizon), _ptr(self.err), _stream())
        keep = (actions, out)
        arm = self._event_setter(events)

        def launch():
            if arm is not None:
                arm()
            st = fn(*args)
            if st != 0:
                _native.check(st, 'gw_turn_rollout')
            return keep[1]
        return launch

    def sim_reset(self, mask=None):
        """SmartGWS.reset only (no observation drawn)."""
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_sim_reset(self.h, _ptr(mask), _ptr(self.err), _stream()),
                          'gw_sim_reset')

    def sim_step(self, actions):
        """sim.step(action_dict): reward = accumulated (not consumed), done, all_done."""
        assert actions.dtype == torch.int32 and actions.is_contiguous()
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_sim_step(self.h, _ptr(actions), _ptr(self.reward),
                                             _ptr(self.done), _ptr(self.all_done), _ptr(self.err),
                                             _stream()), 'gw_sim_step')
        return self.reward, self.done, self.all_done

    def observe(self, lane, obs=None):
        """get_obs(lane) in every env (draws in call order); writes obs[:, lane]."""
        out = self.obs if obs is None else obs
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_observe(self.h, int(lane), _ptr(out), _stream()), 'gw_observe')
        return out[:, lane]

    def get_aux_state(self):
        E, A, dev = self.E, self.A, self.device
        pw = (self.n_passive + 31) // 32
        st = dict(racc=torch.zeros((E, A), dtype=torch.float64, device=dev),
                  passive=torch.zeros((E, max(pw, 1)), dtype=torch.int32, device=dev),
                  turn_pos=torch.full((E,), -1, dtype=torch.int32, device=dev))
        with torch.cuda.device(dev):
            _native.check(self.L.gw_get_aux_state(self.h, _ptr(st['racc']), _ptr(st['passive']),
                                                  _ptr(st['turn_pos']), _stream()),
                          'gw_get_aux_state')
        return st

    def set_aux_state(self, racc=None, passive=None, turn_pos=None):
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_set_aux_state(self.h, _ptr(racc), _ptr(passive),
                                                  _ptr(turn_pos), _stream()), 'gw_set_aux_state')

    def random_actions(self, key, step, env_offset=0, out=None):
        """Synthetic random policy (Philox, keyed by key / global env / step / agent)."""
        out = self.actions if out is None else out
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_random_actions(self.h, int(key) & 0xFFFFFFFFFFFFFFFF,
                                                   int(step) & 0xFFFFFFFF,
                                                   int(env_offset) & 0xFFFFFFFF, _ptr(out),
                                                   _stream()), 'gw_random_actions')
        return out

    AUTORESET_MODES = {'none': 0, 'same_step': 1, 'next_step': 2}

    # ------------------------------------------------ component plugin API
    def component(self, op, lane=-1, args=None, result=None, obs=None):
        """One component operation (gw_component, GW_OP_*) for entity `lane`
        in every env: args int32[E][act_dim] (MOVE / ATTACK), result
        int32[E][2 + A] (status, n attacked, attacked lanes), obs (OBSERVE)."""
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_component(self.h, int(op), int(lane), _ptr(args), _ptr(result),
                                              _ptr(obs), _ptr(self.err), _stream()), 'gw_component')
        return result

    def maze_reset(self, target, barrier_encodings, free_encodings, cluster_barriers=False,
                   scatter_free_agents=False, no_overlap_at_reset=False, result=None, maze=True):
        """MazePlacementState.reset (state.py:500-619) in every env, or with
        maze=False TargetBarriersFreePlacementState.reset (state.py:279-382)
        (gw_component GW_OP_MAZE_RESET); returns status int32[E] (1 placed)."""
        bits = lambda encs: sum(1 << int(x) for x in encs)
        args = torch.zeros((self.E, self.act_dim), dtype=torch.int32, device=self.device)
        args[:, 0] = (int(bool(no_overlap_at_reset)) | int(bool(cluster_barriers)) << 1 |
                      int(bool(scatter_free_agents)) << 2 | int(not maze) << 3 | int(target) << 8)
        args[:, 1] = bits(barrier_encodings)
        args[:, 2] = bits(free_encodings)
        res = result if result is not None else \
            torch.zeros((self.E, 2 + self.A), dtype=torch.int32, device=self.device)
        self.component(_abi.GW_OP_MAZE_RESET, -1, args, res)
        return res[:, 0]

    def generate_maze(self, start=None, out=None):
        """generate_maze(rows, cols, start) (utils.py:120-212) in every env on
        its own np.random stream: int8[E][rows][cols], 0 passage / 1 wall.
        start: int32[E][2] device tensor (a negative row = None) or None."""
        H, W = self.cc.rows, self.cc.cols
        out = out if out is not None else torch.empty((self.E, H, W), dtype=torch.int8, device=self.device)
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_generate_maze(self.h, _ptr(start), _ptr(out), _stream()),
                          'gw_generate_maze')
        return out

    def move(self, lane, moves):
        """MoveActor.process_action for entity `lane` in every env (batched):
        moves int32[E][2]; returns status int32[E] (1 True, 0 False, -1 None)."""
        args = torch.zeros((self.E, self.act_dim), dtype=torch.int32, device=self.device)
        args[:, :2] = moves
        res = torch.zeros((self.E, 2 + self.A), dtype=torch.int32, device=self.device)
        self.component(_abi.GW_OP_MOVE, lane, args, res)
        return res[:, 0]

    def attack(self, lane, attack):
        """The attack actor's process_action for entity `lane` in every env:
        attack int32[E] (binary) or int32[E][(2r+1)^2] (selective); returns
        (status int32[E], n int32[E], attacked lanes int32[E][A])."""
        args = torch.zeros((self.E, self.act_dim), dtype=torch.int32, device=self.device)
        a = torch.as_tensor(attack, dtype=torch.int32, device=self.device).reshape(self.E, -1)
        args[:, 2:2 + a.shape[1]] = a
        res = torch.zeros((self.E, 2 + self.A), dtype=torch.int32, device=self.device)
        self.component(_abi.GW_OP_ATTACK, lane, args, res)
        return res[:, 0], res[:, 1], res[:, 2:]

    def observe_lane(self, lane):
        """PositionCenteredEncodingObserver.get_obs(lane) in every env (draws in
        call order): writes and returns obs[:, lane]."""
        self.component(_abi.GW_OP_OBSERVE, lane, obs=self.obs)
        return self.obs[:, lane]

    def set_placement_order(self, lane_order):
        """The lane order the next resets place in, per env (int[E][A]; None
        = agents-dict order): PositionState(randomize_placement_order=True)."""
        if lane_order is None:
            _native.check(self.L.gw_set_placement_order(self.h, None, 0), 'gw_set_placement_order')
            self.kernel = int(self.L.gw_env_kernel(self.h))
            return
        o = np.ascontiguousarray(np.asarray(lane_order, dtype=np.int32).reshape(self.E, self.A))
        _native.check(self.L.gw_set_placement_order(self.h, o.ctypes.data_as(C.c_void_p), o.size),
                      'gw_set_placement_order')
        self.kernel = int(self.L.gw_env_kernel(self.h))

    def set_action_order(self, lane_order):
        """The lane order of the action dict the next steps process, per env
        (int[E][A]; None = agents-dict order):
        AllStepManager(randomize_action_input=True)."""
        if lane_order is None:
            _native.check(self.L.gw_set_action_order(self.h, None, 0), 'gw_set_action_order')
            return
        o = np.ascontiguousarray(np.asarray(lane_order, dtype=np.int32).reshape(self.E, self.A))
        _native.check(self.L.gw_set_action_order(self.h, o.ctypes.data_as(C.c_void_p), o.size),
                      'gw_set_action_order')

    def rollout_buffers(self, n_steps):
        """Per-step output slabs for rollout(): obs[n][E][A][...], reward[n][E][A],
        done[n][E][A], all_done[n][E]."""
        E, A, dev = self.E, self.A, self.device
        return dict(obs=torch.empty((n_steps, E, A) + self.obs_shape, dtype=torch.int32, device=dev),
                    reward=torch.empty((n_steps, E, A), dtype=torch.float64, device=dev),
                    done=torch.empty((n_steps, E, A), dtype=torch.uint8, device=dev),
                    all_done=torch.empty((n_steps, E), dtype=torch.uint8, device=dev))

    def _check_rollout_buffers(self, K, out):
        """Every slab of `out` holds >= K steps of this engine's shape, on its
        device (checked when the cached launch arguments change, and for a
        fragment longer than the slabs last checked)."""
        E, A = self.E, self.A
        want = dict(obs=((E, A) + self.obs_shape, torch.int32), reward=((E, A), torch.float64),
                    done=((E, A), torch.uint8), all_done=((E,), torch.uint8))
        for k, (shape, dt) in want.items():
            t = out[k]
            assert t.dtype == dt and t.is_contiguous() and t.device == self.device, (k, t.dtype, t.device)
            assert t.dim() == len(shape) + 1 and tuple(t.shape[1:]) == shape, (k, tuple(t.shape), shape)
            assert t.shape[0] >= K, f"rollout buffer {k!r} holds {t.shape[0]} steps < fragment {K}"
        self._rollout_cap = min(int(out[k].shape[0]) for k in want)

    _rollout_cap = 0

    def rollout(self, actions, horizon=0, autoreset='next_step', skip_done_obs=False, out=None):
        """A fragment of K = actions.shape[0] consecutive steps with auto-reset
        in ONE launch (gw_rollout): the results of K step_autoreset[_next]
        calls with actions[t], written to per-step slabs (returned dict, or
        `out` from rollout_buffers).  The '__all__' before step 0 is
        self.all_done (the previous call's); afterwards self.all_done holds
        the last step's.  skip_done_obs: obs rows of entities without an
        observation in a step are left unwritten (mask them with done)."""
        K = int(actions.shape[0])
        assert actions.dtype == torch.int32 and actions.is_contiguous()
        assert tuple(actions.shape[1:]) == tuple(self.actions.shape), actions.shape
        assert autoreset in ('same_step', 'next_step'), autoreset
        assert actions.device == self.device, (actions.device, self.device)
        out = self.rollout_buffers(K) if out is None else out
        if K > self._rollout_cap:
            self._check_rollout_buffers(K, out)
        # self.all_done is in/out: gw_rollout leaves the last step's __all__ in it
        if torch.cuda.current_device() == self.device.index:
            # the output / engine pointers and the stream are built once per
            # (out, stream): the host cost of a launch is one ctypes call
            s = torch.cuda.current_stream().cuda_stream
            c = getattr(self, '_rollout_args', None)
            key = (s, out['obs'].data_ptr(), out['reward'].data_ptr(), out['done'].data_ptr(),
                   out['all_done'].data_ptr())
            if c is None or c[0] != key:
                self._check_rollout_buffers(K, out)
                c = self._rollout_args = (
                    key, None, (_ptr(out['obs']), _ptr(out['reward']), _ptr(out['done']),
                                _ptr(out['all_done']), _ptr(self.all_done), _ptr(self.acting)),
                    (_ptr(self.err), C.c_void_p(s)))
            st = self.L.gw_rollout(self.h, K, C.c_void_p(actions.data_ptr()), *c[2], int(horizon),
                                   self.AUTORESET_MODES[autoreset], int(bool(skip_done_obs)), *c[3])
        else:
            self._check_rollout_buffers(K, out)
            with torch.cuda.device(self.device):
                st = self.L.gw_rollout(
                    self.h, K, _ptr(actions), _ptr(out['obs']), _ptr(out['reward']), _ptr(out['done']),
                    _ptr(out['all_done']), _ptr(self.all_done), _ptr(self.acting), int(horizon),
                    self.AUTORESET_MODES[autoreset], int(bool(skip_done_obs)), _ptr(self.err), _stream())
        _native.check(st, 'gw_rollout')
        self._check_debug('gw_rollout')
        return out

    def rollout_launcher(self, actions, horizon=0, autoreset='next_step', skip_done_obs=False, out=None,
                         events=None):
        """A prepared gw_rollout launch: the arguments of rollout(actions, ...)
        are validated and built once, on the current stream, and the returned
        zero-argument callable launches exactly that fragment with one ctypes
        call (a training loop re-launching the same slabs, or a benchmark's
        timed region).  It keeps references to `actions` and `out`.  With
        events=(start, stop), every launch records them as part of its kernel
        dispatch (gw_set_launch_events)."""
        K = int(actions.shape[0])
        assert actions.dtype == torch.int32 and actions.is_contiguous()
        assert tuple(actions.shape[1:]) == tuple(self.actions.shape), actions.shape
        assert autoreset in ('same_step', 'next_step'), autoreset
        assert actions.device == self.device, (actions.device, self.device)
        assert torch.cuda.current_device() == self.device.index, "launcher: the engine's device must be current"
        out = self.rollout_buffers(K) if out is None else out
        self._check_rollout_buffers(K, out)
        fn, h = self.L.gw_rollout, self.h
        args = (h, K, _ptr(actions), _ptr(out['obs']), _ptr(out['reward']), _ptr(out['done']),
                _ptr(out['all_done']), _ptr(self.all_done), _ptr(self.acting), int(horizon),
                self.AUTORESET_MODES[autoreset], int(bool(skip_done_obs)), _ptr(self.err), _stream())
        keep = (actions, out)
        arm = self._event_setter(events)

        def launch():
            if arm is not None:
                arm()
            st = fn(*args)
            if st != 0:
                _native.check(st, 'gw_rollout')
            return keep[1]
        return launch

    def rollout_step(self, key, step, env_offset=0, horizon=0, autoreset='next_step'):
        """One synthetic random-policy rollout step in ONE C-ABI call
        (gw_rollout_step: Philox actions into self.actions, then the step with
        the chosen auto-reset convention).  The pointer arguments are built
        once per engine, so the host cost per step is one ctypes call.
        Returns (obs, reward, done, all_done)."""
        args = getattr(self, '_roll_args', None)
        if args is None or args[0] != torch.cuda.current_stream().cuda_stream:
            s = torch.cuda.current_stream().cuda_stream
            args = self._roll_args = (s, _ptr(self.actions), _ptr(self.obs), _ptr(self.reward),
                                      _ptr(self.done), _ptr(self.all_done), _ptr(self.acting),
                                      _ptr(self.err), C.c_void_p(s))
        st = self.L.gw_rollout_step(self.h, int(key) & 0xFFFFFFFFFFFFFFFF, int(step) & 0xFFFFFFFF,
                                    int(env_offset) & 0xFFFFFFFF, *args[1:7], int(horizon),
                                    self.AUTORESET_MODES[autoreset], *args[7:9])
        if st != 0:
            _native.check(st, 'gw_rollout_step')
        return self.obs, self.reward, self.done, self.all_done

    def check_errors(self, allow=0):
        """Raise the reference's exception for the first env whose err flags
        (other than the `allow` bits) are set."""
        err = self.err.cpu().numpy() & ~np.uint32(allow)
        if (err & _abi.GW_ERR_NO_CELL).any():
            e = int(np.nonzero(err & _abi.GW_ERR_NO_CELL)[0][0])
            raise RuntimeError(f"Could not find a cell for an agent (env {e})")
        if (err & _abi.GW_ERR_INIT_POSITION).any():
            e = int(np.nonzero(err & _abi.GW_ERR_INIT_POSITION)[0][0])
            raise AssertionError(f"Initial cell not available (env {e})")
        if (err & _abi.GW_ERR_DOUBLE_REMOVE).any():
            e = int(np.nonzero(err & _abi.GW_ERR_DOUBLE_REMOVE)[0][0])
            raise KeyError(f"Grid.remove of an agent no longer in the grid (env {e}; "
                           f"reach_the_target.py:118-120)")
        if (err & _abi.GW_ERR_VALUE_ERROR).any():
            e = int(np.nonzero(err & _abi.GW_ERR_VALUE_ERROR)[0][0])
            raise ValueError(f"The truth value of an array with more than one element is ambiguous. "
                             f"Use a.any() or a.all() (env {e}: `not attacked_agents` on "
                             f"BinaryAttackActor's numpy array, team_battle_example.py:41)")

    # ------------------------------------------------------------ state
    def get_state(self):
        E, A, dev = self.E, self.A, self.device
        st = dict(pos=torch.zeros((E, A, 2), dtype=torch.int32, device=dev),
                  health=torch.zeros((E, A), dtype=torch.float64, device=dev),
                  flags=torch.zeros((E, A), dtype=torch.uint8, device=dev),
                  seq=torch.zeros((E, A), dtype=torch.int32, device=dev),
                  mt=torch.zeros((E, _abi.GW_MT_STRIDE), dtype=torch.int32, device=dev),
                  steps=torch.zeros((E,), dtype=torch.int32, device=dev))
        with torch.cuda.device(dev):
            _native.check(self.L.gw_get_state(self.h, *[_ptr(st[k]) for k in
                                                        ('pos', 'health', 'flags', 'seq', 'mt',
                                                         'steps')], _stream()), 'gw_get_state')
        return st

    def get_ammo(self):
        """AmmoAgent.ammo of every lane: int32[E][A] (0 for other lanes)."""
        out = torch.zeros((self.E, self.A), dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_get_ammo(self.h, _ptr(out), _stream()), 'gw_get_ammo')
        return out

    def set_ammo(self, ammo):
        a = torch.as_tensor(ammo, dtype=torch.int32, device=self.device).reshape(self.E, self.A).contiguous()
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_set_ammo(self.h, _ptr(a), _stream()), 'gw_set_ammo')
            torch.cuda.current_stream().synchronize()

    def set_state(self, pos=None, health=None, flags=None, seq=None, mt=None, steps=None):
        with torch.cuda.device(self.device):
            _native.check(self.L.gw_set_state(self.h, _ptr(pos), _ptr(health), _ptr(flags),
                                              _ptr(seq), _ptr(mt), _ptr(steps), _stream()),
                          'gw_set_state')
