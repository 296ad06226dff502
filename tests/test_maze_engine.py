"""generate_maze and MazePlacementState on the device (gw_generate_maze,
gw_component GW_OP_MAZE_RESET; csrc/gw_maze.inc) against the reference's own
outputs (tests/golden/maze_gen.json, tests/golden/make_maze.py) and, at batch
sizes, against the C oracle env by env."""
import random

import numpy as np
import pytest
import torch

from abmarl_amd import _abi
from tests import maze_cases as mc

gpu = pytest.mark.gpu
DATA = mc.load()


def _mt_rows(seeds):
    from oracle import oracle
    mt = np.zeros((len(seeds), _abi.GW_MT_STRIDE), np.uint32)
    for i, s in enumerate(seeds):
        mt[i, :_abi.GW_MT_N + 1] = oracle.mt_state(int(s))
    mt[:, 626] = 0xFFFFFFFF
    return mt


def _engine(cc, E):
    from abmarl_amd.engine import GridWorldEngine
    cc.cfg.all_lanes = 1
    return GridWorldEngine(cc, E, seeds=list(range(E)))


def _maze_cc(rows, cols):
    from abmarl_amd.sim.gridworld.agent import GridWorldAgent
    from abmarl_amd.sim.gridworld.compile import agent_spec
    return _abi.CompiledConfig(rows, cols, [agent_spec(GridWorldAgent(id='m', encoding=1))],
                               _abi.GW_SIM_TEAM_BATTLE, {}, {})


@gpu
@pytest.mark.parametrize('k', range(len(DATA['mazes'])))
def test_generate_maze_reference(k):
    """Each fixture maze, in env 0 and env 2 of a 3-env batch (env 1 starts
    elsewhere with another seed); the MT19937 state after it too."""
    m = DATA['mazes'][k]
    eng = _engine(_maze_cc(m['rows'], m['cols']), 3)
    seeds = [m['seed'], m['seed'] + 17, m['seed']]
    eng.set_state(mt=torch.as_tensor(_mt_rows(seeds).view(np.int32), device=eng.device))
    st = [-1, -1] if m['start'] is None else m['start']
    start = torch.tensor([st, [-1, -1], st], dtype=torch.int32, device=eng.device)
    maze = eng.generate_maze(start).cpu().numpy()
    mt = eng.get_state()['mt'].cpu().numpy().view(np.uint32)
    for e in (0, 2):
        assert maze[e].reshape(-1).tolist() == m['maze']
        assert int(mt[e, 624]) == m['mt_pos'] and mc.mt_key_crc(mt[e]) == m['mt_crc']


@gpu
@pytest.mark.parametrize('rows,cols,E', [(16, 16, 1024), (31, 17, 256), (64, 64, 64)])
def test_generate_maze_vs_oracle_batched(rows, cols, E):
    from oracle import oracle
    rng = np.random.default_rng(rows * 100 + cols)
    seeds = rng.integers(0, 2**31, E)
    starts = np.stack([rng.integers(0, rows, E), rng.integers(0, cols, E)], 1).astype(np.int32)
    starts[::7] = -1                                   # start=None in every 7th env
    eng = _engine(_maze_cc(rows, cols), E)
    eng.set_state(mt=torch.as_tensor(_mt_rows(seeds).view(np.int32), device=eng.device))
    maze = eng.generate_maze(torch.as_tensor(starts, device=eng.device)).cpu().numpy()
    mt = eng.get_state()['mt'].cpu().numpy().view(np.uint32)
    for e in range(E):
        want_mt = oracle.mt_state(int(seeds[e]))
        st = None if starts[e, 0] < 0 else starts[e]
        want = oracle.generate_maze(rows, cols, st, want_mt)
        assert np.array_equal(maze[e], want), e
        assert np.array_equal(mt[e, :625], want_mt), e


@gpu
@pytest.mark.parametrize('name', [c['name'] for c in DATA['placements']] + [c['name'] for c in DATA['tbf']])
def test_maze_placement_state_reference(name):
    """The reference's MazePlacementState (and, tbf_*, TargetBarriersFree-
    PlacementState) resets through the component API (reset -> gw_component
    MAZE_RESET): positions, in-cell order, the exception raised and the
    numpy MT19937 state after each."""
    from abmarl_amd.sim.gridworld.components import MazePlacementState, TargetBarriersFreePlacementState
    if name.startswith('tbf_'):
        MazePlacementState = TargetBarriersFreePlacementState  # noqa: N806
    case = next(c for c in DATA['placements'] + DATA['tbf'] if c['name'] == name)
    agents, grid, _ = mc.build(case)
    ids = list(agents)
    state = MazePlacementState(
        grid=grid, agents=agents, target_agent=agents['target'],
        barrier_encodings=set(case['barrier']), free_encodings=set(case['free']),
        cluster_barriers=case.get('cluster', False), scatter_free_agents=case.get('scatter', False),
        no_overlap_at_reset=case.get('no_overlap', False),
        randomize_placement_order=case.get('randomize', False))
    random.seed(case['seed'])
    np.random.seed(case['seed'])
    for rec in case['resets_out']:
        raised = None
        try:
            state.reset()
        except AssertionError:
            raised = 'AssertionError'
        except RuntimeError:
            raised = 'RuntimeError'
        assert raised == rec['raised']
        if raised is None:
            got = []
            for aid in ids:
                a = agents[aid]
                r, c = int(a.position[0]), int(a.position[1])
                got.append([r, c, list(grid[r, c]).index(aid)])
            assert got == rec['cells']
        st = np.random.get_state()
        assert int(st[2]) == rec['mt_pos'] and mc.mt_key_crc(np.asarray(st[1], np.uint32)) == rec['mt_crc']


@gpu
def test_maze_placement_known_answers():
    """tests/sim/gridworld/test_state.py:487-577 (reference): np.random.seed(24),
    target at (3, 2), cluster + scatter: barriers within 2 cells of the
    target, all free agents on (1, 7); with no_overlap_at_reset every cell
    holds at most one agent."""
    from abmarl_amd.sim.gridworld.agent import GridWorldAgent
    from abmarl_amd.sim.gridworld.grid import Grid
    from abmarl_amd.sim.gridworld.components import MazePlacementState
    for no_overlap in (False, True):
        np.random.seed(24)
        target = GridWorldAgent(id='target', encoding=1, initial_position=np.array([3, 2]))
        barriers = {f'barrier_agent{i}': GridWorldAgent(id=f'barrier_agent{i}', encoding=2) for i in range(5)}
        frees = {f'free_agent{i}': GridWorldAgent(id=f'free_agent{i}', encoding=3) for i in range(5)}
        agents = {'target': target, **barriers, **frees}
        grid = Grid(5, 8, overlapping={1: {3}, 3: {3}})
        state = MazePlacementState(grid=grid, agents=agents, target_agent=target, barrier_encodings={2},
                                   free_encodings={1, 3}, cluster_barriers=True, scatter_free_agents=True,
                                   no_overlap_at_reset=no_overlap)
        state.reset()
        np.testing.assert_array_equal(target.position, np.array([3, 2]))
        if not no_overlap:
            for b in barriers.values():
                assert max(abs(target.position - b.position)) <= 2
            for f in frees.values():
                np.testing.assert_array_equal(f.position, np.array([1, 7]))
        else:
            for r in range(5):
                for c in range(8):
                    assert len(grid[r, c]) <= 1


@gpu
@pytest.mark.parametrize('name', ['multi_maze', 'cluster_scatter', 'scatter_only', 'both_sets', 'too_many',
                                  'tbf_multi_maze', 'tbf_cluster_scatter', 'tbf_basic', 'tbf_too_many'])
def test_maze_reset_batched_vs_oracle(name):
    """Batched MazePlacementState.reset (engine.maze_reset) at 512 envs, each
    on its own stream, three consecutive resets, env by env against the
    oracle: positions, placement order, error flags, MT19937 state."""
    from oracle import oracle
    case = next(c for c in DATA['placements'] + DATA['tbf'] if c['name'] == name)
    variant = int(name.startswith('tbf_'))
    _, _, cc = mc.build(case)
    E = 512
    ids = [a[0] for a in case['agents']]
    tgt = ids.index('target')
    eng = _engine(cc, E)
    seeds = np.arange(E) * 7919 + 11
    eng.set_state(mt=torch.as_tensor(_mt_rows(seeds).view(np.int32), device=eng.device))
    mts = [oracle.mt_state(int(s)) for s in seeds]
    kw = dict(cluster=case.get('cluster', False), scatter=case.get('scatter', False),
              no_overlap=case.get('no_overlap', False), variant=variant)
    for _ in range(3):
        eng.err.zero_()
        status = eng.maze_reset(tgt, case['barrier'], case['free'], cluster_barriers=kw['cluster'],
                                scatter_free_agents=kw['scatter'], no_overlap_at_reset=kw['no_overlap'],
                                maze=not variant)
        st = {k: v.cpu().numpy() for k, v in eng.get_state().items()}
        err = eng.err.cpu().numpy()
        status = status.cpu().numpy()
        mt = st['mt'].view(np.uint32)
        for e in range(E):
            want = oracle.maze_place(cc, tgt, case['barrier'], case['free'], mts[e], **kw)
            assert int(err[e]) == want['err'] and int(status[e]) == (0 if want['err'] else 1), e
            assert np.array_equal(mt[e, :625], mts[e]), e
            if want['err']:
                continue
            ing = (st['flags'][e] & _abi.FLAG_IN_GRID) != 0
            assert np.array_equal(ing, want['in_grid'] != 0), e
            assert np.array_equal(st['pos'][e], want['pos']), e
            assert np.array_equal(st['seq'][e], want['seq']), e


@gpu
def test_generate_maze_utility_reference():
    """abmarl_amd.sim.gridworld.utils.generate_maze (the reference's function,
    on the device) on the global np.random stream."""
    from abmarl_amd.sim.gridworld.utils import generate_maze
    for m in DATA['mazes'][:6]:
        np.random.seed(m['seed'])
        maze = generate_maze(m['rows'], m['cols'], None if m['start'] is None else np.array(m['start']))
        assert maze.astype(int).reshape(-1).tolist() == m['maze']
        st = np.random.get_state()
        assert int(st[2]) == m['mt_pos'] and mc.mt_key_crc(np.asarray(st[1], np.uint32)) == m['mt_crc']


def test_maze_placement_state_validation():
    """test_state.py:348-427 (reference): construction-time assertions."""
    from abmarl_amd.sim.gridworld.agent import GridWorldAgent
    from abmarl_amd.sim.gridworld.grid import Grid
    from abmarl_amd.sim.gridworld.components import MazePlacementState, PositionState
    target = GridWorldAgent(id='target', encoding=1)
    other = GridWorldAgent(id='other', encoding=1)
    agents = {'target': target, 'b': GridWorldAgent(id='b', encoding=2)}
    grid = Grid(5, 8, overlapping={1: {3}, 3: {3}})
    s = MazePlacementState(grid=grid, agents=agents, target_agent='target', barrier_encodings={2},
                           free_encodings={1, 3})
    assert isinstance(s, PositionState) and s.target_agent is target
    assert not s.cluster_barriers and not s.scatter_free_agents
    with pytest.raises(AssertionError):
        MazePlacementState(grid=grid, agents=agents, barrier_encodings={2}, free_encodings={1, 3})
    with pytest.raises(AssertionError):
        MazePlacementState(grid=grid, agents=agents, target_agent=other, barrier_encodings={2})
    with pytest.raises(AssertionError):
        MazePlacementState(grid=grid, agents=agents, target_agent='target_agent')
    with pytest.raises(AssertionError):
        MazePlacementState(grid=grid, agents=agents, target_agent=target, barrier_encodings=[2])
    with pytest.raises(AssertionError):
        MazePlacementState(grid=grid, agents=agents, target_agent=target, free_encodings=[1, 3])
    s = MazePlacementState(grid=grid, agents=agents, target_agent=target, free_encodings={1, 3})
    assert s.barrier_encodings == set()
    from abmarl_amd.sim.gridworld.registry import registry
    assert registry['state']['MazePlacementState'] is MazePlacementState


def _user_multi_maze_classes():
    """Test-side user code: a simulation written against this repository's
    component plugin API with the reference MultiMazeNavigation example's
    rules (abmarl/examples/sim/multi_maze_navigation.py:12-74): a
    MazePlacementState reset, MoveActor moves (-0.1 on a refused move,
    -0.01 every step), 1 as the reward of a navigator on the target, done
    when every navigator is there."""
    from abmarl_amd.sim.agent_based_simulation import Agent
    from abmarl_amd.sim.gridworld.base import GridWorldSimulation
    from abmarl_amd.sim.gridworld.agent import GridObservingAgent, MovingAgent
    from abmarl_amd.sim.gridworld.components import (
        MazePlacementState, MoveActor, PositionCenteredEncodingObserver)

    class Runner(GridObservingAgent, MovingAgent):
        def __init__(self, **kw):
            super().__init__(move_range=1, **kw)

    class MazeRunners(GridWorldSimulation):
        def __init__(self, **kw):
            super().__init__(**kw)
            self.placement = MazePlacementState(**kw)
            self.mover = MoveActor(**kw)
            self.observer = PositionCenteredEncodingObserver(**kw)
            self.finalize()

        def _arrived(self, aid):
            return np.array_equal(self.agents[aid].position, self.placement.target_agent.position)

        def reset(self, **kw):
            self.placement.reset(**kw)
            self.pending = dict.fromkeys((a.id for a in self.agents.values() if isinstance(a, Agent)), 0)

        def step(self, action_dict, **kw):
            for aid, act in action_dict.items():
                # two float64 subtractions in this order (not one of -0.11)
                if not self.mover.process_action(self.agents[aid], act, **kw):
                    self.pending[aid] -= 0.1
                self.pending[aid] -= 0.01

        def get_obs(self, aid, **kw):
            return dict(self.observer.get_obs(self.agents[aid], **kw))

        def get_reward(self, aid, **kw):
            r, self.pending[aid] = self.pending[aid], 0
            return 1 if self._arrived(aid) else r

        def get_done(self, aid, **kw):
            return self._arrived(aid)

        def get_all_done(self, **kw):
            return all(self._arrived(a.id) for a in self.agents.values() if isinstance(a, Runner))

        def get_info(self, aid, **kw):
            return {}

    return MazeRunners, Runner


@gpu
@pytest.mark.parametrize('k', range(len(DATA['trajectories'])))
def test_multi_maze_navigation_replays_reference(k):
    """The reference's MultiMazeNavigationSim example, rewritten as test-side
    user code on this repository's components (_user_multi_maze_classes),
    under AllStepManager: every observation, reward bit pattern, done,
    position and the MT19937 state after each step match the reference's
    own trajectory (episodes reset at __all__ or the horizon)."""
    from tests.golden.make_maze import build_multi_maze, multi_maze_actions
    from abmarl_amd.sim.gridworld.agent import GridWorldAgent
    MultiMazeNavigationSim, MultiMazeNavigationAgent = _user_multi_maze_classes()
    from abmarl_amd.managers import AllStepManager
    t = DATA['trajectories'][k]
    sim = build_multi_maze(t, MultiMazeNavigationSim, MultiMazeNavigationAgent, GridWorldAgent)
    man = AllStepManager(sim)
    np.random.seed(t['seed'])
    navs = [f'navigator{i}' for i in range(t['navigators'])]
    acts = multi_maze_actions(t)
    obs = man.reset()
    key = 'position_centered_encoding'
    for step, want in enumerate(t['steps_out']):
        where = f"{t['name']} step {step}"
        assert {a: np.asarray(o[key]).astype(int).tolist() for a, o in obs.items()} == want['obs'], where
        ad = {n: {'move': np.array(acts[step][i])} for i, n in enumerate(navs) if n not in man.done_agents}
        obs, rew, done, _ = man.step(ad)
        assert {a: np.float64(v).view(np.uint64).item() for a, v in rew.items()} == want['reward'], where
        assert {a: bool(v) for a, v in done.items()} == want['done'], where
        assert {a: np.asarray(x.position).astype(int).tolist() for a, x in sim.agents.items()} == want['pos'], where
        st = np.random.get_state()
        assert int(st[2]) == want['mt_pos'] and mc.mt_key_crc(np.asarray(st[1], np.uint32)) == want['mt_crc'], where
        if want['reset']:
            obs = man.reset()


def test_generate_maze_utility_validation():
    """tests/sim/gridworld/test_utils.py:18-31 (reference): argument checks
    (raised on the host, before any device work)."""
    from abmarl_amd.sim.gridworld.utils import generate_maze
    with pytest.raises(AssertionError):
        generate_maze(0, 4)
    with pytest.raises(AssertionError):
        generate_maze(3, -1)
    with pytest.raises(AssertionError):
        generate_maze(3, 3, [0, 1])
    with pytest.raises(AssertionError):
        generate_maze(3, 3, np.array([0]))
    with pytest.raises(IndexError):
        generate_maze(3, 3, np.array([6, 13]))


@gpu
def test_generate_maze_bad_start_on_device():
    """A start outside the maze through the C-ABI: that env's maze is all -1
    and its stream is untouched; the other envs are unaffected."""
    eng = _engine(_maze_cc(5, 5), 3)
    seeds = [3, 4, 5]
    eng.set_state(mt=torch.as_tensor(_mt_rows(seeds).view(np.int32), device=eng.device))
    start = torch.tensor([[1, 1], [5, 0], [2, 7]], dtype=torch.int32, device=eng.device)
    maze = eng.generate_maze(start).cpu().numpy()
    mt = eng.get_state()['mt'].cpu().numpy().view(np.uint32)
    assert (maze[1] == -1).all() and (maze[2] == -1).all()
    assert set(np.unique(maze[0])) <= {0, 1} and maze[0, 1, 1] == 0
    for e in (1, 2):
        assert np.array_equal(mt[e, :625], _mt_rows([seeds[e]])[0, :625])
