"""The oracle's generate_maze / MazePlacementState restatement (gw_oracle.c)
against the reference's own outputs (tests/golden/maze_gen.json), and the
CPython set-order rule it restates against Python's set itself."""
import numpy as np
import pytest

from oracle import oracle
from tests import maze_cases as mc

DATA = mc.load()


@pytest.mark.parametrize('k', range(len(DATA['mazes'])))
def test_generate_maze_matches_reference(k):
    m = DATA['mazes'][k]
    mt = oracle.mt_state(m['seed'])
    maze = oracle.generate_maze(m['rows'], m['cols'], m['start'], mt)
    assert maze.reshape(-1).tolist() == m['maze']
    assert int(mt[624]) == m['mt_pos'] and mc.mt_key_crc(mt) == m['mt_crc']


def test_generate_maze_known_answer():
    """tests/sim/gridworld/test_utils.py:8-17 (reference): 5x9 from (1, 1):
    the start is a passage and no 2x2 block is all passages."""
    mt = oracle.mt_state(0)
    maze = oracle.generate_maze(5, 9, [1, 1], mt)
    assert maze.shape == (5, 9) and maze[1, 1] == 0
    for r in range(4):
        for c in range(8):
            assert maze[r:r + 2, c:c + 2].sum() > 0


@pytest.mark.parametrize('name', [c['name'] for c in DATA['placements']])
def test_maze_placement_matches_reference(name):
    case = next(c for c in DATA['placements'] if c['name'] == name)
    agents, grid, cc = mc.build(case)
    ids = list(agents)
    mt = oracle.mt_state(case['seed'])
    for rec in case['resets_out']:
        order = None if rec['order'] is None else [ids.index(a) for a in rec['order']]
        out = oracle.maze_place(cc, ids.index('target'), case['barrier'], case['free'], mt,
                                cluster=case.get('cluster', False), scatter=case.get('scatter', False),
                                no_overlap=case.get('no_overlap', False), order=order)
        assert mc.RAISED[out['err']] == rec['raised']
        if rec['raised'] is None:
            assert mc.cells_of(out['pos'], out['seq'], out['in_grid']) == rec['cells']
        assert int(mt[624]) == rec['mt_pos'] and mc.mt_key_crc(mt) == rec['mt_crc']


def test_set_order_rule_vs_python():
    """The frontier order the oracle restates (CPython's set of (row, col)
    tuples) against Python's own list(set(...)) for random cell lists of
    every size up to 3000 (table resizes included)."""
    rng = np.random.default_rng(0)
    for n in list(range(1, 80)) + [150, 400, 1000, 3000]:
        cols = int(rng.integers(3, 70))
        rows = max(3, (n + cols - 1) // cols + 2)
        cells = rng.permutation(rows * cols)[:n]
        want = [r * cols + c for r, c in list(set((int(x) // cols, int(x) % cols) for x in cells))]
        assert oracle.pyset_order(cells, cols) == want


@pytest.mark.parametrize('name', [c['name'] for c in DATA['tbf']])
def test_target_barriers_free_placement_matches_reference(name):
    """TargetBarriersFreePlacementState (state.py:169-382): the oracle's
    variant 1 against the reference's resets."""
    case = next(c for c in DATA['tbf'] if c['name'] == name)
    agents, grid, cc = mc.build(case)
    ids = list(agents)
    mt = oracle.mt_state(case['seed'])
    for rec in case['resets_out']:
        order = None if rec['order'] is None else [ids.index(a) for a in rec['order']]
        out = oracle.maze_place(cc, ids.index('target'), case['barrier'], case['free'], mt,
                                cluster=case.get('cluster', False), scatter=case.get('scatter', False),
                                no_overlap=case.get('no_overlap', False), order=order, variant=1)
        assert mc.RAISED[out['err']] == rec['raised']
        if rec['raised'] is None:
            assert mc.cells_of(out['pos'], out['seq'], out['in_grid']) == rec['cells']
        assert int(mt[624]) == rec['mt_pos'] and mc.mt_key_crc(mt) == rec['mt_crc']
