"""Golden vectors for the ravel encoding: random points of the reference's
agent action spaces and the indices the REFERENCE's RavelDiscreteWrapper
assigns them (abmarl/sim/wrappers/ravel_discrete_wrapper.py:76-80).

Run:  python tests/golden/make_ravel.py      (needs /root/reference)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get('ABMARL_REFERENCE', '/root/reference')


def main():
    sys.path.insert(0, HERE)
    import gym_stub
    gym_stub.install()
    sys.path.insert(0, REF)
    from gym.spaces import Dict, Box, Discrete
    from abmarl.sim.wrappers.ravel_discrete_wrapper import ravel
    rng = np.random.RandomState(5)
    out = {}
    # TeamBattle BattleAgent: attack Discrete(2), move Box(-1, 1, (2,))
    tb = Dict({'attack': Discrete(2), 'move': Box(-1, 1, (2,), int)})
    pts = [(int(rng.randint(0, 2)), rng.randint(-1, 2, size=2)) for _ in range(64)]
    out['tb_points'] = np.array([[m[0], m[1], a] for a, m in pts], np.int64)
    out['tb_index'] = np.array([ravel(tb, {'attack': a, 'move': m}) for a, m in pts], np.int64)
    # TeamBattle with simultaneous_attacks 3 and move range 2
    tb2 = Dict({'attack': Discrete(4), 'move': Box(-2, 2, (2,), int)})
    pts = [(int(rng.randint(0, 4)), rng.randint(-2, 3, size=2)) for _ in range(64)]
    out['tb2_points'] = np.array([[m[0], m[1], a] for a, m in pts], np.int64)
    out['tb2_index'] = np.array([ravel(tb2, {'attack': a, 'move': m}) for a, m in pts], np.int64)
    # ReachTheTarget target: SelectiveAttackActor Box(0, 1, (3, 3))
    sel = Dict({'attack': Box(0, 1, (3, 3), int)})
    cells = rng.randint(0, 2, size=(64, 3, 3))
    out['sel_points'] = cells.reshape(64, 9).astype(np.int64)
    out['sel_index'] = np.array([ravel(sel, {'attack': c}) for c in cells], np.int64)
    # runner: move Box(-2, 2, (2,))
    run = Dict({'move': Box(-2, 2, (2,), int)})
    mv = rng.randint(-2, 3, size=(64, 2))
    out['run_points'] = mv.astype(np.int64)
    out['run_index'] = np.array([ravel(run, {'move': m}) for m in mv], np.int64)
    np.savez_compressed(os.path.join(HERE, 'ravel.npz'), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == '__main__':
    main()
