"""Known answers for create_grid_and_mask (utils.py:5-117) from the REFERENCE
(run in this container): random grids with blocking agents around an
observer, the mask the reference returns for each.

Output: tests/golden/masks.npz -- per case the grid size, mask range, the
observer's and the blockers' cells (packed) and the reference's mask.
Run:  python tests/golden/make_masks.py      (needs /root/reference)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get('ABMARL_REFERENCE', '/root/reference')


def main(n=400, seed=0):
    sys.path.insert(0, HERE)
    import gym_stub
    gym_stub.install()
    sys.path.insert(0, REF)
    from abmarl.sim.gridworld.utils import create_grid_and_mask
    from abmarl.sim.gridworld.grid import Grid
    from abmarl.sim.gridworld.agent import GridWorldAgent
    rng = np.random.RandomState(seed)
    MAXB, MAXD = 8, 13
    meta = np.zeros((n, 4), np.int32)                 # rows, cols, mask range, n blockers
    cells = np.full((n, MAXB + 1), -1, np.int32)      # observer cell, then the blockers'
    masks = np.zeros((n, MAXD, MAXD), np.uint8)
    for k in range(n):
        R, C = rng.randint(3, 12), rng.randint(3, 12)
        nb, mr = rng.randint(1, MAXB), rng.randint(1, 7)
        cl = rng.choice(R * C, nb + 1, replace=False)
        grid = Grid(R, C)
        grid.reset()
        agents = {}
        for i, x in enumerate(cl):
            a = GridWorldAgent(id=f'a{i}', encoding=1, blocking=i > 0,
                               initial_position=np.array([x // C, x % C]))
            grid.place(a, (x // C, x % C))
            agents[a.id] = a
        _, m = create_grid_and_mask(agents['a0'], grid, mr, agents)
        meta[k] = (R, C, mr, nb)
        cells[k, :nb + 1] = cl
        masks[k, :2 * mr + 1, :2 * mr + 1] = m
    path = os.path.join(HERE, 'masks.npz')
    np.savez_compressed(path, meta=meta, cells=cells, masks=masks)
    print(f"masks: {n} cases -> {os.path.getsize(path)} B")


if __name__ == '__main__':
    main()
