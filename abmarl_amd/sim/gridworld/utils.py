"""GridWorld utilities (reference: abmarl/sim/gridworld/utils.py).

generate_maze (utils.py:120-212) runs on the device: Prim's algorithm drawing
from the global np.random stream, with the frontier in CPython's
list(set(...)) order exactly as the reference (gw_generate_maze,
csrc/gw_maze.inc).  The numpy RNG state is handed to the engine before the
call and taken back after it, so the caller's stream advances by exactly the
reference's draws.

create_grid_and_mask (utils.py:5-117) is the host form for user-written
components (registry.register): the built-in components evaluate the same
masks on the device (shadow LUTs and shadow_hides in csrc/gw_engine.hip).
"""
import numpy as np
import torch

from abmarl_amd import _abi


def shadow_hidden(rd, cd, r, c):
    """Which window offsets (r, c) (integer arrays) a blocker at offset
    (rd, cd) hides: the cells strictly between the two rays from the
    observer's center through the blocker cell's corners, on the far side of
    the blocker (utils.py:46-115, the eight cases in the reference's float64
    arithmetic); never the blocker's own cell.  The device's shadow_hides is
    the same function."""
    r = np.asarray(r)
    c = np.asarray(c)
    if rd == 0 and cd == 0:
        return np.zeros(np.broadcast(r, c).shape, dtype=bool)
    rd_f, cd_f = float(rd), float(cd)
    if cd == 0:                                     # below / above: rays in c
        far = r >= rd if rd > 0 else r <= rd
        dd = -0.5 if rd > 0 else 0.5
        left = (cd_f - 0.5) / (rd_f + dd) * r
        right = (cd_f + 0.5) / (rd_f + dd) * r
        hide = far & (left < c) & (c < right)
    else:                                           # rays in r
        far = c >= cd if cd > 0 else c <= cd
        if rd > 0:
            far = far & (r >= rd)
        elif rd < 0:
            far = far & (r <= rd)
        if rd == 0:
            lo_d = up_d = -0.5 if cd > 0 else 0.5   # right / left
        elif (rd > 0) == (cd > 0):
            lo_d, up_d = 0.5, -0.5                  # below-right / above-left
        else:
            lo_d, up_d = -0.5, 0.5                  # below-left / above-right
        lo = (rd_f - 0.5) / (cd_f + lo_d) * c
        up = (rd_f + 0.5) / (cd_f + up_d) * c
        hide = far & (lo < r) & (r < up)
    return hide & ~((r == rd) & (c == cd))


def create_grid_and_mask(agent, grid, mask_range, agents):
    """The (2R+1)^2 local grid around the agent (grid cells, None off the
    grid) and its visibility mask (1 visible, 0 hidden behind an active
    blocking agent), as utils.py:5-117 returns them."""
    d = 2 * mask_range + 1
    local_grid = np.empty((d, d), dtype=object)
    r, c = agent.position
    r_lower, r_upper = max(0, r - mask_range), min(grid.rows - 1, r + mask_range) + 1
    c_lower, c_upper = max(0, c - mask_range), min(grid.cols - 1, c + mask_range) + 1
    local_grid[(r_lower + mask_range - r):(r_upper + mask_range - r),
               (c_lower + mask_range - c):(c_upper + mask_range - c)] = \
        grid[r_lower:r_upper, c_lower:c_upper]
    mask = np.ones((d, d))
    off = np.arange(-mask_range, mask_range + 1)
    rr, cc = np.meshgrid(off, off, indexing='ij')
    for other in agents.values():
        if other.active and other.blocking:
            rd, cd = other.position - agent.position
            if -mask_range <= rd <= mask_range and -mask_range <= cd <= mask_range:
                mask[shadow_hidden(int(rd), int(cd), rr, cc)] = 0
    return local_grid, mask

_engines = {}


def _engine(rows, cols):
    from abmarl_amd.engine import GridWorldEngine
    from abmarl_amd.sim.gridworld.agent import GridWorldAgent
    from abmarl_amd.sim.gridworld.compile import agent_spec
    eng = _engines.get((rows, cols))
    if eng is None:
        cc = _abi.CompiledConfig(rows, cols, [agent_spec(GridWorldAgent(id='maze', encoding=1))],
                                 _abi.GW_SIM_TEAM_BATTLE, {}, {})
        cc.cfg.all_lanes = 1
        eng = _engines[(rows, cols)] = GridWorldEngine(cc, 1, seeds=[0])
    return eng


def generate_maze(rows, cols, start=None):
    """A maze as a float array, 0 passage and 1 wall (utils.py:120-212)."""
    assert type(rows) is int and rows > 0, "Rows must be a positive integer."
    assert type(cols) is int and cols > 0, "Columns must be a positive integer."
    if start is not None:
        assert type(start) is np.ndarray, "Starting cell must be a numpy array."
        assert start.shape == (2,), "Starting cell must be a 2D coordinate."
        r, c = int(start[0]), int(start[1])
        if not (-(rows + 2) <= r + 1 < rows + 2 and -(cols + 2) <= c + 1 < cols + 2):
            # the reference's grid[tuple(start + 1)] = 0 on the bordered grid
            raise IndexError(f"index {[r + 1, c + 1]} is out of bounds for the bordered "
                             f"{rows + 2}x{cols + 2} maze grid")
        if not (0 <= r < rows and 0 <= c < cols):
            raise NotImplementedError("a start outside the maze (numpy's wrapped / border index) "
                                      "is not supported on the device")
    eng = _engine(rows, cols)
    st = np.random.get_state()
    assert st[0] == 'MT19937'
    mt = np.zeros((1, _abi.GW_MT_STRIDE), np.uint32)
    mt[0, :_abi.GW_MT_N] = st[1]
    mt[0, _abi.GW_MT_N] = st[2]
    eng.set_state(mt=torch.as_tensor(mt.view(np.int32), device=eng.device))
    s = None
    if start is not None:
        s = torch.tensor([[int(start[0]), int(start[1])]], dtype=torch.int32, device=eng.device)
    maze = eng.generate_maze(s)
    out = eng.get_state()['mt'].cpu().numpy().view(np.uint32)[0]
    np.random.set_state(('MT19937', out[:_abi.GW_MT_N].copy(), int(out[_abi.GW_MT_N])) + tuple(st[3:]))
    return maze[0].cpu().numpy().astype(float)
