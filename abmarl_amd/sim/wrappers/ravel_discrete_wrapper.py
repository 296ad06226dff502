"""Ravel discrete spaces into one Discrete index (reference:
abmarl/sim/wrappers/ravel_discrete_wrapper.py:13-191).

A space is a mixed-radix number: its components in order (Dict keys sorted,
Tuple order, array elements in C order), the first component most
significant — numpy's ravel_multi_index convention, as in the reference.
Radices: Discrete n; MultiDiscrete nvec; MultiBinary 2 per bit; bounded
integer Box high + 1 - low per element; a nested Dict/Tuple is one digit
whose radix is its own cardinality.

The batched GPU env decodes raveled actions on the device with the same
convention (abmarl_amd/external/rllib_multiagentenv_wrapper.py).
"""
import numpy as np

from abmarl_amd.spaces import Box, Discrete, MultiDiscrete, MultiBinary, Dict, Tuple
from abmarl_amd.sim.agent_based_simulation import Agent
from abmarl_amd.sim.wrappers.sar_wrapper import SARWrapper


def _parts(space):
    """(radix, sub-space or None) digits of one level of the space."""
    if isinstance(space, Discrete):
        return [(space.n, None)]
    if isinstance(space, MultiDiscrete):
        return [(int(n), None) for n in space.nvec.reshape(-1)]
    if isinstance(space, MultiBinary):
        return [(2, None)] * int(np.prod(space.shape))
    if isinstance(space, Box):
        return [(int(h) + 1 - int(lo), None)
                for lo, h in zip(space.low.reshape(-1), space.high.reshape(-1))]
    if isinstance(space, Dict):
        return [(cardinality(s), s) for s in space.spaces.values()]
    if isinstance(space, (Tuple, tuple, list)):
        return [(cardinality(s), s) for s in space]
    raise TypeError(f"{space} cannot be ravelled")


def cardinality(space):
    n = 1
    for r, _ in _parts(space):
        n *= r
    return n


def _digits(space, point):
    if isinstance(space, Discrete):
        return [int(point)]
    if isinstance(space, (MultiDiscrete, MultiBinary)):
        return [int(v) for v in np.asarray(point).reshape(-1)]
    if isinstance(space, Box):
        return [int(v) for v in (np.asarray(point) - space.low).reshape(-1)]
    if isinstance(space, Dict):
        return [ravel(s, point[k]) for k, s in space.spaces.items()]
    return [ravel(s, p) for s, p in zip(space, point)]


def ravel(space, point):
    """The index of `point` in `space`."""
    index = 0
    for (radix, _), d in zip(_parts(space), _digits(space, point)):
        index = index * radix + d
    return index


def unravel(space, index):
    """The point of `space` with this index."""
    parts = _parts(space)
    digits = []
    index = int(index)
    for radix, _ in reversed(parts):
        digits.append(index % radix)
        index //= radix
    digits.reverse()
    if isinstance(space, Discrete):
        return digits[0]
    if isinstance(space, (MultiDiscrete, MultiBinary)):
        return list(digits)
    if isinstance(space, Box):
        return np.reshape(np.array(digits), space.shape) + space.low
    if isinstance(space, Dict):
        return {k: unravel(s, d) for (k, s), d in zip(space.spaces.items(), digits)}
    return tuple(unravel(s, d) for s, d in zip(space, digits))


def ravel_space(space):
    return Discrete(cardinality(space))


def check_space(space):
    """True when the space can be ravelled (discrete or bounded integer Box)."""
    if isinstance(space, (Discrete, MultiDiscrete, MultiBinary)):
        return True
    if isinstance(space, Box):
        return np.issubdtype(space.dtype, np.integer) and bool(np.all(space.bounded_below)) \
            and bool(np.all(space.bounded_above))
    if isinstance(space, Dict):
        return all(check_space(s) for s in space.spaces.values())
    if isinstance(space, (Tuple, tuple, list)):
        return all(check_space(s) for s in space)
    return False


class RavelDiscreteWrapper(SARWrapper):
    """Discrete observations and actions for every Agent (ravel_discrete_wrapper.py:150-191)."""

    def __init__(self, sim):
        super().__init__(sim)
        for aid, agent in self.agents.items():
            if not isinstance(agent, Agent):
                continue
            assert check_space(agent.observation_space), f"{aid}: observation must be discretizable."
            assert check_space(agent.action_space), f"{aid} action must be discretizable."
            agent.observation_space = ravel_space(agent.observation_space)
            agent.action_space = ravel_space(agent.action_space)
            inner = self.sim.agents[aid]
            if getattr(agent, 'null_observation', None):
                agent.null_observation = ravel(inner.observation_space, agent.null_observation)
            if getattr(agent, 'null_action', None):
                agent.null_action = ravel(inner.action_space, agent.null_action)

    def wrap_observation(self, from_agent, observation):
        return ravel(from_agent.observation_space, observation)

    def unwrap_observation(self, from_agent, observation):
        return unravel(from_agent.observation_space, observation)

    def wrap_action(self, from_agent, action):
        return unravel(from_agent.action_space, action)

    def unwrap_action(self, from_agent, action):
        return ravel(from_agent.action_space, action)
