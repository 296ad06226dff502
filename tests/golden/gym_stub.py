"""Minimal ``gym.spaces`` stand-in used ONLY by make_golden.py to import the
reference in this container (gym is not installed here).

The reference uses gym solely to declare observation/action spaces
(Box/Discrete/Dict, abmarl/sim/gridworld/{actor,observer}.py constructors and
agent_based_simulation.py:106-118 finalize); no step, reset or RNG logic of the
hot path touches these classes.  Space sampling/seeding is a no-op here: the
golden runs feed explicit actions.
"""
import sys
import types

import numpy as np


def install():
    if 'gym' in sys.modules:
        return
    gym = types.ModuleType('gym')
    spaces = types.ModuleType('gym.spaces')
    box_mod = types.ModuleType('gym.spaces.box')

    class Space:
        def __init__(self, shape=None, dtype=None):
            self.shape = shape
            self.dtype = dtype

        def seed(self, seed=None):
            return [seed]

        def __contains__(self, x):
            return self.contains(x)

    class Box(Space):
        def __init__(self, low, high, shape=None, dtype=np.float32):
            shape = tuple(shape) if shape is not None else np.shape(low)
            super().__init__(shape, np.dtype(dtype))
            self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), shape).copy()
            self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), shape).copy()

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low)) and \
                bool(np.all(x <= self.high))

        def is_bounded(self, manner='both'):
            return True

        def __eq__(self, other):
            return isinstance(other, Box) and self.shape == other.shape and \
                np.array_equal(self.low, other.low) and np.array_equal(self.high, other.high)

    class Discrete(Space):
        def __init__(self, n):
            super().__init__((), np.int64)
            self.n = n

        def contains(self, x):
            return int(x) == x and 0 <= x < self.n

        def __eq__(self, other):
            return isinstance(other, Discrete) and self.n == other.n

    class MultiDiscrete(Space):
        def __init__(self, nvec):
            self.nvec = np.asarray(nvec)
            super().__init__(self.nvec.shape, np.int64)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= 0)) and bool(np.all(x < self.nvec))

    class MultiBinary(Space):
        def __init__(self, n):
            super().__init__((n,), np.int8)
            self.n = n

        def contains(self, x):
            return True

    class Dict(Space):
        def __init__(self, spaces=None, **kw):
            spaces = dict(spaces or {}, **kw)
            self.spaces = dict(sorted(spaces.items()))
            super().__init__(None, None)

        def __getitem__(self, k):
            return self.spaces[k]

        def __setitem__(self, k, v):
            self.spaces[k] = v

        def __iter__(self):
            return iter(self.spaces)

        def __len__(self):
            return len(self.spaces)

        def items(self):
            return self.spaces.items()

        def keys(self):
            return self.spaces.keys()

        def values(self):
            return self.spaces.values()

        def contains(self, x):
            return isinstance(x, dict) and all(k in x and s.contains(x[k])
                                               for k, s in self.spaces.items())

        def __eq__(self, other):
            return isinstance(other, Dict) and self.spaces == other.spaces

    class Tuple(Space):
        def __init__(self, spaces):
            self.spaces = tuple(spaces)
            super().__init__(None, None)

    class Env:
        pass

    for name, obj in dict(Space=Space, Box=Box, Discrete=Discrete, MultiDiscrete=MultiDiscrete,
                          MultiBinary=MultiBinary, Dict=Dict, Tuple=Tuple).items():
        setattr(spaces, name, obj)
    box_mod.Box = Box
    box_mod.get_inf = lambda dtype, sign: np.inf
    spaces.box = box_mod
    gym.spaces = spaces
    gym.Env = Env
    sys.modules['gym'] = gym
    sys.modules['gym.spaces'] = spaces
    sys.modules['gym.spaces.box'] = box_mod
