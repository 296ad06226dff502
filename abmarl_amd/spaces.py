"""Observation/action space descriptors.

The reference declares spaces with ``gym.spaces`` (Box/Discrete/Dict,
abmarl/tools/gym_utils.py:1-25); gym is not part of this stack, so the engine
ships minimal space classes with the same constructor signatures,
``contains``/``sample``/``seed`` and equality, enough for RLlib-style
duck typing (``MultiAgentWrapper.observation_space`` etc.).
"""
import numpy as np


class Space:
    def __init__(self, shape=None, dtype=None):
        self.shape = shape
        self.dtype = None if dtype is None else np.dtype(dtype)
        self._rng = np.random.RandomState()

    def seed(self, seed=None):
        self._rng = np.random.RandomState(seed)
        return [seed]

    def __contains__(self, x):
        return self.contains(x)


class Box(Space):
    """n-dimensional box; ``contains`` follows abmarl/tools/gym_utils.py:7-24."""

    def __init__(self, low, high, shape=None, dtype=np.float32):
        shape = tuple(shape) if shape is not None else np.shape(low)
        super().__init__(shape, dtype)
        lo = np.broadcast_to(np.asarray(low, dtype=np.float64), shape)
        hi = np.broadcast_to(np.asarray(high, dtype=np.float64), shape)
        # boundedness is judged before the cast (an int Box cannot hold inf)
        self.bounded_below = np.isfinite(lo)
        self.bounded_above = np.isfinite(hi)
        with np.errstate(invalid='ignore'):
            self.low = np.where(self.bounded_below, lo, 0).astype(self.dtype) \
                if np.issubdtype(self.dtype, np.integer) else lo.astype(self.dtype)
            self.high = np.where(self.bounded_above, hi, 0).astype(self.dtype) \
                if np.issubdtype(self.dtype, np.integer) else hi.astype(self.dtype)

    def contains(self, x):
        if type(x) is int:
            x = np.array([x], dtype=int)
        elif type(x) is float:
            x = np.array([x], dtype=float)
        elif not isinstance(x, np.ndarray):
            x = np.asarray(x, dtype=self.dtype)
        return bool(np.can_cast(x.dtype, self.dtype) and x.shape == self.shape and
                    np.all(x >= self.low) and np.all(x <= self.high))

    def sample(self):
        if np.issubdtype(self.dtype, np.integer):
            return self._rng.randint(self.low, self.high + 1, size=self.shape).astype(self.dtype)
        return self._rng.uniform(self.low, self.high, size=self.shape).astype(self.dtype)

    def __eq__(self, other):
        return isinstance(other, Box) and self.shape == other.shape and \
            np.allclose(self.low, other.low) and np.allclose(self.high, other.high)

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


class Discrete(Space):
    def __init__(self, n):
        super().__init__((), np.int64)
        self.n = int(n)

    def contains(self, x):
        try:
            return int(x) == x and 0 <= int(x) < self.n
        except (TypeError, ValueError):
            return False

    def sample(self):
        return int(self._rng.randint(self.n))

    def __eq__(self, other):
        return isinstance(other, Discrete) and self.n == other.n

    def __repr__(self):
        return f"Discrete({self.n})"


class MultiDiscrete(Space):
    """Vector of discrete values, element i in [0, nvec[i])."""

    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        super().__init__(self.nvec.shape, np.int64)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.nvec.shape and bool(np.all((0 <= x) & (x < self.nvec)))

    def sample(self):
        return (self._rng.random_sample(self.nvec.shape) * self.nvec).astype(np.int64)

    def __eq__(self, other):
        return isinstance(other, MultiDiscrete) and np.array_equal(self.nvec, other.nvec)

    def __repr__(self):
        return f"MultiDiscrete({self.nvec.tolist()})"


class MultiBinary(Space):
    def __init__(self, n):
        super().__init__((n,), np.int8)
        self.n = n

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all((x == 0) | (x == 1)))

    def sample(self):
        return self._rng.randint(0, 2, size=self.shape).astype(np.int8)

    def __eq__(self, other):
        return isinstance(other, MultiBinary) and self.n == other.n


class Dict(Space):
    """Keys are kept sorted, like gym's Dict."""

    def __init__(self, spaces=None, **kwargs):
        spaces = dict(spaces or {}, **kwargs)
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

    def keys(self):
        return self.spaces.keys()

    def values(self):
        return self.spaces.values()

    def items(self):
        return self.spaces.items()

    def seed(self, seed=None):
        for i, s in enumerate(self.spaces.values()):
            s.seed(None if seed is None else seed + i)
        return [seed]

    def contains(self, x):
        return isinstance(x, dict) and set(x) == set(self.spaces) and \
            all(s.contains(x[k]) for k, s in self.spaces.items())

    def sample(self):
        return {k: s.sample() for k, s in self.spaces.items()}

    def __eq__(self, other):
        return isinstance(other, Dict) and self.spaces == other.spaces

    def __repr__(self):
        return "Dict(" + ", ".join(f"{k}: {v}" for k, v in self.spaces.items()) + ")"


class Tuple(Space):
    """Ordered product of spaces (gym's Tuple)."""

    def __init__(self, spaces):
        self.spaces = tuple(spaces)
        super().__init__(None, None)

    def __getitem__(self, i):
        return self.spaces[i]

    def __len__(self):
        return len(self.spaces)

    def __iter__(self):
        return iter(self.spaces)

    def seed(self, seed=None):
        for i, s in enumerate(self.spaces):
            s.seed(None if seed is None else seed + i)
        return [seed]

    def contains(self, x):
        if isinstance(x, list):
            x = tuple(x)
        return isinstance(x, tuple) and len(x) == len(self.spaces) and \
            all(s.contains(p) for s, p in zip(self.spaces, x))

    def sample(self):
        return tuple(s.sample() for s in self.spaces)

    def __eq__(self, other):
        return isinstance(other, Tuple) and self.spaces == other.spaces

    def __repr__(self):
        return "Tuple(" + ", ".join(map(repr, self.spaces)) + ")"


def check_space(space, strict=False):
    """abmarl/tools/gym_utils.py:27-51."""
    if isinstance(space, (Box, Discrete, MultiDiscrete, MultiBinary)):
        return True
    if isinstance(space, Dict):
        return all(check_space(s) for s in space.spaces.values())
    if isinstance(space, Tuple):
        return all(check_space(s) for s in space.spaces)
    if not strict and isinstance(space, dict):
        return all(check_space(s) for s in space.values())
    if not strict and isinstance(space, tuple):
        return all(check_space(s) for s in space)
    return False


def make_dict(space):
    """abmarl/tools/gym_utils.py:54-66."""
    assert isinstance(space, (dict, Space)), "Cannot convert this to a Dict."
    for key, sub in list(space.items()):
        if isinstance(sub, dict):
            space[key] = make_dict(sub)
        else:
            assert isinstance(sub, Space), "Cannot convert this to a Dict."
    return Dict(space) if type(space) is dict else space
