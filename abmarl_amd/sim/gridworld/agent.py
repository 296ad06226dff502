"""GridWorld agent mixins (reference: abmarl/sim/gridworld/agent.py).

These are host-side descriptions.  The engine turns an agents dict into a
structure-of-arrays table (``gw_agent_spec``, include/gw_engine.h): encoding,
kind bits, ranges, attack strength/accuracy and initial position/health.  The
per-step values (position, health, active) live on the GPU; for the dict API
they are mirrored back onto these objects after every call.
"""
import numpy as np

from abmarl_amd.sim import host_version
from abmarl_amd.sim.agent_based_simulation import PrincipleAgent, ActingAgent, ObservingAgent


class GridWorldAgent(PrincipleAgent):
    """agent.py:7-119 — encoding (not -2/-1/0), initial_position, blocking."""

    def __init__(self, initial_position=None, blocking=False, encoding=None, render_shape='o',
                 render_color='gray', render_size=200, **kwargs):
        super().__init__(**kwargs)
        self.encoding = encoding
        self.initial_position = initial_position
        self.blocking = blocking
        self.render_shape = render_shape
        self.render_color = render_color
        self.render_size = render_size
        self.position = None

    @property
    def encoding(self):
        return self._encoding

    @encoding.setter
    def encoding(self, value):
        assert type(value) is int, f"{self.id}'s encoding must be an integer."
        assert value != -2, "-2 encoding reserved for masked observation."
        assert value != -1, "-1 encoding reserved for out of bounds."
        assert value != 0, "0 encoding reserved for empty cell."
        self._encoding = value

    @property
    def position(self):
        """The agent's position in the grid (agent.py:54-63)."""
        return self._position

    @position.setter
    def position(self, value):
        self._position = value
        host_version.bump()

    @property
    def initial_position(self):
        return self._initial_position

    @initial_position.setter
    def initial_position(self, value):
        if value is not None:
            assert type(value) is np.ndarray, "Initial position must be a numpy array."
            assert value.shape == (2,), "Initial position must be a 2-element array."
            assert value.dtype in [int, float], "Initial position must be numerical."
        self._initial_position = value

    @property
    def blocking(self):
        return self._blocking

    @blocking.setter
    def blocking(self, value):
        assert type(value) is bool, "Blocking must be either True or False."
        self._blocking = value

    @property
    def configured(self):
        return super().configured and self.encoding is not None and self.blocking is not None


class GridObservingAgent(ObservingAgent, GridWorldAgent):
    """agent.py:122-144."""

    def __init__(self, view_range=None, **kwargs):
        super().__init__(**kwargs)
        self.view_range = view_range

    @property
    def view_range(self):
        return self._view_range

    @view_range.setter
    def view_range(self, value):
        assert type(value) is int and 0 <= value, "View range must be a nonnegative integer."
        self._view_range = value

    @property
    def configured(self):
        return super().configured and self.view_range is not None


class MovingAgent(ActingAgent, GridWorldAgent):
    """agent.py:147-169."""

    def __init__(self, move_range=None, **kwargs):
        super().__init__(**kwargs)
        self.move_range = move_range

    @property
    def move_range(self):
        return self._move_range

    @move_range.setter
    def move_range(self, value):
        assert type(value) is int and 0 <= value, "Move range must be a nonnegative integer."
        self._move_range = value

    @property
    def configured(self):
        return super().configured and self.move_range is not None


class HealthAgent(GridWorldAgent):
    """agent.py:172-210 — health clamped to [0, 1]; active = health > 0."""

    def __init__(self, initial_health=None, **kwargs):
        super().__init__(**kwargs)
        self.initial_health = initial_health
        self._health = None

    @property
    def health(self):
        return self._health

    @health.setter
    def health(self, value):
        assert type(value) in [int, float], "Health must be a numeric value."
        self._health = min(max(value, 0), 1)
        self.active = self._health > 0

    @property
    def initial_health(self):
        return self._initial_health

    @initial_health.setter
    def initial_health(self, value):
        if value is not None:
            assert type(value) in [int, float], "Initial health must be a numeric value."
            assert 0 < value <= 1, "Initial health must be between 0 and 1."
        self._initial_health = value


class AttackingAgent(ActingAgent, GridWorldAgent):
    """agent.py:213-288."""

    def __init__(self, attack_range=None, attack_strength=None, attack_accuracy=None,
                 simultaneous_attacks=1, **kwargs):
        super().__init__(**kwargs)
        self.attack_range = attack_range
        self.attack_strength = attack_strength
        self.attack_accuracy = attack_accuracy
        self.simultaneous_attacks = simultaneous_attacks

    @property
    def attack_range(self):
        return self._attack_range

    @attack_range.setter
    def attack_range(self, value):
        assert type(value) is int and 0 <= value, "Attack range must be a nonnegative integer."
        self._attack_range = value

    @property
    def attack_strength(self):
        return self._attack_strength

    @attack_strength.setter
    def attack_strength(self, value):
        assert type(value) in [int, float], "Attack strength must be a numeric value."
        assert 0 <= value <= 1, "Attack strength must be between 0 and 1."
        self._attack_strength = value

    @property
    def attack_accuracy(self):
        return self._attack_accuracy

    @attack_accuracy.setter
    def attack_accuracy(self, value):
        assert type(value) in [int, float], "Attack accuracy must be a numeric value."
        assert 0 <= value <= 1, "Attack accuracy must be between 0 and 1."
        self._attack_accuracy = value

    @property
    def simultaneous_attacks(self):
        return self._simultaneous_attacks

    @simultaneous_attacks.setter
    def simultaneous_attacks(self, value):
        assert type(value) is int, "Simultaneous attacks must be an integer."
        assert value >= 0, "Simultaneous attacks must be nonnegative."
        self._simultaneous_attacks = value

    @property
    def configured(self):
        return super().configured and self.attack_range is not None and \
            self.attack_strength is not None and self.attack_accuracy is not None


class AmmoAgent(GridWorldAgent):
    """agent.py:291-322: a limited number of attacks; AmmoState.reset gives
    it initial_ammo, every attack spends what it lands (actor.py:343-351)."""

    def __init__(self, initial_ammo=None, **kwargs):
        super().__init__(**kwargs)
        self.initial_ammo = initial_ammo

    @property
    def ammo(self):
        return self._ammo

    @ammo.setter
    def ammo(self, value):
        assert type(value) is int, "Ammo must be an integer."
        self._ammo = 0 if value < 0 else value
        host_version.bump()

    @property
    def initial_ammo(self):
        return self._initial_ammo

    @initial_ammo.setter
    def initial_ammo(self, value):
        assert type(value) is int, "Initial ammo must be a an integer."
        self._initial_ammo = value


class _AmmoObservingMeta(type):
    def __instancecheck__(cls, instance):
        return isinstance(instance, ObservingAgent) and isinstance(instance, AmmoAgent)


class AmmoObservingAgent(AmmoAgent, ObservingAgent, metaclass=_AmmoObservingMeta):
    """agent.py:324-339: what AmmoObserver serves -- any agent that is both
    an ObservingAgent and an AmmoAgent counts as one (isinstance)."""


class OrientationAgent(GridWorldAgent):
    """agent.py:342-373: orientation 1 left, 2 down, 3 right, 4 up;
    initial_orientation None means random at reset (OrientationState)."""

    def __init__(self, initial_orientation=None, **kwargs):
        super().__init__(**kwargs)
        self.initial_orientation = initial_orientation
        self._orientation = None

    @property
    def orientation(self):
        return self._orientation

    @orientation.setter
    def orientation(self, value):
        assert value in range(1, 5), "Orientation must be 1, 2, 3, or 4."
        self._orientation = value

    @property
    def initial_orientation(self):
        return self._initial_orientation

    @initial_orientation.setter
    def initial_orientation(self, value):
        if value is not None:
            assert value in range(1, 5), "Initial orientation must be 1, 2, 3, or 4."
        self._initial_orientation = value
