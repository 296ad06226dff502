"""SmartGridWorldSimulation backed by the HIP engine.

Reference: abmarl/sim/gridworld/smart.py:10-120.  Components are given as sets
of registered names or classes exactly as in the reference.  Because the
reference stores the state components in a Python ``set`` (smart.py:37), the
order in which PositionState and HealthState draw from the RNG at reset is
set-iteration order there; here it is pinned by ``state_order``
('position_health' by default, or 'health_position').

Runtime (a subclass that names an engine program, ``_engine_program``): the
simulation compiles itself to a ``gw_config`` and runs on a one-env
``GridWorldEngine``.  A subclass with its own step() and no engine program
(a user-written simulation) runs as the reference's smart.py does: reset /
get_obs / get_done / get_all_done iterate its components, and each
component call is a device operation (component_runtime.py).  The engine fuses the AllStepManager protocol
(step -> obs -> rewards -> dones -> done_agents, all_step_manager.py:51-95)
into one kernel, so ``step`` computes every live agent's observation, reward
and done at once and ``get_obs`` / ``get_reward`` / ``get_done`` return those
results.  The global numpy legacy RNG (np.random) is carried through the
engine on every call (its MT19937 state is uploaded before and read back
after), so a sim driven by AllStepManager consumes and produces exactly what
the reference would from the same np.random.seed.
"""
from abc import ABC

import numpy as np

from abmarl_amd import _abi
from abmarl_amd.sim.agent_based_simulation import Agent
from abmarl_amd.sim.gridworld.base import GridWorldSimulation
from abmarl_amd.sim.gridworld.components import (
    StateBaseComponent, ObserverBaseComponent, DoneBaseComponent, ActorBaseComponent)
from abmarl_amd.sim.gridworld.registry import registry
from abmarl_amd.sim.gridworld.compile import compile_sim


def _build_components(items, kind, base, kwargs):
    assert type(items) is set, f"{kind.capitalize()}s must be a set of {kind} components"
    out = []
    # deterministic order: by class name (the reference's order is set order)
    resolved = []
    for item in items:
        if type(item) is str:
            assert item in registry[kind], f"{item} is not registered as a {kind}."
            resolved.append(registry[kind][item])
        elif isinstance(item, type) and issubclass(item, base):
            resolved.append(item)
        else:
            raise ValueError(f"{item} must be a {kind} component or the name of a registered "
                             f"{kind} component.")
    for cls in sorted(resolved, key=lambda c: c.__name__):
        out.append(cls(**kwargs))
    return out


class SmartGridWorldSimulation(GridWorldSimulation, ABC):
    # engine program implementing this class's step(); set by subclasses
    _engine_program = None

    def __init__(self, states=None, observers=None, dones=None, state_order='position_health',
                 device=None, **kwargs):
        super().__init__(**kwargs)
        self._states = _build_components(states, 'state', StateBaseComponent, kwargs) \
            if states else []
        self._observers = _build_components(observers, 'observer', ObserverBaseComponent,
                                            kwargs) if observers else []
        self._dones = _build_components(dones, 'done', DoneBaseComponent, kwargs) \
            if dones else []
        assert state_order in ('position_health', 'health_position'), \
            "state_order must be 'position_health' or 'health_position'"
        self.state_order = state_order
        self._device = device
        self._runtime = None
        self.rewards = {}

    # ------------------------------------------------------------ compile
    def _actors(self):
        return [v for v in vars(self).values() if isinstance(v, ActorBaseComponent)]

    def _program_extras(self):
        return {}

    def compiled(self):
        """This simulation as an engine configuration (_abi.CompiledConfig)."""
        assert self._engine_program is not None, \
            f"{type(self).__name__} has no engine step program"
        # the states of the sets, and those a subclass holds as attributes
        # (e.g. an AmmoState added to an example program) whose type the sets
        # do not already hold (an attribute twin of a set's PositionState is
        # the same component kind, reset once by the program)
        held = {type(s) for s in self._states}
        states = list(self._states) + [v for v in vars(self).values()
                                       if isinstance(v, StateBaseComponent) and v not in self._states
                                       and type(v) not in held]
        return compile_sim(self, self._engine_program, states, self._observers,
                           self._dones, self._actors(), self.state_order,
                           **self._program_extras())

    def _rt(self):
        if self._runtime is None:
            from abmarl_amd.sim.gridworld.runtime import DictRuntime
            self._runtime = DictRuntime(self, self.compiled(), self._device)
        return self._runtime

    # ------------------------------------------------------------ ABS API
    # (no engine program: the component path, smart.py:86-117 with every
    # component call on the device)
    def reset(self, **kwargs):
        assert self._states, "Smart Simulation requires '_states' attribute."
        if self._engine_program is None:
            # the reference iterates a set (smart.py:37); state_order pins it
            first = 'PositionState' if self.state_order == 'position_health' else 'HealthState'
            for state in sorted(self._states, key=lambda s: type(s).__name__ != first):
                state.reset(**kwargs)
        else:
            self._rt().reset()
        self.rewards = {a.id: 0 for a in self.agents.values() if isinstance(a, Agent)}

    def step(self, action_dict, **kwargs):
        assert self._engine_program is not None, \
            f"{type(self).__name__} has no engine program: implement step() with its components"
        self._rt().step(action_dict)

    def get_obs(self, agent_id, **kwargs):
        assert self._observers, "Smart Simulation requires '_observers' attribute."
        if self._engine_program is None:
            agent = self.agents[agent_id]
            return {k: v for observer in self._observers
                    for k, v in observer.get_obs(agent, **kwargs).items()}
        return self._rt().get_obs(agent_id)

    def get_reward(self, agent_id, **kwargs):
        if self._engine_program is None:
            reward = self.rewards[agent_id]
            self.rewards[agent_id] = 0
            return reward
        return self._rt().get_reward(agent_id)

    def get_done(self, agent_id, **kwargs):
        assert self._dones, "Smart Simulation requires '_dones' attribute."
        if self._engine_program is None:
            agent = self.agents[agent_id]
            return all(done.get_done(agent, **kwargs) for done in self._dones)
        return self._rt().get_done(agent_id)

    def get_all_done(self, **kwargs):
        assert self._dones, "Smart Simulation requires '_dones' attribute."
        if self._engine_program is None:
            return all(done.get_all_done(**kwargs) for done in self._dones)
        return self._rt().get_all_done()

    def get_info(self, agent_id, **kwargs):
        return {}

    @property
    def done_agents(self):
        """Agents the fused manager protocol considers done."""
        return self._rt().done_agents()

