"""Component registry (reference: abmarl/sim/gridworld/registry.py:14-77).

Only components the engine can execute are registered; ``register`` of any
other subclass raises, because the fused step cannot run arbitrary Python.
"""
from abmarl_amd.sim.gridworld.components import (
    ActorBaseComponent, MoveActor, CrossMoveActor, DriftMoveActor, BinaryAttackActor,
    SelectiveAttackActor, DoneBaseComponent, ActiveDone, OneTeamRemainingDone, TargetAgentDone,
    TargetDestroyedDone,
    ObserverBaseComponent, PositionCenteredEncodingObserver, AbsoluteEncodingObserver,
    StateBaseComponent, PositionState, MazePlacementState, TargetBarriersFreePlacementState,
    HealthState, OrientationState,
)

_subclass_check_mapping = {
    'actor': ActorBaseComponent,
    'done': DoneBaseComponent,
    'observer': ObserverBaseComponent,
    'state': StateBaseComponent,
}

_registered_components = {
    'actor': {MoveActor, CrossMoveActor, DriftMoveActor, BinaryAttackActor, SelectiveAttackActor},
    'done': {ActiveDone, OneTeamRemainingDone, TargetAgentDone, TargetDestroyedDone},
    'observer': {PositionCenteredEncodingObserver, AbsoluteEncodingObserver},
    'state': {PositionState, MazePlacementState, TargetBarriersFreePlacementState, HealthState,
              OrientationState},
}

registry = {
    kind: {c.__name__: c for c in comps} for kind, comps in _registered_components.items()
}


def register(component):
    """Register an engine-executable component under its type and class name."""
    for kind, base in _subclass_check_mapping.items():
        if issubclass(component, base):
            if not any(issubclass(component, c) for c in _registered_components[kind]):
                raise TypeError(
                    f"{component.__name__} has no HIP implementation; only subclasses of "
                    f"{sorted(c.__name__ for c in _registered_components[kind])} can run on the "
                    "engine.")
            _registered_components[kind].add(component)
            registry[kind][component.__name__] = component
            return
    raise TypeError(f"{component.__name__} must be an actor, done, state, or observer component.")
