"""Compile a host-side GridWorld simulation into the engine's gw_config.

Every value the reference reads from Python objects inside its step loop is
lowered here, once, to constant tables:
  agents dict order          -> entity index (the reference iterates dicts in
                                insertion order everywhere: team_battle_example.py:35,
                                all_step_manager.py:68-83)
  isinstance checks          -> kind bits (GW_K_*)
  Grid.overlapping (sym.)    -> overlap bitmask per encoding (grid.py:53-71,95-103)
  attack_mapping             -> bitmask per encoding (actor.py:385)
  component flags            -> stacked_attacks / observe_self / no_overlap_at_reset
  SmartGWS._states set order -> state_order (pinned)
"""
from abmarl_amd import _abi
from abmarl_amd.sim.agent_based_simulation import ObservingAgent, ActingAgent
from abmarl_amd.sim.gridworld.agent import (
    GridWorldAgent, GridObservingAgent, MovingAgent, AttackingAgent, HealthAgent, OrientationAgent,
    AmmoAgent)
from abmarl_amd.sim.gridworld.components import (
    PositionState, HealthState, OrientationState, AmmoState, _TargetPlacementState,
    BinaryAttackActor, SelectiveAttackActor,
    PositionCenteredEncodingObserver, AbsoluteEncodingObserver, ActiveDone, OneTeamRemainingDone,
    TargetAgentDone, TargetDestroyedDone, MoveActor, DriftMoveActor)


class UnsupportedConfig(ValueError):
    pass


def agent_spec(agent, program_type=None, food_type=None):
    kind = 0
    if program_type is not None and isinstance(agent, program_type):
        kind |= _abi.GW_K_PROGRAM
    if food_type is not None and isinstance(agent, food_type):
        kind |= _abi.GW_K_FOOD
    if isinstance(agent, OrientationAgent):
        kind |= _abi.GW_K_ORIENTATION
    if isinstance(agent, ObservingAgent):
        kind |= _abi.GW_K_OBSERVING
    if isinstance(agent, ActingAgent):
        kind |= _abi.GW_K_ACTING
    if isinstance(agent, GridObservingAgent):
        kind |= _abi.GW_K_GRID_OBSERVER
    if isinstance(agent, MovingAgent):
        kind |= _abi.GW_K_MOVING
    if isinstance(agent, AttackingAgent):
        kind |= _abi.GW_K_ATTACKING
    if isinstance(agent, HealthAgent):
        kind |= _abi.GW_K_HEALTH
    if agent.blocking:
        kind |= _abi.GW_K_BLOCKING
    if isinstance(agent, AmmoAgent):
        kind |= _abi.GW_K_AMMO
    s = _abi.AgentSpec()
    s.encoding = agent.encoding
    s.kind = kind
    if agent.initial_position is not None:
        s.init_row, s.init_col = int(agent.initial_position[0]), int(agent.initial_position[1])
    else:
        s.init_row = s.init_col = -1
    s.view_range = getattr(agent, 'view_range', 0) or 0
    s.move_range = getattr(agent, 'move_range', 0) or 0
    s.attack_range = getattr(agent, 'attack_range', 0) or 0
    s.simultaneous_attacks = getattr(agent, 'simultaneous_attacks', 0) or 0
    s.attack_strength = float(getattr(agent, 'attack_strength', 0) or 0)
    s.attack_accuracy = float(getattr(agent, 'attack_accuracy', 0) or 0)
    ih = getattr(agent, 'initial_health', None)
    s.initial_health = -1.0 if ih is None else float(ih)
    s.initial_orientation = int(getattr(agent, 'initial_orientation', None) or 0)
    s.initial_ammo = int(agent.initial_ammo) if isinstance(agent, AmmoAgent) else 0
    return s


# the component methods a fused program (and the component API) runs as
# device code: the public ones and the reference's protected hooks they call
# (actor.py:363-417 attack criteria / subset / determination, state.py:116-152
# placement lists and placement)
_DEVICE_METHODS = ('reset', 'process_action', 'get_obs', 'get_done', 'get_all_done',
                   '_basic_criteria', '_subset_attackables', '_determine_attack',
                   '_build_available_positions', '_update_available_positions',
                   '_place_initial_position_agent', '_place_variable_position_agent')


def _overridden(obj, builtins):
    """The device methods a subclass of a built-in component overrides: the
    program would run the built-in's device form and silently ignore them."""
    base = next((b for b in type(obj).__mro__ if b in builtins), None)
    if base is None or type(obj) is base:
        return []
    # (a hook the built-in does not define here is still the reference's
    # hook, which the device code implements: defining it is an override)
    return [m for m in _DEVICE_METHODS if getattr(type(obj), m, None) is not getattr(base, m, None)]


def compile_sim(sim, program, states, observers, dones, actors, state_order,
                nav_agent=-1, target_agent=-1, program_type=None, food_type=None,
                pacman_agent=-1, tunnel=(-1, -1, -1, -1), pac_rewards=(0, 0, 0, 0, 0)):
    """program_type: the sim program's own agent class (GW_K_PROGRAM bit),
    e.g. ReachTheTarget's RunningAgent or Pacman's BaddieAgent; food_type:
    Pacman's FoodAgent (GW_K_FOOD)."""
    agents = list(sim.agents.values())
    for a in agents:
        if not isinstance(a, GridWorldAgent):
            raise UnsupportedConfig(f"{a.id} is not a GridWorldAgent")
    n = len(agents)
    if n == 0:
        raise UnsupportedConfig("no agents")
    encs = [a.encoding for a in agents]
    if min(encs) < 1 or max(encs) > _abi.GW_MAX_ENC:
        raise UnsupportedConfig(f"encodings must be in 1..{_abi.GW_MAX_ENC}")
    if sim.grid.rows * sim.grid.cols > _abi.GW_MAX_CELLS:
        raise UnsupportedConfig(f"grid larger than {_abi.GW_MAX_CELLS} cells")

    builtins = (PositionState, HealthState, OrientationState, AmmoState, MoveActor, DriftMoveActor,
                BinaryAttackActor, SelectiveAttackActor, PositionCenteredEncodingObserver,
                AbsoluteEncodingObserver, ActiveDone, OneTeamRemainingDone, TargetAgentDone,
                TargetDestroyedDone)
    for x in list(states) + list(actors) + list(observers) + list(dones):
        if getattr(x, '_program_done', None) == program:
            continue                          # the sim program's own done component
        over = _overridden(x, builtins)
        if over:
            raise UnsupportedConfig(f"{type(x).__name__} overrides {', '.join(over)} of a built-in "
                                    "component: the engine (fused program and component API alike) "
                                    "runs the built-in's device code.  Write the behaviour as a "
                                    "component of your own, derived from the base component class "
                                    "(run on the host by the component runtime)")
    for s in states:
        if isinstance(s, _TargetPlacementState):
            raise UnsupportedConfig(f"{type(s).__name__} runs through the component API "
                                    "(a simulation without an engine program)")
        if not isinstance(s, (PositionState, HealthState, OrientationState, AmmoState)):
            raise UnsupportedConfig(f"{type(s).__name__} has no HIP implementation")
    pos_states = [s for s in states if isinstance(s, PositionState)]
    health_states = [s for s in states if isinstance(s, HealthState)]
    if len(pos_states) != 1:
        raise UnsupportedConfig("exactly one PositionState is required")
    if any(isinstance(a, HealthAgent) for a in agents) and not health_states:
        raise UnsupportedConfig("HealthAgents require a HealthState")
    if any(isinstance(a, AmmoAgent) and isinstance(a, AttackingAgent) for a in agents) and \
            not any(isinstance(s, AmmoState) for s in states):
        # without AmmoState.reset the agent has no ammo: the reference raises
        # AttributeError at its first attack (actor.py:346)
        raise UnsupportedConfig("attacking AmmoAgents require an AmmoState")
    if program == _abi.GW_SIM_PACMAN and any(isinstance(a, AmmoAgent) for a in agents):
        # pac_kernel keeps no ammo lane state (nothing in the Pacman program
        # attacks, so AmmoState.reset would be its only use)
        raise UnsupportedConfig("AmmoAgents have no HIP implementation in the Pacman program")

    obs_range = 0
    observe_self = True
    obs_kind = _abi.GW_OBS_POSITION_CENTERED
    pco = [o for o in observers if isinstance(o, PositionCenteredEncodingObserver)]
    aeo = [o for o in observers if isinstance(o, AbsoluteEncodingObserver)]
    if len(pco) + len(aeo) != len(observers) or len(observers) > 1:
        raise UnsupportedConfig("the engine implements one PositionCenteredEncodingObserver "
                                "or one AbsoluteEncodingObserver")
    if any(isinstance(s, OrientationState) for s in states) and program != _abi.GW_SIM_PACMAN:
        raise UnsupportedConfig("OrientationState runs in the Pacman program only")
    ranges = {a.view_range for a in agents if isinstance(a, GridObservingAgent)}
    if aeo:
        if program != _abi.GW_SIM_PACMAN:
            raise UnsupportedConfig("AbsoluteEncodingObserver runs in the Pacman program only")
        if any(a.blocking for a in agents):
            raise UnsupportedConfig("AbsoluteEncodingObserver with blocking entities has no HIP "
                                    "implementation")
        obs_kind = _abi.GW_OBS_ABSOLUTE
    elif pco:
        observe_self = pco[0].observe_self
        # different view ranges: each window top-left in a (2 max + 1)^2 slot
        obs_range = max(ranges) if ranges else 0
    if obs_range > _abi.GW_MAX_RANGE:
        raise UnsupportedConfig(f"view_range > {_abi.GW_MAX_RANGE}")

    attack = [x for x in actors if isinstance(x, (BinaryAttackActor, SelectiveAttackActor))]
    if len(attack) > 1:
        raise UnsupportedConfig("one attack actor per simulation")
    amap = {}
    stacked = False
    attack_kind = _abi.GW_ATTACK_BINARY
    if attack:
        stacked = attack[0].stacked_attacks
        if isinstance(attack[0], SelectiveAttackActor):
            attack_kind = _abi.GW_ATTACK_SELECTIVE
        for k, v in attack[0].attack_mapping.items():
            if 1 <= k <= _abi.GW_MAX_ENC:
                amap[k] = sum(1 << e for e in v if 1 <= e <= _abi.GW_MAX_ENC)
        for a in agents:
            if isinstance(a, AttackingAgent):
                if a.encoding not in attack[0].attack_mapping:
                    # the reference raises KeyError at actor.py:385 on the first candidate
                    raise UnsupportedConfig(f"{a.id}'s encoding is not in attack_mapping")
                if a.attack_range > _abi.GW_MAX_ATTACK_RANGE:
                    raise UnsupportedConfig(f"attack_range > {_abi.GW_MAX_ATTACK_RANGE}")
    for x in actors:
        if isinstance(x, DriftMoveActor) and program == _abi.GW_SIM_PACMAN:
            continue
        if not isinstance(x, (BinaryAttackActor, SelectiveAttackActor, MoveActor)):
            raise UnsupportedConfig(f"{type(x).__name__} has no HIP implementation")

    done_kind = 0
    ids = list(sim.agents)
    done_target = [-1] * n
    destroy_target = [-1] * n
    for d in dones:
        if getattr(d, '_program_done', None) == program:
            continue                          # decided by the sim program itself
        if isinstance(d, OneTeamRemainingDone):
            done_kind |= _abi.GW_DONE_ONE_TEAM
        elif isinstance(d, ActiveDone):
            done_kind |= _abi.GW_DONE_ACTIVE
        elif isinstance(d, (TargetAgentDone, TargetDestroyedDone)):
            if sum(isinstance(x, type(d)) for x in dones) > 1:
                raise UnsupportedConfig(f"one {type(d).__name__} per simulation")
            tgt = done_target if isinstance(d, TargetAgentDone) else destroy_target
            done_kind |= _abi.GW_DONE_TARGET_AGENT if isinstance(d, TargetAgentDone) \
                else _abi.GW_DONE_TARGET_DESTROYED
            for aid, tid in d.target_mapping.items():
                tgt[ids.index(aid)] = ids.index(tid)
            for i, a in enumerate(agents):
                if tgt[i] < 0 and isinstance(a, ObservingAgent) and isinstance(a, ActingAgent):
                    # get_done(agent) indexes target_mapping[agent.id] (done.py:91,131)
                    raise UnsupportedConfig(f"{a.id} is not in {type(d).__name__}.target_mapping "
                                            "(the reference raises KeyError in get_done)")
        else:
            raise UnsupportedConfig(f"{type(d).__name__} has no HIP implementation")
    # OneTeamRemainingDone.get_done is ActiveDone.get_done (done.py:140)
    order = {'position_health': _abi.GW_ORDER_POSITION_HEALTH,
             'health_position': _abi.GW_ORDER_HEALTH_POSITION}[state_order]
    specs = [agent_spec(a, program_type, food_type) for a in agents]
    for i, s in enumerate(specs):
        s.done_target, s.destroy_target = done_target[i], destroy_target[i]
    cc = _abi.CompiledConfig(
        sim.grid.rows, sim.grid.cols, specs,
        program,
        sim.grid.overlap_bits(), amap, stacked_attacks=stacked, observe_self=observe_self,
        no_overlap_at_reset=pos_states[0].no_overlap_at_reset, state_order=order,
        done_kind=done_kind, obs_range=obs_range, nav_agent=nav_agent, target_agent=target_agent,
        attack_kind=attack_kind, obs_kind=obs_kind, pacman_agent=pacman_agent, tunnel=tunnel,
        pac_rewards=pac_rewards)
    # PositionState(randomize_placement_order=True) (state.py:97-101): the
    # host shuffles with Python's random before each reset, exactly as the
    # reference does, and hands the order to the engine
    # (gw_set_placement_order; the dict-level API, one env per runtime)
    cc.randomize_placement_order = bool(pos_states[0].randomize_placement_order)
    # the reference's TeamBattle / ReachTheTarget steps raise ValueError when
    # BinaryAttackActor returns a numpy array of 2 or more agents (`not
    # attacked_agents`, team_battle_example.py:41); a simulation whose
    # `attack_array_as_list` is True opts into the list reading instead
    cc.cfg.attack_array_as_list = int(bool(getattr(sim, 'attack_array_as_list', False)))
    return cc
