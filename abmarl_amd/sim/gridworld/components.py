"""State / Actor / Observer / Done components (the reference's plugin API).

Each class keeps the reference's name, constructor arguments, validation and
space assignment.  They run on the engine two ways:
  * as descriptors of the fused step programs (TeamBattleSim, ...): what each
    one contributes to the compiled configuration is in compile.py;
  * called directly, as the reference's components are by a user-written
    step(): PositionState / HealthState.reset, MoveActor / BinaryAttackActor /
    SelectiveAttackActor.process_action and PositionCenteredEncodingObserver
    .get_obs are device operations (gw_component, component_runtime.py) on
    the agents and the Grid they were built with; the done components read
    that state.

Reference: abmarl/sim/gridworld/state.py:13-166,622-656,659-675;
actor.py:13-234,237-501; observer.py:13-250; done.py:10-153.
"""
import random
from abc import ABC, abstractmethod

import numpy as np

from abmarl_amd import _abi
from abmarl_amd.spaces import Box, Discrete
from abmarl_amd.sim.gridworld.base import GridWorldBaseComponent
from abmarl_amd.sim.gridworld.component_runtime import ComponentRuntime, register_component
from abmarl_amd.sim.gridworld.agent import (
    GridWorldAgent, GridObservingAgent, MovingAgent, AttackingAgent, OrientationAgent, AmmoAgent)


class _EngineExecuted:
    def _engine_only(self, name):
        raise RuntimeError(
            f"{type(self).__name__}.{name} runs inside the fused HIP step; drive the simulation "
            "through its manager (AllStepManager / MultiAgentWrapper) or GridWorldEngine.")


# ----------------------------------------------------------------- states
class StateBaseComponent(GridWorldBaseComponent, _EngineExecuted, ABC):
    """state.py:13-22."""

    def reset(self, **kwargs):
        self._engine_only('reset')


class PositionState(StateBaseComponent):
    """state.py:25-166: initial positions first, then random cells drawn from
    per-encoding ordered availability lists (np.random.choice)."""

    def __init__(self, no_overlap_at_reset=False, randomize_placement_order=False, **kwargs):
        super().__init__(**kwargs)
        assert type(no_overlap_at_reset) is bool, "No overlap at reset must be a boolean."
        assert type(randomize_placement_order) is bool, \
            "Randomize placement order must be True or False."
        self.no_overlap_at_reset = no_overlap_at_reset
        self.randomize_placement_order = randomize_placement_order
        register_component(self)

    def reset(self, **kwargs):
        """Grid.reset, then every agent placed (gw_component POSITION_RESET)."""
        rt = ComponentRuntime.of(self)
        if self.randomize_placement_order:
            # state.py:97-101: random.shuffle of the agents dict's items, kept
            # for the next reset (Python's own random: the reference's draws)
            items = self.__dict__.setdefault('_place_items', list(self.agents))
            random.shuffle(items)
            rt.eng.set_placement_order([rt.index[aid] for aid in items if aid in rt.index])
        status, _, err = rt.op(_abi.GW_OP_POSITION_RESET, args=[int(self.no_overlap_at_reset)])
        if err & _abi.GW_ERR_INIT_POSITION:
            raise AssertionError("Cell is not available for an agent with an initial position.")
        if err & _abi.GW_ERR_NO_CELL or not status:
            raise RuntimeError("Could not find a cell for an agent")


class _TargetPlacementState(PositionState):
    """The constructor, properties and reset shared by the two target-relative
    placements (state.py:169-382, 385-619); _maze selects the variant."""

    _maze = False

    def __init__(self, target_agent=None, barrier_encodings=None, free_encodings=None,
                 cluster_barriers=False, scatter_free_agents=False, **kwargs):
        super().__init__(**kwargs)
        self.target_agent = target_agent
        self.barrier_encodings = barrier_encodings
        self.free_encodings = free_encodings
        self.cluster_barriers = cluster_barriers
        self.scatter_free_agents = scatter_free_agents

    @property
    def target_agent(self):
        return self._target_agent

    @target_agent.setter
    def target_agent(self, value):
        if type(value) is str:
            assert value in self.agents, "The target agent must be an agent in the simulation."
            value = self.agents[value]
        else:
            assert value in self.agents.values(), \
                "The target agent must be an agent in the simulation."
        assert isinstance(value, GridWorldAgent), "Target agent must be a GridWorld agent."
        self._target_agent = value

    @staticmethod
    def _encoding_set(value, what):
        if value is None:
            return set()
        assert type(value) is set, f"{what} encodings must be a set."
        for encoding in value:
            assert type(encoding) is int, f"Each {what.lower()} encoding must be an integer."
        return value

    @property
    def barrier_encodings(self):
        return self._barrier_encodings

    @barrier_encodings.setter
    def barrier_encodings(self, value):
        self._barrier_encodings = self._encoding_set(value, "Barrier")

    @property
    def free_encodings(self):
        return self._free_encodings

    @free_encodings.setter
    def free_encodings(self, value):
        self._free_encodings = self._encoding_set(value, "Free")

    @property
    def cluster_barriers(self):
        return self._cluster_barriers

    @cluster_barriers.setter
    def cluster_barriers(self, value):
        assert type(value) is bool, "Cluster barriers must be a boolean."
        self._cluster_barriers = value

    @property
    def scatter_free_agents(self):
        return self._scatter_free_agents

    @scatter_free_agents.setter
    def scatter_free_agents(self, value):
        assert type(value) is bool, "Scatter free agents must be a boolean."
        self._scatter_free_agents = value

    def reset(self, **kwargs):
        """Grid.reset, the maze from the target's cell (its initial position
        or np.random.randint(0, (rows, cols))), then every agent placed."""
        rt = ComponentRuntime.of(self)
        if self.randomize_placement_order:
            items = self.__dict__.setdefault('_place_items', list(self.agents))
            random.shuffle(items)
            rt.eng.set_placement_order([rt.index[aid] for aid in items if aid in rt.index])
        for agent in self.agents.values():
            assert agent.encoding in {*self.barrier_encodings, *self.free_encodings}, \
                "All agent encodings must be either barrier or free cell."
        bits = lambda encs: sum(1 << int(e) for e in encs)
        packed = (int(self.no_overlap_at_reset) | int(self.cluster_barriers) << 1 |
                  int(self.scatter_free_agents) << 2 | int(not self._maze) << 3 |
                  rt.index[self.target_agent.id] << 8)
        status, _, err = rt.op(_abi.GW_OP_MAZE_RESET,
                               args=[packed, bits(self.barrier_encodings), bits(self.free_encodings)])
        if err & _abi.GW_ERR_INIT_POSITION:
            raise AssertionError("Cell is not available for an agent with an initial position.")
        if err & _abi.GW_ERR_NO_CELL or not status:
            raise RuntimeError("Could not find a cell for an agent")


class TargetBarriersFreePlacementState(_TargetPlacementState):
    """state.py:169-382: the target placed first (its initial position or
    np.random.randint(0, (rows, cols))); barrier agents clustered near it,
    free agents scattered away from it (gw_component MAZE_RESET, variant 1:
    no maze, every cell available to both kinds)."""

    _maze = False


class MazePlacementState(_TargetPlacementState):
    """state.py:385-619: a maze generated around the target agent
    (generate_maze, utils.py:120-212) partitions the cells; barrier-encoded
    agents go on its walls, free-encoded ones on its passages
    (gw_component MAZE_RESET: maze and placement on the device)."""

    _maze = True


class HealthState(StateBaseComponent):
    """state.py:622-641: initial_health or np.random.uniform(0, 1)."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        register_component(self)

    def reset(self, **kwargs):
        """gw_component HEALTH_RESET."""
        ComponentRuntime.of(self).op(_abi.GW_OP_HEALTH_RESET)


class AmmoState(StateBaseComponent):
    """state.py:644-656: every AmmoAgent gets its initial_ammo.  No draw, so
    its place among the states changes nothing; the engine's programs run it
    inside their fused reset, and called directly it sets the agents (the
    component runtime uploads the ammo with the next device operation)."""

    def reset(self, **kwargs):
        for agent in self.agents.values():
            if isinstance(agent, AmmoAgent):
                agent.ammo = agent.initial_ammo


class OrientationState(StateBaseComponent):
    """state.py:659-675: initial_orientation or np.random.randint(1, 5)."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        register_component(self)

    def reset(self, **kwargs):
        """gw_component ORIENT_RESET: the draws on the device, in agent order."""
        rt = ComponentRuntime.of(self)
        rt.op(_abi.GW_OP_ORIENT_RESET)
        res = rt.last_result
        for aid, agent in self.agents.items():
            if isinstance(agent, OrientationAgent):
                agent.orientation = int(res[2 + rt.index[aid]])


# ----------------------------------------------------------------- actors
class ActorBaseComponent(GridWorldBaseComponent, _EngineExecuted, ABC):
    """actor.py:13-52."""

    def process_action(self, agent, action_dict, **kwargs):
        self._engine_only('process_action')

    @property
    @abstractmethod
    def key(self):
        pass

    @property
    @abstractmethod
    def supported_agent_type(self):
        pass


class MoveActor(ActorBaseComponent):
    """actor.py:55-114: action space Box(-move_range, move_range, (2,), int)."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        for agent in self.agents.values():
            if isinstance(agent, self.supported_agent_type):
                agent.action_space[self.key] = Box(-agent.move_range, agent.move_range, (2,), int)
                agent.null_action[self.key] = np.zeros((2,), dtype=int)
        register_component(self)

    def process_action(self, agent, action_dict, **kwargs):
        """True if the move succeeded (gw_component MOVE); None for agents that
        are not MovingAgents (actor.py:82-114)."""
        if not isinstance(agent, self.supported_agent_type):
            return None
        status, _, err = ComponentRuntime.of(self).op(_abi.GW_OP_MOVE, agent,
                                                      np.asarray(action_dict[self.key]).reshape(2))
        if err & _abi.GW_ERR_NOT_IN_GRID:
            raise KeyError(agent.id)                  # Grid.remove of an agent not in its cell
        return bool(status)

    @property
    def key(self):
        return 'move'

    @property
    def supported_agent_type(self):
        return MovingAgent


class CrossMoveActor(ActorBaseComponent):
    """actor.py:117-192: Discrete(5) moves: 0 stay, 1 left, 2 down, 3 right, 4 up."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        for agent in self.agents.values():
            if isinstance(agent, self.supported_agent_type):
                agent.action_space[self.key] = Discrete(5)
                agent.null_action[self.key] = 0
        register_component(self)

    @staticmethod
    def _check_cross(cross_action):
        # CrossMoveActor.grid_action (actor.py:152)
        assert cross_action in [0, 1, 2, 3, 4], "Cross action must be 0, 1, 2, 3, or 4."

    def process_action(self, agent, action_dict, **kwargs):
        """True if the move succeeded (gw_component CROSS_MOVE); None for
        agents that are not MovingAgents (actor.py:161-192)."""
        if not isinstance(agent, self.supported_agent_type):
            return None
        cross = action_dict[self.key]
        self._check_cross(cross)
        status, _, err = ComponentRuntime.of(self).op(_abi.GW_OP_CROSS_MOVE, agent, [int(cross)])
        if err & _abi.GW_ERR_NOT_IN_GRID:
            raise KeyError(agent.id)                  # Grid.remove of an agent not in its cell
        return bool(status)

    @property
    def key(self):
        return 'move'

    @property
    def supported_agent_type(self):
        return MovingAgent


class DriftMoveActor(CrossMoveActor):
    """actor.py:195-234: a failed or absent change of direction drifts the
    agent one cell along its orientation (OrientationAgent + MovingAgent)."""

    def process_action(self, agent, action_dict, **kwargs):
        """gw_component DRIFT_MOVE: the change of direction, else the drift
        along the orientation (which, as in the reference, replaces
        action_dict['move']); None for agents that are not Orientation +
        Moving."""
        if not (isinstance(agent, OrientationAgent) and isinstance(agent, MovingAgent)):
            return None
        cross = action_dict[self.key]
        if cross != 0:
            self._check_cross(cross)
        rt = ComponentRuntime.of(self)
        status, _, err = rt.op(_abi.GW_OP_DRIFT_MOVE, agent, [int(cross), int(agent.orientation or 0)])
        res = rt.last_result
        if res[1] or status == -2:
            action_dict[self.key] = agent.orientation     # actor.py:233
        if status == -2:
            self._check_cross(agent.orientation)          # no orientation: the reference's assert
        if err & _abi.GW_ERR_NOT_IN_GRID:
            raise KeyError(agent.id)
        if int(res[2]) != (agent.orientation or 0):
            agent.orientation = int(res[2])               # actor.py:229-230
        return bool(status)


class AttackActorBaseComponent(ActorBaseComponent, ABC):
    """actor.py:237-438."""

    def __init__(self, attack_mapping=None, stacked_attacks=False, **kwargs):
        super().__init__(**kwargs)
        assert type(attack_mapping) is dict, "Attack mapping must be dictionary."
        for k, v in attack_mapping.items():
            assert type(k) is int, "All keys in attack mapping must be an integer."
            assert type(v) is set, "All values in attack mapping must be a set."
            for i in v:
                assert type(i) is int, "All elements in the attack mapping values must be integers."
        assert type(stacked_attacks) is bool, "Stacked attacks must be a boolean."
        self.attack_mapping = attack_mapping
        self.stacked_attacks = stacked_attacks
        for agent in self.agents.values():
            if isinstance(agent, self.supported_agent_type):
                self._assign_space(agent)
        register_component(self)

    def process_action(self, attacking_agent, action_dict, **kwargs):
        """(attack_status, attacked_agents) as actor.py:306-361: (False, []) when
        not attempted, (True, []) when it failed; damage is applied and killed
        agents leave the grid (gw_component ATTACK)."""
        if not isinstance(attacking_agent, self.supported_agent_type):
            return False, []
        if isinstance(attacking_agent, AmmoAgent):
            attacking_agent.ammo        # no AmmoState.reset yet: the reference's AttributeError
        # this actor's parameters travel with the call: stacked | selective, the
        # attacker's attack_mapping entry as an encoding bitmask
        flags = int(self.stacked_attacks) | (2 if isinstance(self, SelectiveAttackActor) else 0)
        amap = sum(1 << e for e in self.attack_mapping.get(attacking_agent.encoding, ())
                   if 1 <= e <= _abi.GW_MAX_ENC)
        status, attacked, _ = ComponentRuntime.of(self).op(
            _abi.GW_OP_ATTACK, attacking_agent,
            [flags, amap] + list(self._attack_args(action_dict[self.key])))
        if status & 2:
            # _subset_attackables' np.random.choice returns a numpy array
            # (actor.py:412-414), which the ammo filter did not turn into a
            # list: returned as one, so `not attacked` behaves as there
            arr = np.empty(len(attacked), dtype=object)
            arr[:] = attacked
            return True, arr
        return bool(status), attacked

    def _attack_args(self, action):
        return np.asarray(action, dtype=np.int64).reshape(-1)

    @property
    def key(self):
        return 'attack'

    @property
    def supported_agent_type(self):
        return AttackingAgent

    @abstractmethod
    def _assign_space(self, agent):
        pass


class BinaryAttackActor(AttackActorBaseComponent):
    """actor.py:441-501: Discrete(simultaneous_attacks + 1) attacks in the local grid."""

    def _assign_space(self, agent):
        agent.action_space[self.key] = Discrete(agent.simultaneous_attacks + 1)
        agent.null_action[self.key] = 0


class SelectiveAttackActor(AttackActorBaseComponent):
    """actor.py:659-728: Box(0, simultaneous_attacks, (2r+1, 2r+1)) attacks per cell."""

    def _assign_space(self, agent):
        d = 2 * agent.attack_range + 1
        agent.action_space[self.key] = Box(0, agent.simultaneous_attacks, (d, d), int)
        agent.null_action[self.key] = np.zeros((d, d), dtype=int)


# -------------------------------------------------------------- observers
class ObserverBaseComponent(GridWorldBaseComponent, _EngineExecuted, ABC):
    """observer.py:13-52."""

    def get_obs(self, agent, **kwargs):
        self._engine_only('get_obs')

    @property
    @abstractmethod
    def key(self):
        pass

    @property
    @abstractmethod
    def supported_agent_type(self):
        pass


class PositionCenteredEncodingObserver(ObserverBaseComponent):
    """observer.py:153-250: Box(-2, max_encoding, (2v+1, 2v+1), int)."""

    def __init__(self, observe_self=True, **kwargs):
        super().__init__(**kwargs)
        assert type(observe_self) is bool, "Observe self must be a boolean."
        self.observe_self = observe_self
        max_encoding = max(agent.encoding for agent in self.agents.values())
        for agent in self.agents.values():
            if isinstance(agent, self.supported_agent_type):
                side = agent.view_range * 2 + 1
                agent.observation_space[self.key] = Box(-2, max_encoding, (side, side), int)
                agent.null_observation[self.key] = -2 * np.ones((side, side), dtype=int)
        register_component(self)

    def get_obs(self, agent, **kwargs):
        """The agent's (2v+1)^2 window (gw_component OBSERVE; crowded cells
        draw np.random.choice in the reference's order); {} for agents that
        are not GridObservingAgents (observer.py:204-250)."""
        if not isinstance(agent, self.supported_agent_type):
            return {}
        return {self.key: ComponentRuntime.of(self).observe(agent, self.observe_self)}

    @property
    def key(self):
        return 'position_centered_encoding'

    @property
    def supported_agent_type(self):
        return GridObservingAgent


class AbsoluteEncodingObserver(ObserverBaseComponent):
    """observer.py:55-150: Box(-2, max_encoding, (rows, cols), int); the
    observer itself is -1, cells outside its view range -2."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        max_encoding = max(agent.encoding for agent in self.agents.values())
        for agent in self.agents.values():
            if isinstance(agent, self.supported_agent_type):
                agent.observation_space[self.key] = Box(
                    -2, max_encoding, (self.rows, self.cols), int)
                agent.null_observation[self.key] = -2 * np.ones((self.rows, self.cols), dtype=int)
        register_component(self)

    def get_obs(self, agent, **kwargs):
        """The (rows, cols) grid (gw_component OBSERVE_ABS: blocking masks and
        crowded-cell draws on the device, in the reference's order); {} for
        agents that are not GridObservingAgents."""
        if not isinstance(agent, self.supported_agent_type):
            return {}
        return {self.key: ComponentRuntime.of(self).observe_absolute(agent)}

    @property
    def key(self):
        return 'absolute_encoding'

    @property
    def supported_agent_type(self):
        return GridObservingAgent


# ------------------------------------------------------------------ dones
class DoneBaseComponent(GridWorldBaseComponent, _EngineExecuted, ABC):
    """done.py:10-36."""

    def get_done(self, agent, **kwargs):
        self._engine_only('get_done')

    def get_all_done(self, **kwargs):
        self._engine_only('get_all_done')


class ActiveDone(DoneBaseComponent):
    """done.py:39-56: done = not active; all done = no active agent."""

    def get_done(self, agent, **kwargs):
        return not agent.active

    def get_all_done(self, **kwargs):
        return not any(agent.active for agent in self.agents.values())


class OneTeamRemainingDone(ActiveDone):
    """done.py:140-153: all done when the active agents share <= 1 encoding."""

    def get_all_done(self, **kwargs):
        return len({agent.encoding for agent in self.agents.values() if agent.active}) <= 1


class _TargetMappingDone(DoneBaseComponent):
    """The target_mapping property shared by done.py:59-99 and :102-137."""

    def __init__(self, target_mapping=None, **kwargs):
        super().__init__(**kwargs)
        self.target_mapping = target_mapping

    @property
    def target_mapping(self):
        """Maps the agent to its respective target (by agent id)."""
        return self._target_mapping

    @target_mapping.setter
    def target_mapping(self, value):
        assert type(value) is dict, "Target mapping must be a dictionary."
        for agent_id, target_id in value.items():
            assert agent_id in self.agents, f"{agent_id} must be an agent in the simulation."
            assert isinstance(self.agents[agent_id], GridWorldAgent), \
                f"{agent_id} must be a GridWorldAgent."
            assert target_id in self.agents, "Target must be an agent in the simulation."
            assert isinstance(self.agents[target_id], GridWorldAgent), \
                "Target must be a GridWorldAgent."
        self._target_mapping = value


class TargetAgentDone(_TargetMappingDone):
    """done.py:59-99: an agent is done when it is on its target's position
    (np.array_equal of the positions); all done when every mapped agent is."""

    def get_done(self, agent, **kwargs):
        return np.array_equal(agent.position, self.agents[self.target_mapping[agent.id]].position)

    def get_all_done(self, **kwargs):
        return all(self.get_done(self.agents[aid]) for aid in self.target_mapping)


class TargetDestroyedDone(_TargetMappingDone):
    """done.py:102-137: an agent is done when its target is inactive; all
    done when every mapped agent's target is."""

    def get_done(self, agent, **kwargs):
        return not self.agents[self.target_mapping[agent.id]].active

    def get_all_done(self, **kwargs):
        return all(self.get_done(self.agents[aid]) for aid in self.target_mapping)
