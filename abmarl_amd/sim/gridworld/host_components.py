"""The registry's components that run on the HOST (off the fused programs).

EncodingBasedAttackActor, RestrictedSelectiveAttackActor,
StackedPositionCenteredEncodingObserver, AbsolutePositionObserver and
AmmoObserver (actor.py:504-656, observer.py:253-410 in the reference) are part
of the plugin API -- a configuration may name them (registry.py:20-47) -- but
no benchmarked program uses them, so they have no HIP form.  They run the way
a user-written component does (registry.register, component_runtime.py): as
Python on the agents and the Grid that the built-in device operations mirror
after every call, drawing from the one global numpy legacy stream, which the
component runtime hands to and takes back from the device around each device
operation.  A simulation therefore interleaves them freely with the built-in
components, and the draws come in the reference's order: per candidate, the
accuracy draw of _basic_criteria (np.random.uniform, actor.py:363-392) after
the id / active / mapping tests; then np.random.choice for the subset
(actor.py:394-414) or the per-cell pick (actor.py:636-654); then the ammo
filter (actor.py:343-351).

The fused programs (TeamBattleSim, ...) refuse them at construction
(compile.py: no HIP implementation).
"""
import numpy as np

from abmarl_amd.spaces import Box, Dict, Discrete, MultiDiscrete
from abmarl_amd.sim.agent_based_simulation import ObservingAgent
from abmarl_amd.sim.gridworld.agent import AmmoAgent, AmmoObservingAgent, GridObservingAgent
from abmarl_amd.sim.gridworld.components import AttackActorBaseComponent, ObserverBaseComponent
from abmarl_amd.sim.gridworld.utils import create_grid_and_mask


# ----------------------------------------------------------------- actors
class _HostAttackActor(AttackActorBaseComponent):
    """An attack actor whose process_action runs on the host: the subclass
    picks the attacked agents (_determine_attack), then the ammo limit, the
    damage and the removal of the killed from the grid (actor.py:306-361)."""

    def process_action(self, attacking_agent, action_dict, **kwargs):
        if not isinstance(attacking_agent, self.supported_agent_type):
            return False, []
        status, hit = self._determine_attack(attacking_agent, action_dict[self.key])
        if isinstance(attacking_agent, AmmoAgent):
            left = attacking_agent.ammo
            if len(hit) > left:
                # more picks than rounds: which ones land is a draw without
                # replacement (the list form, as the reference's .tolist())
                hit = np.random.choice(hit, size=left, replace=False).tolist()
            attacking_agent.ammo = left - len(hit)
        for victim in hit:
            if victim.active:             # a pick that died earlier in this list takes nothing
                victim.health = victim.health - attacking_agent.attack_strength
                if not victim.active:
                    self.grid.remove(victim, victim.position)
        return status, hit

    def _basic_criteria(self, attacking_agent, candidate):
        """Not itself, alive, an encoding the attacker may attack, and the
        accuracy draw passed (drawn only when the first three hold)."""
        if candidate.id == attacking_agent.id or not candidate.active:
            return False
        if candidate.encoding not in self.attack_mapping[attacking_agent.encoding]:
            return False
        return not np.random.uniform() > attacking_agent.attack_accuracy

    def _subset_attackables(self, attackable_agents, number_of_attacks):
        """All of them when the attacks outnumber them and may not stack;
        otherwise np.random.choice (with replacement iff stacked)."""
        if number_of_attacks > len(attackable_agents) and not self.stacked_attacks:
            return attackable_agents
        return np.random.choice(attackable_agents, size=number_of_attacks, replace=self.stacked_attacks)

    def _window(self, agent):
        """(local grid, visibility mask) of the attacker's attack range
        (create_grid_and_mask: cells are dicts or None off the grid, mask 0
        behind an active blocking agent)."""
        return create_grid_and_mask(agent, self.grid, agent.attack_range, self.agents)


class EncodingBasedAttackActor(_HostAttackActor):
    """actor.py:504-580: Dict({encoding: Discrete(simultaneous_attacks + 1)})
    over the attacker's attackable encodings; up to that many attacks on each
    encoding, chosen among the candidates of that encoding in the attack
    range (one scan of the window, candidates in row-major cell order and
    insertion order inside a cell)."""

    def _assign_space(self, agent):
        encs = self.attack_mapping[agent.encoding]
        agent.action_space[self.key] = Dict({e: Discrete(agent.simultaneous_attacks + 1) for e in encs})
        agent.null_action[self.key] = {e: 0 for e in encs}

    def _determine_attack(self, agent, attack):
        if not any(n for n in attack.values()):
            return False, []
        local, mask = self._window(agent)
        side = 2 * agent.attack_range + 1
        by_enc = {e: [] for e in attack}
        for k in range(side * side):
            r, c = divmod(k, side)
            cell = local[r, c]
            if not mask[r, c] or cell is None:
                continue
            for other in cell.values():
                if self._basic_criteria(agent, other):
                    by_enc[other.encoding].append(other)
        hit = []
        for enc, n in attack.items():
            if by_enc[enc]:
                hit.extend(self._subset_attackables(by_enc[enc], n))
        return True, hit


class RestrictedSelectiveAttackActor(_HostAttackActor):
    """actor.py:583-656: MultiDiscrete([(2r+1)^2 + 1] * simultaneous_attacks);
    each entry 0 is no attack, else cell k - 1 of the window unravelled
    column-major (row (k-1) % (2r+1), column (k-1) // (2r+1)), where ONE
    candidate is picked (np.random.choice), skipping agents this action
    already hit unless attacks stack."""

    def _assign_space(self, agent):
        cells = (2 * agent.attack_range + 1) ** 2
        agent.action_space[self.key] = MultiDiscrete([cells + 1] * agent.simultaneous_attacks)
        agent.null_action[self.key] = np.zeros((agent.simultaneous_attacks,), dtype=int)

    def _determine_attack(self, agent, attack):
        if not any(attack):
            return False, []
        local, mask = self._window(agent)
        side = 2 * agent.attack_range + 1
        hit = []
        for code in attack:
            if code == 0:
                continue
            k = code - 1
            r, c = k % side, int(k / side)
            pool = []
            cell = local[r, c]
            if mask[r, c] and cell is not None:
                for other in cell.values():
                    # the accuracy draw comes first, the repeat test after it
                    if self._basic_criteria(agent, other) and (self.stacked_attacks or other not in hit):
                        pool.append(other)
            if pool:
                hit.append(np.random.choice(pool))
        return True, hit


# -------------------------------------------------------------- observers
class _HostObserver(ObserverBaseComponent):
    """An observer whose get_obs runs on the host."""

    def _spaces(self, space, null):
        for agent in self.agents.values():
            if isinstance(agent, self.supported_agent_type):
                agent.observation_space[self.key] = space(agent)
                agent.null_observation[self.key] = null(agent)


class StackedPositionCenteredEncodingObserver(_HostObserver):
    """observer.py:253-334: the (2v+1, 2v+1, max encoding) window, layer e
    counting the occupants of encoding e + 1; -1 off the grid and -2 hidden
    behind a blocker in every layer, 0 for an empty cell.  No draws."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.number_of_encodings = max(a.encoding for a in self.agents.values())
        n = self.number_of_encodings
        side = lambda a: 2 * a.view_range + 1
        self._spaces(lambda a: Box(-2, len(self.agents), (side(a), side(a), n), int),
                     lambda a: -2 * np.ones((side(a), side(a), n), dtype=int))

    @property
    def key(self):
        return 'stacked_position_centered_encoding'

    @property
    def supported_agent_type(self):
        return GridObservingAgent

    def get_obs(self, agent, **kwargs):
        if not isinstance(agent, self.supported_agent_type):
            return {}
        local, mask = create_grid_and_mask(agent, self.grid, agent.view_range, self.agents)
        side = 2 * agent.view_range + 1
        n = self.number_of_encodings
        obs = np.zeros((side, side, n), dtype=int)
        for r in range(side):
            for c in range(side):
                cell = local[r, c]
                if not mask[r, c]:
                    obs[r, c, :] = -2
                elif cell is None:
                    obs[r, c, :] = -1
                else:
                    for other in cell.values():
                        if 1 <= other.encoding <= n:
                            obs[r, c, other.encoding - 1] += 1
        return {self.key: obs}


class AbsolutePositionObserver(_HostObserver):
    """observer.py:337-373: an ObservingAgent observes its own position,
    Box([0, 0], [rows - 1, cols - 1], int)."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        hi = np.array([self.grid.rows - 1, self.grid.cols - 1], dtype=int)
        self._spaces(lambda a: Box(np.zeros(2, dtype=int), hi, dtype=int),
                     lambda a: np.zeros((2,), dtype=int))

    @property
    def key(self):
        return 'position'

    @property
    def supported_agent_type(self):
        return ObservingAgent

    def get_obs(self, agent, **kwargs):
        if not isinstance(agent, self.supported_agent_type):
            return {}
        return {self.key: agent.position}


class AmmoObserver(_HostObserver):
    """observer.py:376-410: an AmmoObservingAgent observes its own ammo,
    Box(0, initial_ammo, (1,), int)."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._spaces(lambda a: Box(0, a.initial_ammo, shape=(1,), dtype=int), lambda a: 0)

    @property
    def key(self):
        return 'ammo'

    @property
    def supported_agent_type(self):
        return AmmoObservingAgent

    def get_obs(self, agent, **kwargs):
        if not isinstance(agent, self.supported_agent_type):
            return {}
        return {self.key: agent.ammo}
