/*
 * gw_engine.h — C-ABI of the MI355X batched GridWorld step engine.
 *
 * This is the drop-in boundary for Abmarl's GridWorld hot path.  One handle
 * holds E independent environments of one simulation configuration; every
 * call advances all (or a masked subset of) them on one HIP stream.
 *
 * Reference interfaces each entry point replaces (paths under
 * gillette7/Abmarl, abmarl/):
 *
 *   gw_create   GridWorldSimulation.build_sim          sim/gridworld/base.py:38-59
 *               + SmartGridWorldSimulation.__init__     sim/gridworld/smart.py:26-84
 *               + AllStepManager.__init__               managers/all_step_manager.py:8-17
 *   gw_seed     np.random.seed(seed) per env            (numpy legacy MT19937 init_genrand)
 *   gw_reset    AllStepManager.reset                    managers/all_step_manager.py:37-49
 *               -> SmartGridWorldSimulation.reset       sim/gridworld/smart.py:86-91
 *                  -> PositionState.reset               sim/gridworld/state.py:88-166
 *                  -> HealthState.reset                 sim/gridworld/state.py:629-641
 *               -> get_obs for every live agent         sim/gridworld/observer.py:204-250
 *   gw_step     AllStepManager.step                     managers/all_step_manager.py:51-95
 *               -> TeamBattleSim.step                   examples/sim/team_battle_example.py:33-59
 *                  -> BinaryAttackActor.process_action  sim/gridworld/actor.py:306-361,455-501
 *                  -> MoveActor.process_action          sim/gridworld/actor.py:82-114
 *               -> MazeNavigationSim.step               examples/sim/maze_navigation.py:25-42
 *               -> get_obs / get_reward / get_done      sim/gridworld/smart.py:93-117
 *                  -> ActiveDone / OneTeamRemainingDone sim/gridworld/done.py:39-56,140-153
 *               -> PacmanSim.step                     examples/sim/pacman.py:80-135
 *                  -> DriftMoveActor.process_action   sim/gridworld/actor.py:195-234
 *               -> AbsoluteEncodingObserver.get_obs   sim/gridworld/observer.py:95-150
 *   gw_turn_reset / gw_turn_step   TurnBasedManager.reset/step  managers/turn_based_manager.py:22-94
 *   gw_sim_reset / gw_sim_step / gw_observe   SmartGWS.reset / sim.step / get_obs
 *   gw_get_state / gw_set_state   (no reference equivalent: engine SoA snapshot,
 *               used for checkpoint and for parity tests)
 *   gw_destroy  (Python GC of the simulation objects)
 *
 * Conventions
 *   - All I/O buffers are caller-owned DEVICE pointers (allocated by the
 *     caller, e.g. torch).  The engine owns only its internal state.
 *   - Calls are stream-ordered on the `stream` argument (a hipStream_t, 0 =
 *     default stream) and are not re-entrant per handle.
 *   - Return value: GW_OK or a negative gw_status.  Per-env failures that the
 *     reference raises as Python exceptions are reported in err_flags[E]
 *     (GW_ERR_*); the Python facade maps them back to the same exception types.
 *   - No torch / HIP types appear in the signatures: streams are void*.
 *
 * Entities and lanes
 *   gw_config.agents lists every entity of the simulation (agents-dict order,
 *   up to GW_MAX_ENTITIES).  gw_create splits them in two:
 *     static entities: no Observing/Acting/GridObserver/Moving/Attacking/Health
 *       mixin, an initial_position, an encoding that overlaps nothing and that
 *       no attack_mapping names (e.g. the maze walls of
 *       examples/rllib_maze_navigation.py).  They never move, die, act or
 *       observe, and no other entity can share their cell, so they live in
 *       the per-config cell-table template (and block sight when blocking);
 *     lanes: every other entity, at most GW_MAX_AGENTS (one wavefront lane
 *       each), or GW_MAX_LANES for the ReachTheTarget program, which runs on
 *       one workgroup per env when it has more than GW_MAX_AGENTS lanes.
 *   Every per-entity array below ([E][A]...) is indexed by LANE, A =
 *   gw_num_lanes(h); gw_lane_entities gives the entity index of each lane.
 *   Static entities sit at their initial position, active, in every env.
 */
#ifndef GW_ENGINE_H
#define GW_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ limits */
#define GW_MAX_AGENTS   64   /* lanes: one wavefront lane per dynamic entity  */
#define GW_MAX_LANES   256   /* ReachTheTarget program with SelectiveAttackActor:
                                one workgroup per env, one thread per dynamic
                                entity (BASELINE config 4: 256 entities)      */
#define GW_MAX_ENTITIES 4096 /* lanes + static entities                       */
#define GW_MAX_ENC      15   /* encodings 1..15                               */
#define GW_MAX_CELLS 16384   /* rows*cols (and the LDS budget: 160 KiB per env) */
#define GW_MAX_RANGE    64   /* view range (windows up to 129x129; ranges above 7
                                run on the generic window path of the one-wave
                                kernel)                                        */
#define GW_MAX_ATTACK_RANGE 7 /* attack range                                 */
#define GW_ACT_DIM       3   /* binary-attack sims: actions[e][a] = {move_row, move_col, attack};
                                see gw_act_dim() for the general width                */
#define GW_MT_N        624   /* MT19937 state words                           */
#define GW_MT_STRIDE   704   /* words per env in the MT state array: key[624], pos @624,
                                internal @625..703 (a write of the key through gw_set_state
                                invalidates the engine's cached words)            */

/* ----------------------------------------------------------- status codes */
typedef int32_t gw_status;
#define GW_OK               0
#define GW_E_INVALID      (-1)  /* bad config / argument                  */
#define GW_E_HIP          (-2)  /* HIP runtime error                      */
#define GW_E_UNSUPPORTED  (-3)  /* config outside what the engine builds  */

/* per-env error flags (err_flags[e], OR-ed) */
#define GW_ERR_NO_CELL        1u  /* PositionState: RuntimeError "Could not find a cell"  state.py:158-162 */
#define GW_ERR_INIT_POSITION  2u  /* PositionState: AssertionError initial cell taken     state.py:147-149 */
#define GW_ERR_DOUBLE_REMOVE  4u  /* ReachTheTarget: KeyError, Grid.remove of an agent the target
                                     already killed on its own cell (reach_the_target.py:118-120) */
#define GW_ERR_TUNNEL_PLACE   8u  /* Pacman: Grid.place at the far end of the tunnel refused the
                                     agent, which is left off the grid (pacman.py:88-93);
                                     its next move would raise KeyError in Grid.remove */
#define GW_ERR_NOT_IN_GRID   16u  /* gw_component MOVE of an entity that is not in the grid:
                                     Grid.remove raises KeyError (actor.py:108-110);
                                     the entity stays where it was                    */
#define GW_ERR_VALUE_ERROR   32u  /* TeamBattle / ReachTheTarget step with BinaryAttackActor:
                                     `not attacked_agents` on the numpy array of 2 or more
                                     picks _subset_attackables returns (actor.py:412-414)
                                     raises ValueError (team_battle_example.py:41,
                                     reach_the_target.py:127); the step stops after that
                                     attacker's attack (damage, ammo and draws applied)
                                     unless gw_config.attack_array_as_list              */

/* ------------------------------------------------------------ agent kinds */
/* bit flags describing which reference mixins an entity derives from        */
#define GW_K_OBSERVING     0x01u /* ObservingAgent            agent_based_simulation.py:120 */
#define GW_K_ACTING        0x02u /* ActingAgent               agent_based_simulation.py:66  */
#define GW_K_GRID_OBSERVER 0x04u /* GridObservingAgent        gridworld/agent.py:122         */
#define GW_K_MOVING        0x08u /* MovingAgent               gridworld/agent.py:147         */
#define GW_K_ATTACKING     0x10u /* AttackingAgent            gridworld/agent.py:213         */
#define GW_K_HEALTH        0x20u /* HealthAgent               gridworld/agent.py:172         */
#define GW_K_PROGRAM       0x80u /* the sim program's own agent class (ReachTheTarget:
                                    RunningAgent, reach_the_target.py:75-81)        */
#define GW_K_ORIENTATION  0x100u /* OrientationAgent          gridworld/agent.py:342-373   */
#define GW_K_FOOD         0x200u /* Pacman FoodAgent (pacman.py:17-19); with GW_SIM_PACMAN,
                                    GW_K_PROGRAM marks its BaddieAgent (pacman.py:22-24) */
#define GW_K_LANE         0x400u /* never a static entity: the caller may read or edit
                                    it (the component runtime keeps blocking entities
                                    as lanes: the absolute observer's masks take lanes) */
#define GW_K_AMMO         0x800u /* AmmoAgent                 gridworld/agent.py:291-322: a
                                    limited number of attacks (AttackActorBaseComponent.
                                    process_action's ammo filter, actor.py:343-351) */
#define GW_K_BLOCKING      0x40u /* GridWorldAgent.blocking   gridworld/agent.py:66-75;
                                    active blocking entities mask cells from
                                    observers and attackers (utils.py:5-117) */

/* ---------------------------------------------------------- sim programs */
#define GW_SIM_TEAM_BATTLE  1   /* examples/sim/team_battle_example.py:33-59 */
#define GW_SIM_MAZE_NAV     2   /* examples/sim/maze_navigation.py:25-42     */
#define GW_SIM_REACH_TARGET 3   /* examples/sim/reach_the_target.py:84-158   */
#define GW_SIM_PACMAN       4   /* examples/sim/pacman.py:29-158: DriftMoveActor moves, the
                                   tunnel, food and baddies (see "Pacman program" below) */
#define GW_SIM_TRAFFIC      5   /* examples/sim/traffic_corridor.py:24-49: moves in dict order,
                                   -0.1 on a failed move, +1 when get_done(agent) right after
                                   its move (the done components, e.g. TargetAgentDone)     */

/* observer of the sim's GridObservingAgents */
#define GW_OBS_POSITION_CENTERED 0  /* observer.py:153-250: (2v+1)^2 window, -1 off-grid   */
#define GW_OBS_ABSOLUTE          1  /* observer.py:55-150: rows x cols, -1 = the observer,
                                       -2 = outside its view range                    */

/* attack actor of the sim */
#define GW_ATTACK_BINARY     0  /* BinaryAttackActor     actor.py:441-501: one int, 0..simultaneous */
#define GW_ATTACK_SELECTIVE  1  /* SelectiveAttackActor  actor.py:659-728: (2R+1)^2 ints, attacks per cell */

/* done components (bit set; get_done = AND, get_all_done = AND: smart.py:106-117) */
#define GW_DONE_ACTIVE        0x1u /* ActiveDone            done.py:39-56   */
#define GW_DONE_ONE_TEAM      0x2u /* OneTeamRemainingDone  done.py:140-153 */
#define GW_DONE_TARGET_AGENT  0x4u /* TargetAgentDone       done.py:59-99: done = on the
                                      position of gw_agent_spec.done_target; all done = every
                                      mapped entity done                                   */
#define GW_DONE_TARGET_DESTROYED 0x8u /* TargetDestroyedDone done.py:102-137: done = the entity
                                      gw_agent_spec.destroy_target is inactive; all done = every
                                      mapped entity's target inactive                      */
/* done_kind 0 (no done component) is the reference's all([]): every agent done. */

/* reset-time state component order (SmartGridWorldSimulation iterates a set) */
#define GW_ORDER_POSITION_HEALTH 0
#define GW_ORDER_HEALTH_POSITION 1

typedef struct gw_agent_spec {
    int32_t  encoding;             /* >= 1                                     */
    uint32_t kind;                 /* GW_K_* bits                              */
    int32_t  init_row, init_col;   /* initial_position, or -1,-1 for random    */
    int32_t  view_range;
    int32_t  move_range;
    int32_t  attack_range;
    int32_t  simultaneous_attacks;
    double   attack_strength;
    double   attack_accuracy;
    double   initial_health;       /* < 0 means None (uniform(0,1) at reset)   */
    int32_t  initial_orientation;  /* OrientationAgent: 1..4, 0 = None (randint(1, 5)) */
    int32_t  done_target;          /* TargetAgentDone.target_mapping[this] (entity index), -1 */
    int32_t  destroy_target;       /* TargetDestroyedDone.target_mapping[this], -1            */
    int32_t  initial_ammo;         /* AmmoAgent.initial_ammo (GW_K_AMMO): the ammo every reset
                                      gives it (AmmoState.reset, state.py:644-656)           */
} gw_agent_spec;

typedef struct gw_config {
    int32_t  rows, cols;
    int32_t  n_agents;             /* entities, in agents-dict order (lanes +
                                      static entities, see "Entities and lanes") */
    int32_t  sim_kind;             /* GW_SIM_*                                  */
    /* overlap[e] bit f set <=> encoding e may share a cell with encoding f
       (already made symmetric, grid.py:53-71; missing key == empty set)       */
    uint32_t overlap[GW_MAX_ENC + 1];
    /* attack_mapping[e] bit f set <=> e may attack f (actor.py:278-287)       */
    uint32_t attack_mapping[GW_MAX_ENC + 1];
    int32_t  stacked_attacks;      /* AttackActorBaseComponent.stacked_attacks  */
    int32_t  observe_self;         /* PositionCenteredEncodingObserver          */
    int32_t  no_overlap_at_reset;  /* PositionState                             */
    int32_t  state_order;          /* GW_ORDER_*                                */
    uint32_t done_kind;            /* GW_DONE_* bits                            */
    int32_t  obs_range;            /* shared view_range of every grid observer  */
    int32_t  target_agent;         /* MazeNav: index of 'target' (else -1)      */
    int32_t  nav_agent;            /* MazeNav: index of 'navigator' (else -1)   */
    const gw_agent_spec* agents;   /* host pointer, n_agents entries            */
    int32_t  attack_kind;          /* GW_ATTACK_*                               */
    int32_t  obs_kind;             /* GW_OBS_*                                  */
    /* Pacman program (GW_SIM_PACMAN) */
    int32_t  pacman_agent;         /* index of 'pacman' (else -1)               */
    int32_t  tunnel[4];            /* r0, c0, r1, c1: the teleporting cells (pacman.py:88-93) */
    double   pac_rewards[5];       /* reward_scheme: bad_move, entropy, eat_food, kill, die */
    /* kernel selection: 0 = automatic (one wave per env; ReachTheTarget with
       more than GW_MAX_AGENTS lanes on a workgroup per env), 1 = force the
       workgroup-per-env kernel (ReachTheTarget; parity tests run the small
       reference fixtures through it), 2..4 = the workgroup kernel with that
       many waves per env (at least ceil(lanes / 64)): the threads past the
       lanes share the table, observation-store and crowded-draw work (small
       batches: more waves per env when there are fewer envs than SIMDs)     */
    int32_t  force_workgroup;
    /* 1: the caller passes the SAME obs buffer to every call of this handle
       (as the Python engine does with its own), so the one-wave kernels do
       not rewrite the rows that already hold -2 and stay -2 (entities done
       before this step, non-observers): steady-state obs stores shrink with
       the done fraction.  0: every row is written every call.              */
    int32_t  persistent_obs;
    /* 1: every entity is a lane (no static entities in the cell template):
       the component plugin API keeps all entity state in lanes              */
    int32_t  all_lanes;
    /* one-lane-per-env kernel (MazeNavigation with the navigator and the
       target as its only dynamic entities, both at initial positions: 64
       envs per wave): 0 = automatic (used when eligible), 1 = required
       (gw_create fails if the config is not eligible), -1 = never (one
       wavefront per env)                                                     */
    int32_t  env_per_lane;
    /* 1: a component-API handle (gw_component only, no step program): either
       attack kind on the workgroup-per-env engine above 64 lanes           */
    int32_t  component_api;
    /* 0 (the reference): an attacker whose BinaryAttackActor returns the numpy
       array of 2 or more picks makes the step's `not attacked_agents` raise
       ValueError (GW_ERR_VALUE_ERROR; TeamBattle and ReachTheTarget programs).
       1 (opt-in): the attacked agents are read as a list, `len(...) == 0`
       being the failed-attack test -- the example's evident meaning, which
       the reference itself cannot run.                                      */
    int32_t  attack_array_as_list;
} gw_config;

/* Width of one entity's action: {move_row, move_col, attack...}.  The attack
   part is one int (binary) or per-cell attack counts (selective): room for
   (2R+1)^2 ints, R = the largest attack range; an agent of range r uses the
   first (2r+1)^2 of them as its row-major window.  A negative first attack
   int marks an entity that is not in the action dict.                       */
static inline int32_t gw_config_act_dim(const gw_config* cfg)
{
    if (cfg->attack_kind != GW_ATTACK_SELECTIVE) return GW_ACT_DIM;
    int32_t r = 0;
    for (int32_t a = 0; a < cfg->n_agents; a++)
        if ((cfg->agents[a].kind & GW_K_ATTACKING) && cfg->agents[a].attack_range > r)
            r = cfg->agents[a].attack_range;
    return 2 + (2 * r + 1) * (2 * r + 1);
}

typedef struct gw_engine* gw_handle;

/* Build an engine for n_envs environments of `cfg` on HIP device `device`.
   Validates the config against the engine's limits (GW_E_UNSUPPORTED).     */
gw_status gw_create(const gw_config* cfg, int32_t n_envs, int32_t device, gw_handle* out);

/* Seed env e's MT19937 with seeds[e] (np.random.seed semantics).
   seeds: device uint32[E].                                                   */
gw_status gw_seed(gw_handle h, const uint32_t* seeds, void* stream);

/* Reset the selected envs: all of them when mask, all_done and horizon are
   all unset (NULL, NULL, <= 0); otherwise every env e with mask[e] != 0, or
   all_done[e] != 0 (the previous step's __all__), or steps[e] >= horizon.
   Writes the reset observation of every entity of the reset envs into obs
   (untouched for other envs).
     mask      device uint8[E] or NULL
     all_done  device uint8[E] or NULL  (the previous step's __all__)
     obs       device int32[E][A][S][S], S = 2*obs_range+1
     err_flags device uint32[E]: a reset env's flags are replaced by the
               reset's own (GW_ERR_NO_CELL / GW_ERR_INIT_POSITION or 0), so
               an error raised before the reset does not outlive it; flags
               of envs not reset are untouched.  (gw_turn_reset and
               gw_sim_reset do the same.)                                   */
gw_status gw_reset(gw_handle h, const uint8_t* mask, const uint8_t* all_done,
                   int32_t horizon, int32_t* obs, uint32_t* err_flags, void* stream);

/* One AllStepManager.step for every env.
     actions   device int32[E][A][gw_act_dim(h)]  (ignored for done entities)
     obs       device int32[E][A][S][S]  (-2 for entities that are done)
     reward    device double[E][A]      (0 for entities that are done)
     done      device uint8[E][A]       (1 for entities that were already done)
     all_done  device uint8[E]          ('__all__')
     acting    device uint64[E] or NULL (+= number of acting agents, for metrics)
     err_flags device uint32[E] or NULL (|= GW_ERR_*: a step the reference
               would raise in; that env's outputs are not written.  In the
               auto-reset calls below such an env is reset like one whose
               episode ended: all_done[e] = 1, and gw_step_autoreset writes
               the next episode's first observation in the same launch)     */
gw_status gw_step(gw_handle h, const int32_t* actions, int32_t* obs, double* reward,
                  uint8_t* done, uint8_t* all_done, uint64_t* acting, uint32_t* err_flags,
                  void* stream);

/* gw_step followed, in the same launch, by AllStepManager.reset of every env
   whose '__all__' is set or that reached `horizon` steps (horizon > 0).  For
   those envs obs holds the first observation of the next episode, while
   reward / done / all_done are the terminal step's (RLlib VectorEnv
   auto-reset convention).  err_flags: device uint32[E] or NULL.            */
gw_status gw_step_autoreset(gw_handle h, const int32_t* actions, int32_t* obs, double* reward,
                            uint8_t* done, uint8_t* all_done, uint64_t* acting, int32_t horizon,
                            uint32_t* err_flags, void* stream);

/* NEXT_STEP auto-reset (gymnasium vector-env convention; the batched form
   of RLlib calling AllStepManager.reset after '__all__'): an env whose
   previous call ended its episode — all_done[e] set on INPUT, or steps[e] >=
   horizon (horizon > 0) — is reset by this call instead of stepped: obs =
   the first observation of the new episode, reward 0, done 1 only for
   entities that are not Agents, all_done 0, its actions ignored and nothing
   added to acting.  Every other env takes one step.  all_done is in/out.    */
gw_status gw_step_autoreset_next(gw_handle h, const int32_t* actions, int32_t* obs, double* reward,
                                 uint8_t* done, uint8_t* all_done, uint64_t* acting, int32_t horizon,
                                 uint32_t* err_flags, void* stream);

/* Snapshot / restore of the engine state (device buffers, caller-owned).
     pos     int32[E][A][2]   (row, col)
     health  double[E][A]
     flags   uint8[E][A]      bit0 in-grid, bit1 live (not in done_agents), bit2 active,
                              bits3-5 orientation (Pacman program); the engine-internal
                              bit6 (obs row already -2) is masked out of a snapshot and
                              cleared by a restore (the next step rewrites every row)
     seq     uint32[E][A]     placement order inside a cell (dict insertion order)
     mt      uint32[E][GW_MT_STRIDE]  key[624], pos at [624], engine-internal after
     steps   int32[E]                                                          */
gw_status gw_get_state(gw_handle h, int32_t* pos, double* health, uint8_t* flags,
                       uint32_t* seq, uint32_t* mt, int32_t* steps, void* stream);
gw_status gw_set_state(gw_handle h, const int32_t* pos, const double* health,
                       const uint8_t* flags, const uint32_t* seq, const uint32_t* mt,
                       const int32_t* steps, void* stream);

/* AmmoAgent.ammo of every lane (GW_K_AMMO lanes; 0 for the others), the
   state beside gw_get_state: device int32[E][A].  Every reset of an env
   (gw_reset, the auto-reset calls, gw_sim_reset) sets its ammo lanes to
   initial_ammo (AmmoState.reset, state.py:644-656: no draw, so its place
   in the state order changes nothing); every attack of an ammo lane with
   more attacked entries than ammo keeps np.random.choice(attacked, ammo,
   replace=False) of them (= permutation(n)[:ammo] draws) and subtracts the
   kept count (actor.py:343-351).                                          */
gw_status gw_get_ammo(gw_handle h, int32_t* ammo, void* stream);
gw_status gw_set_ammo(gw_handle h, const int32_t* ammo, void* stream);

/* Philox-4x32-10 random policy (uniform over MoveActor Box(-r,r,(2,)) and
   BinaryAttackActor Discrete(k+1)): actions for every entity of every env,
   keyed by (key, env_offset + env, step, agent) so that a sharded run draws
   the same actions for a global env id on any number of GPUs.  Not part of
   the reference; it is the benchmark's synthetic policy.                     */
gw_status gw_random_actions(gw_handle h, uint64_t key, uint32_t step, uint32_t env_offset,
                            int32_t* actions, void* stream);

/* ---------------------------------------------------------------------
 * The component plugin API (ActorBaseComponent.process_action, actor.py:13-52;
 * ObserverBaseComponent.get_obs, observer.py:13-52; StateBaseComponent.reset,
 * state.py:13-22) as device operations: ONE component call for one entity
 * (lane) in every env, on the engine's state (positions, health, active,
 * in-grid, in-cell order, the MT19937 stream), so that a step() composed of
 * component calls in Python runs them on the GPU in its own order.  The
 * one-wave engine only (GW_KERNEL_WAVE).
 *   GW_OP_POSITION_RESET  PositionState.reset (state.py:88-166): every cell
 *                         emptied, every entity placed again; args[e][0] =
 *                         no_overlap_at_reset (NULL args: the config's)
 *   GW_OP_HEALTH_RESET    HealthState.reset (state.py:629-641)
 *   GW_OP_MOVE            MoveActor.process_action(lane, {'move': args[e][0:2]})
 *   GW_OP_ATTACK          an attack actor's process_action(lane, {'attack':
 *                         args[e][2] (binary) or args[e][2:] (selective cells)});
 *                         args[e][0] = stacked_attacks | 2 (SelectiveAttackActor),
 *                         args[e][1] = attack_mapping[the attacker's encoding] bits
 *   GW_OP_OBSERVE         PositionCenteredEncodingObserver.get_obs(lane): writes
 *                         obs[e][lane] only (draws in call order); args[e][0] =
 *                         observe_self (NULL args: the config's)
 *   The components' own parameters travel with each call, so several actors
 *   or observers with different parameters may share one handle.
 *   args     device int32[E][gw_act_dim(h)]
 *   result   device int32[E][2 + A] or NULL: [0] status (MOVE 1 True, 0 False,
 *            -1 None for a non-MovingAgent; ATTACK 1 attempted, 0 not; resets 1
 *            placed, 0 raised), [1] n attacked, [2..] attacked lanes in list order
 *   obs      device int32[E][A][S][S] (OBSERVE)
 *   err_flags device uint32[E] or NULL (|= GW_ERR_*)                          */
#define GW_OP_POSITION_RESET 1
#define GW_OP_HEALTH_RESET   2
#define GW_OP_MOVE           3
#define GW_OP_ATTACK         4
#define GW_OP_OBSERVE        5
/*   GW_OP_MAZE_RESET      MazePlacementState.reset (state.py:500-619): the maze
 *                         generated from the target's cell (generate_maze,
 *                         utils.py:120-212, draws from the env's stream), the
 *                         target placed there, initial-position entities, then
 *                         barrier / free entities on maze walls / passages;
 *                         args[e][0] = no_overlap_at_reset | cluster_barriers << 1 |
 *                         scatter_free_agents << 2 | variant << 3 | target lane << 8,
 *                         args[e][1] = barrier_encodings bits, args[e][2] =
 *                         free_encodings bits.  variant 1 =
 *                         TargetBarriersFreePlacementState.reset (state.py:279-382):
 *                         no maze, every cell available to both kinds.
 *                         Every entity must be a lane (gw_config.all_lanes);
 *                         result[e][0] = 1 placed, 0 raised (err_flags:
 *                         GW_ERR_NO_CELL / GW_ERR_INIT_POSITION).               */
#define GW_OP_MAZE_RESET     6
/*   GW_OP_CROSS_MOVE      CrossMoveActor.process_action(lane, {'move': args[e][0]})
 *                         (actor.py:161-192): 0 stay, 1 left, 2 down, 3 right, 4 up
 *                         (the host asserts the range, actor.py:152); result[e][0]
 *                         as GW_OP_MOVE
 *   GW_OP_DRIFT_MOVE      DriftMoveActor.process_action (actor.py:208-234):
 *                         args[e][0] the cross action, args[e][1] the agent's
 *                         orientation (1..4, 0 = None); result[e][0] 1 / 0 / -1
 *                         None (not Orientation + Moving) / -2 a drift without an
 *                         orientation (the reference's AssertionError),
 *                         result[e][1] = 1 when the drift ran (the reference then
 *                         replaced action_dict['move'] by the orientation),
 *                         result[e][2] = the orientation afterwards
 *   GW_OP_ORIENT_RESET    OrientationState.reset (state.py:666-675): initial or
 *                         np.random.randint(1, 5) per OrientationAgent in agent
 *                         order; result[e][2 + lane] = the lane's orientation (0:
 *                         not an OrientationAgent); result required
 *   GW_OP_OBSERVE_ABS     AbsoluteEncodingObserver.get_obs(lane) (observer.py:95-150),
 *                         blocking entities included, any view range (args[e][0];
 *                         NULL args: the spec's): writes obs[e][lane][rows][cols]
 *                         (obs device int32[E][A][rows][cols])
 *   The orientation lives with the caller (the component runtime uploads it
 *   per call); the engine's flags keep no orientation for these handles.   */
#define GW_OP_CROSS_MOVE     7
#define GW_OP_DRIFT_MOVE     8
#define GW_OP_ORIENT_RESET   9
#define GW_OP_OBSERVE_ABS   10
gw_status gw_component(gw_handle h, int32_t op, int32_t lane, const int32_t* args, int32_t* result,
                       int32_t* obs, uint32_t* err_flags, void* stream);

/* A fragment of n_steps consecutive AllStepManager steps with auto-reset
   (1 SAME_STEP, 2 NEXT_STEP) in one call: the same results as n_steps
   calls of gw_step_autoreset / gw_step_autoreset_next with actions[t], but
   the one-wave kernel runs each env's steps back to back in ONE launch (no
   launch-wide barrier between steps; lane state, RNG and cell table stay on
   chip).  Per-step slabs:
     actions     device int32[n][E][A][gw_act_dim(h)]   (inputs, resident)
     obs         device int32[n][E][A][obs shape]
     reward      device double[n][E][A];  done  device uint8[n][E][A]
     all_done    device uint8[n][E]       ('__all__' of every step)
     all_done_in device uint8[E] or NULL  (in/out: the '__all__' before step
                 0, e.g. the previous fragment's; NULL = none set.  Overwritten
                 with the last step's '__all__' = slab n-1, so consecutive
                 fragments pass the same buffer)
     acting      device uint64[E] or NULL (+= acting agents over the steps)
   skip_done_obs = 1: obs rows of entities that get no observation in a
   step (done before it, or not grid observers) are left unwritten in that
   step's slab instead of being filled with -2 (the reference returns no obs
   for them; mask with done).  The Pacman kernel runs it in one launch too
   (rows always written).  The workgroup-per-env kernel runs it in one
   launch too, the env's state on chip across its steps; with
   skip_done_obs it writes only the rows of the lanes in [obs_lo, obs_hi)
   (the contiguous range of grid-observer lanes, fixed at gw_create),
   rounded out to whole 16-byte stores: rows of lanes that are not grid
   observers are unspecified there, as on the one-wave kernel, and rows of
   done observers inside the range hold -2.
   The handle's persistent obs rows (gw_config.persistent_obs) are not used. */
gw_status gw_rollout(gw_handle h, int32_t n_steps, const int32_t* actions, int32_t* obs, double* reward,
                     uint8_t* done, uint8_t* all_done, uint8_t* all_done_in, uint64_t* acting,
                     int32_t horizon, int32_t autoreset, int32_t skip_done_obs, uint32_t* err_flags,
                     void* stream);

/* Timing hook (no reference counterpart: instrumentation of the launch the
   reference's step loop is timed around).  The NEXT kernel launch of the
   handle's step / reset kernels (gw_step*, gw_rollout, gw_rollout_step's
   step, gw_turn_step, gw_turn_rollout, gw_reset ...) records start_event
   when its kernel starts and stop_event when it ends,
   as part of the kernel dispatch (hipExtLaunchKernel), so a timed region
   needs no event record calls around the launch; the events (hipEvent_t,
   created by the caller) are cleared by that launch.  Both NULL: clear.   */
gw_status gw_set_launch_events(gw_handle h, void* start_event, void* stop_event);

/* One step of a synthetic random-policy rollout in one call: gw_random_actions
   into `actions`, then on the same stream gw_step (autoreset 0),
   gw_step_autoreset (1) or gw_step_autoreset_next (2) on those actions.  The
   outputs are those of the step call.  (AllStepManager protocol; the Pacman
   program's turn-based protocol is gw_turn_step.)                           */
gw_status gw_rollout_step(gw_handle h, uint64_t key, uint32_t step, uint32_t env_offset,
                          int32_t* actions, int32_t* obs, double* reward, uint8_t* done,
                          uint8_t* all_done, uint64_t* acting, int32_t horizon, int32_t autoreset,
                          uint32_t* err_flags, void* stream);

/* ---------------------------------------------------------------------
 * Pacman program (GW_SIM_PACMAN): the turn-based and simulation-only
 * protocols.  Entities of GW_K_FOOD are passive (one bit per env, not a
 * lane); observations are AbsoluteEncodingObserver grids, int32[E][A][rows][cols]
 * (gw_obs_shape).  Actions: actions[e][a] = {cross_move 0..4, unused, present};
 * present < 0 marks an agent that is not in the action dict.
 * ------------------------------------------------------------------- */

/* TurnBasedManager.reset (managers/turn_based_manager.py:22-32) of the envs
   with mask[e] != 0 (all when NULL): SmartGWS.reset, then the observation of
   the next agent of the (never restarted) turn cycle only.
     returned  device uint8[E][A]: 1 for the lane whose obs was written
     turn      device int32[E]:    the lane whose action the next call takes */
gw_status gw_turn_reset(gw_handle h, const uint8_t* mask, int32_t* obs, uint8_t* returned,
                        int32_t* turn, uint32_t* err_flags, void* stream);

/* TurnBasedManager.step (turn_based_manager.py:34-94) with NEXT_STEP
   auto-reset: the lane turn[e] acts (its action row), then the outputs of the
   agents the manager returns — the next live agent of the cycle, or every
   live agent once '__all__' — are written (returned[e][a] = 1); reward is the
   agent's accumulated reward since it last received one.  An env whose
   previous call ended it (all_done[e] on input, or steps >= horizon > 0) is
   reset instead (gw_turn_reset outputs, reward 0, all_done 0).            */
gw_status gw_turn_step(gw_handle h, const int32_t* actions, int32_t* obs, double* reward,
                       uint8_t* done, uint8_t* all_done, uint8_t* returned, int32_t* turn,
                       uint64_t* acting, int32_t horizon, uint32_t* err_flags, void* stream);

/* n_steps consecutive gw_turn_step calls in ONE launch (each env's wave runs
   its turns back to back; lanes, cell table, food bits and stream stay on
   chip): actions[t] feeds turn t, whose outputs go to slab t of
     obs device int32[n][E][A][rows][cols] (rows of lanes not returned in
         turn t are left unwritten: mask with returned),
     reward double[n][E][A], done / returned uint8[n][E][A],
     all_done uint8[n][E], turn int32[n][E];
   all_done_in device uint8[E] or NULL: in/out as in gw_rollout (the
   '__all__' before turn 0; overwritten with the last turn's).            */
gw_status gw_turn_rollout(gw_handle h, int32_t n_steps, const int32_t* actions, int32_t* obs,
                          double* reward, uint8_t* done, uint8_t* all_done, uint8_t* all_done_in,
                          uint8_t* returned, int32_t* turn, uint64_t* acting, int32_t horizon,
                          uint32_t* err_flags, void* stream);

/* The simulation alone, for a manager that lives in the host (the dict API):
   gw_sim_reset = SmartGWS.reset (no observation drawn); gw_sim_step =
   sim.step(action_dict) (reward[e][a] = the agent's accumulated reward, not
   consumed; done = get_done; all_done = get_all_done); gw_observe =
   get_obs(lane) for every env, drawing in call order (observer.py:131-134). */
gw_status gw_sim_reset(gw_handle h, const uint8_t* mask, uint32_t* err_flags, void* stream);
gw_status gw_sim_step(gw_handle h, const int32_t* actions, double* reward, uint8_t* done,
                      uint8_t* all_done, uint32_t* err_flags, void* stream);
gw_status gw_observe(gw_handle h, int32_t lane, int32_t* obs, void* stream);

/* Program state beside gw_get_state: reward accumulators double[E][A]
   (SmartGWS.rewards), passive entities still on the grid uint32[E][ceil(P/32)]
   (P = gw_num_passive), the turn cycle position int32[E] (-1 before the
   first reset).  NULL pointers are skipped.                                 */
gw_status gw_get_aux_state(gw_handle h, double* racc, uint32_t* passive_bits, int32_t* turn_pos,
                           void* stream);
gw_status gw_set_aux_state(gw_handle h, const double* racc, const uint32_t* passive_bits,
                           const int32_t* turn_pos, void* stream);

gw_status gw_destroy(gw_handle h);

/* PositionState(randomize_placement_order=True) (state.py:97-101): the
   order in which the next resets place each env's lanes, lane_order[E][A]
   (host memory; a permutation of 0..A-1 per env: the shuffled agents dict,
   static entities left out -- they overlap nothing, so their place in the
   order changes nothing).  n = 0 restores agents-dict order.  One-wave
   kernel only (a MazeNavigation handle leaves the one-lane kernel).       */
gw_status gw_set_placement_order(gw_handle h, const int32_t* lane_order, int32_t n);

/* AllStepManager(randomize_action_input=True) (all_step_manager.py:62-65):
   the order of the action dict the next steps process, lane_order[E][A]
   (host memory; per env a permutation of 0..A-1: the lanes in the shuffled
   dict first, the others after).  The attack and move passes of the
   TeamBattle (team_battle_example.py:33-59) and ReachTheTarget
   (reach_the_target.py:95-126) programs and the TrafficCorridor moves
   (traffic_corridor.py:41-49) and the Pacman program's baddie moves
   (pacman.py:104-117) go in that order, and movers enter their cells in it.
   n = 0 restores agents-dict order.  One-wave kernels only.                 */
gw_status gw_set_action_order(gw_handle h, const int32_t* lane_order, int32_t n);

/* generate_maze(rows, cols, start) (sim/gridworld/utils.py:120-212) in every
   env, drawing from the env's np.random stream: Prim's algorithm with the
   frontier in CPython's list(set(...)) order, exactly as the reference.
     start  device int32[E][2] (row, col), a negative row = start None
            (np.random.randint(1, shape - 1)); NULL = None for every env;
            a start outside the maze leaves the env's stream untouched and
            its maze all -1
     maze   device int8[E][rows][cols]: 0 passage, 1 wall                     */
gw_status gw_generate_maze(gw_handle h, const int32_t* start, int8_t* maze, void* stream);

/* Introspection */
int32_t     gw_num_envs(gw_handle h);
int32_t     gw_obs_side(gw_handle h);
/* per-lane observation shape: (S, S) position-centred, (rows, cols) absolute */
gw_status   gw_obs_shape(gw_handle h, int32_t* rows, int32_t* cols);
int32_t     gw_num_passive(gw_handle h);
int32_t     gw_num_lanes(gw_handle h);
/* the step kernel's execution model: GW_KERNEL_WAVE (one wavefront per env),
   GW_KERNEL_WORKGROUP (ReachTheTarget: one workgroup of ceil(A/64) waves per
   env), GW_KERNEL_PACMAN (the Pacman program, one wavefront per env),
   GW_KERNEL_LANE (MazeNavigation: one lane per env, 64 envs per wave)       */
#define GW_KERNEL_WAVE      0
#define GW_KERNEL_WORKGROUP 1
#define GW_KERNEL_PACMAN    2
#define GW_KERNEL_LANE      3
int32_t     gw_env_kernel(gw_handle h);
int32_t     gw_act_dim(gw_handle h);
/* Resident workgroups per CU of this engine's step launch (the HIP occupancy
   calculator on its kernel, block size and dynamic LDS); block_threads and
   lds_bytes (either may be NULL) receive that block size and LDS.  A launch
   of E envs runs in ONE dispatch round when E <= blocks_per_cu * CUs (for
   the workgroup kernel one env = one workgroup; the lane kernel packs
   several envs per workgroup).  No reference counterpart: a diagnostic of
   the launch shape.                                  */
gw_status   gw_step_occupancy(gw_handle h, int32_t* blocks_per_cu, int32_t* block_threads, int64_t* lds_bytes);
/* entity index (into gw_config.agents) of each lane; out: host int32[A]     */
gw_status   gw_lane_entities(gw_handle h, int32_t* out);
const char* gw_last_error(void);
int32_t     gw_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GW_ENGINE_H */
