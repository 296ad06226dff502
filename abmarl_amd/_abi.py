"""ctypes mirror of ``include/gw_engine.h`` (constants and config structs).

Only plain C types cross the boundary: the engine takes device pointers as
integers (``tensor.data_ptr()``) and streams as ``void*``.
"""
import ctypes as C

GW_MAX_AGENTS = 64
GW_MAX_LANES = 256
GW_KERNEL_WAVE, GW_KERNEL_WORKGROUP, GW_KERNEL_PACMAN, GW_KERNEL_LANE = 0, 1, 2, 3
GW_MAX_ENTITIES = 4096
GW_MAX_ENC = 15
GW_MAX_CELLS = 16384
GW_MAX_RANGE = 64
GW_MAX_ATTACK_RANGE = 7
GW_FIXED_RANGE = 7          # windows up to this range are compiled per side (engine-internal)
GW_ACT_DIM = 3
GW_MT_N = 624
GW_MT_STRIDE = 704

GW_OK = 0
GW_E_INVALID = -1
GW_E_HIP = -2
GW_E_UNSUPPORTED = -3

GW_ERR_NO_CELL = 1
GW_ERR_INIT_POSITION = 2
GW_ERR_DOUBLE_REMOVE = 4
GW_ERR_TUNNEL_PLACE = 8
GW_ERR_NOT_IN_GRID = 16
GW_ERR_VALUE_ERROR = 32

GW_OP_POSITION_RESET = 1
GW_OP_HEALTH_RESET = 2
GW_OP_MOVE = 3
GW_OP_ATTACK = 4
GW_OP_OBSERVE = 5
GW_OP_MAZE_RESET = 6
GW_OP_CROSS_MOVE = 7
GW_OP_DRIFT_MOVE = 8
GW_OP_ORIENT_RESET = 9
GW_OP_OBSERVE_ABS = 10

GW_K_OBSERVING = 0x01
GW_K_ACTING = 0x02
GW_K_GRID_OBSERVER = 0x04
GW_K_MOVING = 0x08
GW_K_ATTACKING = 0x10
GW_K_HEALTH = 0x20
GW_K_PROGRAM = 0x80
GW_K_BLOCKING = 0x40
GW_K_ORIENTATION = 0x100
GW_K_FOOD = 0x200
GW_K_LANE = 0x400
GW_K_AMMO = 0x800

GW_SIM_TEAM_BATTLE = 1
GW_SIM_MAZE_NAV = 2
GW_SIM_REACH_TARGET = 3
GW_SIM_PACMAN = 4
GW_SIM_TRAFFIC = 5

GW_OBS_POSITION_CENTERED = 0
GW_OBS_ABSOLUTE = 1

GW_ATTACK_BINARY = 0
GW_ATTACK_SELECTIVE = 1

GW_DONE_ACTIVE = 0x1
GW_DONE_ONE_TEAM = 0x2
GW_DONE_TARGET_AGENT = 0x4
GW_DONE_TARGET_DESTROYED = 0x8

GW_ORDER_POSITION_HEALTH = 0
GW_ORDER_HEALTH_POSITION = 1

# flags bits in gw_get_state
FLAG_IN_GRID = 1
FLAG_LIVE = 2
FLAG_ACTIVE = 4
FLAG_OBS_M2 = 0x40   # engine-internal (gw_config.persistent_obs): the lane's obs row holds -2


class AgentSpec(C.Structure):
    _fields_ = [
        ("encoding", C.c_int32),
        ("kind", C.c_uint32),
        ("init_row", C.c_int32),
        ("init_col", C.c_int32),
        ("view_range", C.c_int32),
        ("move_range", C.c_int32),
        ("attack_range", C.c_int32),
        ("simultaneous_attacks", C.c_int32),
        ("attack_strength", C.c_double),
        ("attack_accuracy", C.c_double),
        ("initial_health", C.c_double),
        ("initial_orientation", C.c_int32),
        ("done_target", C.c_int32),
        ("destroy_target", C.c_int32),
        ("initial_ammo", C.c_int32),
    ]

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        # entity indices; -1 = not in the done component's target_mapping
        if 'done_target' not in kwargs:
            self.done_target = -1
        if 'destroy_target' not in kwargs:
            self.destroy_target = -1


class Config(C.Structure):
    _fields_ = [
        ("rows", C.c_int32),
        ("cols", C.c_int32),
        ("n_agents", C.c_int32),
        ("sim_kind", C.c_int32),
        ("overlap", C.c_uint32 * (GW_MAX_ENC + 1)),
        ("attack_mapping", C.c_uint32 * (GW_MAX_ENC + 1)),
        ("stacked_attacks", C.c_int32),
        ("observe_self", C.c_int32),
        ("no_overlap_at_reset", C.c_int32),
        ("state_order", C.c_int32),
        ("done_kind", C.c_uint32),
        ("obs_range", C.c_int32),
        ("target_agent", C.c_int32),
        ("nav_agent", C.c_int32),
        ("agents", C.POINTER(AgentSpec)),
        ("attack_kind", C.c_int32),
        ("obs_kind", C.c_int32),
        ("pacman_agent", C.c_int32),
        ("tunnel", C.c_int32 * 4),
        ("pac_rewards", C.c_double * 5),
        ("force_workgroup", C.c_int32),
        ("persistent_obs", C.c_int32),
        ("all_lanes", C.c_int32),
        ("env_per_lane", C.c_int32),
        ("component_api", C.c_int32),
        ("attack_array_as_list", C.c_int32),
    ]


class CompiledConfig:
    """Owns a ``Config`` and the ``AgentSpec`` array it points to."""

    def __init__(self, rows, cols, specs, sim_kind, overlap, attack_mapping,
                 stacked_attacks=False, observe_self=True, no_overlap_at_reset=False,
                 state_order=GW_ORDER_POSITION_HEALTH, done_kind=GW_DONE_ACTIVE,
                 obs_range=0, target_agent=-1, nav_agent=-1, attack_kind=0,
                 obs_kind=GW_OBS_POSITION_CENTERED, pacman_agent=-1, tunnel=(-1, -1, -1, -1),
                 pac_rewards=(0.0, 0.0, 0.0, 0.0, 0.0), force_workgroup=False):
        self.n_agents = len(specs)
        self._specs = (AgentSpec * max(1, self.n_agents))()
        for i, s in enumerate(specs):
            self._specs[i] = s
        cfg = Config()
        cfg.rows, cfg.cols, cfg.n_agents, cfg.sim_kind = rows, cols, self.n_agents, sim_kind
        for e in range(GW_MAX_ENC + 1):
            cfg.overlap[e] = int(overlap.get(e, 0))
            cfg.attack_mapping[e] = int(attack_mapping.get(e, 0))
        cfg.stacked_attacks = int(bool(stacked_attacks))
        cfg.observe_self = int(bool(observe_self))
        cfg.no_overlap_at_reset = int(bool(no_overlap_at_reset))
        cfg.state_order = state_order
        cfg.done_kind = done_kind
        cfg.obs_range = obs_range
        cfg.target_agent = target_agent
        cfg.nav_agent = nav_agent
        cfg.agents = C.cast(self._specs, C.POINTER(AgentSpec))
        cfg.attack_kind = attack_kind
        cfg.obs_kind = obs_kind
        cfg.pacman_agent = pacman_agent
        for i in range(4):
            cfg.tunnel[i] = int(tunnel[i])
        for i in range(5):
            cfg.pac_rewards[i] = float(pac_rewards[i])
        cfg.force_workgroup = int(force_workgroup)   # 0 auto, 1 workgroup kernel, 2..4 waves per env
        self.cfg = cfg
        self.rows, self.cols = rows, cols
        self.obs_kind = obs_kind
        self.obs_side = 2 * obs_range + 1
        # per-entity observation shape (gw_obs_shape)
        self.obs_shape = (rows, cols) if obs_kind == GW_OBS_ABSOLUTE else (self.obs_side,) * 2
        self.specs = list(specs)
        self.randomize_placement_order = False
        self.attack_kind = attack_kind

    @property
    def act_dim(self):
        """gw_config_act_dim (include/gw_engine.h)."""
        if self.attack_kind != GW_ATTACK_SELECTIVE:
            return GW_ACT_DIM
        r = max([s.attack_range for s in self.specs if s.kind & GW_K_ATTACKING] or [0])
        return 2 + (2 * r + 1) ** 2

    def ptr(self):
        return C.byref(self.cfg)
