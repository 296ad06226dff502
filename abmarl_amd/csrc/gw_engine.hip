// gw_engine.hip — MI355X (gfx950) batched GridWorld step engine.
//
// Execution model: ONE WAVEFRONT PER ENVIRONMENT, one lane per entity
// (A <= 64).  The reference's step is a sequence of Python loops over the
// agents dict whose random draws come from one sequential MT19937 stream
// (numpy legacy RandomState).  Whatever changes the RNG stream or the grid in
// reference order is kept in reference order here; everything else is
// lane-parallel:
//
//   attack pass (team_battle_example.py:35-47, actor.py:306-501)
//       a lane-parallel pre-check on the LDS cell table finds the attackers
//       whose window holds no possible target (they only take the -0.1);
//       the others run serially in agent order: one ballot = the window scan,
//       candidates ordered by (window cell, in-cell insertion order) with
//       ballot ranks, accuracy / permutation draws in reference order.
//   move pass   (team_battle_example.py:50-55, actor.py:82-114)
//       movers whose source/target cells no other mover touches are resolved
//       in parallel against the post-attack cell table; the rest run serially
//       in agent order with Grid.query as one ballot.
//   observation (all_step_manager.py:68-71, observer.py:204-250)
//       lane-parallel: each window row is 2-3 LDS dword reads of a padded
//       byte table (0 empty, enc single, 0x80 crowded, 0xFF off-grid); the
//       rare crowded cells (np.random.choice draws) are resolved afterwards in
//       (agent, row, col) order; int8 staging -> coalesced int32 stores.
//   reward / done / __all__ (smart.py:101-117, done.py:39-56,140-153,
//       all_step_manager.py:72-93): lane-parallel + ballots / DPP reductions.
//   auto-reset (optional, same launch): AllStepManager.reset for the envs
//       whose episode ended (PositionState / HealthState / observation).
//
// The grid's insertion-ordered dict cells are represented by a per-agent
// placement sequence number (seq): the order of agents inside a cell is the
// order of their seq.  No grid array lives in HBM; LDS tables are rebuilt per
// launch from the agents' positions.
//
// Data layout in HBM (SoA, env-major, lane-contiguous => coalesced):
//   pos[E][A] int2, health[E][A] f64, flags[E][A] u8, seq[E][A] u32,
//   mt[E][704] u32 (key[624], pos @624, seq counter @625, cached block base
//   @626, 64 tempered words from it @640), steps[E] i32.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdarg.h>
#include <stdlib.h>
#include <vector>
#include <type_traits>

#include "../../include/gw_engine.h"

#define WAVE 64
#define F_IN_GRID 1u
#define F_LIVE 2u
#define F_ACTIVE 4u
#define F_OBS_M2 0x40u      // persistent obs buffer: this lane's row holds -2 (engine-internal)
#define MT_POS_SLOT 624
#define MT_CTR_SLOT 625
#define MT_CBASE_SLOT 626   // base of the cached tempered block (0xFFFFFFFF: none)
#define MT_CACHE 640        // [64] tempered key[cbase + i]
#define SEQ_RENORM (1u << 23)
#define CELL_CROWD 0x80u
// observation windows up to this range (S <= 15) are compiled per window side
// (the parts, -DGW_PART_S); wider ones run the generic path (part 0)
#define GW_FIXED_RANGE 7
#define CELL_OFF 0xFFu
// lane_step_kernel (gw_lane.inc): lanes per env for an S x S window (the
// window's cell count rounded up to 16, 32 or 64; host and device)
__host__ __device__ constexpr int lane_group(int S) { return S * S <= 16 ? 16 : (S * S <= 32 ? 32 : 64); }

// create_grid_and_mask (utils.py:46-115): does a blocker at offset (rd, cd)
// from the observer hide the cell at offset (r, c)?  The eight cases differ
// only in the half-plane scanned and in the +-0.5 offsets of the two rays;
// the arithmetic is the reference's, in double.  Whether a cell is hidden
// does not depend on the mask range (the range only bounds the scan), so
// one function serves every range (host LUTs, device on the fly).
__host__ __device__ inline bool shadow_hides(int rd, int cd, int r, int c)
{
    if ((rd == 0 && cd == 0) || (r == rd && c == cd)) return false;    // not the blocker itself
    const double r_d = rd, c_d = cd;
    if (cd == 0) {                                          // below / above: rays in c
        if (rd > 0 ? r < rd : r > rd) return false;
        const double dd = rd > 0 ? -0.5 : 0.5;
        const double left = (c_d - 0.5) / (r_d + dd) * r, right = (c_d + 0.5) / (r_d + dd) * r;
        return left < c && c < right;
    }
    if (cd > 0 ? c < cd : c > cd) return false;             // rays in r
    if (rd > 0 && r < rd) return false;
    if (rd < 0 && r > rd) return false;
    // offsets of (rd -+ 0.5) / (cd + lo_d | up_d) per case
    double lo_d, up_d;
    if (rd == 0) { lo_d = up_d = cd > 0 ? -0.5 : 0.5; }             // right / left
    else if ((rd > 0) == (cd > 0)) { lo_d = 0.5; up_d = -0.5; }     // below-right / above-left
    else { lo_d = -0.5; up_d = 0.5; }                               // below-left / above-right
    const double lo = (r_d - 0.5) / (c_d + lo_d) * c, up = (r_d + 0.5) / (c_d + up_d) * c;
    return lo < r && r < up;
}

namespace {

// ------------------------------------------------------------ device config
struct DevAgent {               // per-entity constants (spec table in HBM)
    int32_t enc;
    uint32_t kind;
    uint32_t ov, amap;          // overlap / attack-mapping masks of enc (no dependent load)
    int32_t init_r, init_c;
    int32_t view_range, move_range, attack_range, simul;
    double strength, accuracy, init_health;
    int32_t init_orient;
    // done components' targets (gw_agent_spec.done_target / destroy_target):
    // the target's lane, -1 not mapped, -2 a static entity (at tgt_pos =
    // row << 16 | col, always active)
    int32_t tgt_lane, tgt_pos, dtgt_lane;
    int32_t init_ammo;          // AmmoAgent.initial_ammo (GW_K_AMMO)
};

struct Params {
    // engine state
    int2* pos; double* health; uint8_t* flags; uint32_t* seq; uint32_t* mt; int32_t* steps;
    int32_t* ammo;                         // [E][A] AmmoAgent.ammo (0 for other lanes)
    const DevAgent* spec;
    // I/O
    const int32_t* actions; int32_t* obs; double* reward; uint8_t* done; uint8_t* all_done;
    uint64_t* acting; uint32_t* err;
    const uint8_t* mask; const uint8_t* prev_all_done; int32_t horizon; int32_t autoreset;
    uint64_t* stamps;   // diagnostic build only (-DGW_STAMPS): [E][32] s_memtime
    uint32_t* dbg;      // diagnostic build only (-DGW_CHECKS): [16] first violation
    // config
    int32_t E, A, H, W, max_enc, sim_kind, nav, target;
    int32_t observe_self, stacked, no_overlap_at_reset, state_order;
    int32_t arr_as_list;                   // gw_config.attack_array_as_list
    uint32_t done_kind;
    int32_t pad, pitch, tbl_rows;          // padded byte table geometry
    int32_t pair_cap;                      // crowded (observer, cell) pairs that fit after the obs stage
    int32_t act_dim;                       // ints per entity action (gw_config_act_dim)
    int32_t attack_kind;                   // GW_ATTACK_*
    const uint4* tbl_tmpl;                 // empty padded table (0xFF border), 16-B granules
    const uint4* ob_tmpl;                  // the same unpadded, row-major [H][W] (Pacman's copy)
    uint32_t overlap[GW_MAX_ENC + 1];
    uint32_t amap[GW_MAX_ENC + 1];
    // static entities (gw_engine.h "Entities and lanes") and blocking
    int32_t n_free;                        // cells not held by a static entity
    const uint16_t* free_cell;             // [n_free] free index -> cell; NULL = identity
    const uint16_t* cell_free;             // [HW] cell -> free index
    const uint32_t* static_bits;           // [ceil(HW/32)] static cells; NULL = none
    uint32_t static_encs;                  // encodings of static entities (always active)
    int32_t blockers;                      // any blocking entity
    int32_t lane_blockers;                 // any blocking lane
    // shadow LUT: range r, blocker at (dr, dc): mask_words(r) words at
    // shadow_off[r] + ((dr+r)(2r+1) + dc+r) * mask_words(r); bit k = window
    // cell k (row-major) hidden (utils.py:46-115)
    const uint32_t* shadow;
    // hidden cells due to static blockers for an entity at `cell`, range r:
    // smask_off[r] + cell * mask_words(r) (smask_off[r] < 0: not built)
    const uint32_t* smask;
    int32_t shadow_off[GW_FIXED_RANGE + 1];
    int32_t smask_off[GW_FIXED_RANGE + 1];
    // Pacman program (GW_SIM_PACMAN, gw_pacman.inc)
    int32_t obs_kind, pacman, mode, obs_lane;
    int32_t tunnel[4];
    double prw[5];                         // bad_move, entropy, eat_food, kill, die
    int32_t n_passive, pwords;             // passive entities (food), bit words per env
    const int16_t* passive_cell;           // [n_passive] cell
    const int16_t* cell_passive;           // [HW] passive index | encoding << 8, -1 = none
    const uint32_t* passive_cnt;           // [ceil(HW/4)] packed u8: passive entities per cell
    const int8_t* passive_enc;             // [n_passive]
    uint32_t* pbits;                       // [E][pwords] passive present
    double* racc;                          // [E][A] SmartGWS.rewards accumulators
    int32_t* cyc;                          // [E] TurnBasedManager cycle position (lane)
    uint8_t* returned;                     // [E][A] lanes in the returned dicts
    int32_t* turn;                         // [E] lane whose action the next call takes
    uint64_t agent_lanes;                  // lanes that are Agents (the turn cycle)
    // ReachTheTarget on a workgroup per env (gw_rtt.inc)
    int32_t nwv;                           // waves per env (blockDim = 64 * nwv)
    int32_t obs_lo, obs_hi;                // lanes [obs_lo, obs_hi) hold every grid observer
    int32_t par_moves;                     // no Grid.query can refuse a mover: parallel move pass
    int32_t place_par;                     // placement without duplicate removals: parallel (Jacobi)
    int32_t persistent_obs;                // gw_config.persistent_obs: skip rows already -2
    // gw_rollout: steps per launch (1 for the single-step calls), the
    // previous call's __all__ (NEXT_STEP input; the single-step calls pass
    // all_done itself), rows of lanes without an observation left unwritten
    int32_t nsteps;
    const uint8_t* ad_in;
    uint8_t* ad_out;                       // gw_rollout: the last step's __all__ (may alias ad_in)
    // PositionState(randomize_placement_order=True): per env, the lanes in
    // placement order ([E][A], gw_set_placement_order; NULL = lane order)
    const int32_t* place_order;
    // AllStepManager(randomize_action_input=True): per env, the lanes in
    // action-dict order and each lane's rank in it ([E][A] each,
    // gw_set_action_order; NULL = agents-dict order).  Generic kernel only.
    const int32_t* act_order;
    const int32_t* act_rank;
    int32_t skip_done_obs;
    // observers with different view ranges: slot-geometry (S x S) shadow LUT
    // and static-blocker masks per range (bit wr * S + wc), offsets per range
    // gw_component: the op's result rows [E][2 + A] and the observed lane
    // of OBSERVE (-1 otherwise: every live observer)
    int32_t* comp_out;
    int32_t obs_only;
    int32_t comp_amap;                     // wg_comp_kernel ATTACK: the attacker's attack_mapping bits (-1: the table's)
    int32_t hetero_view;
    const uint32_t* hshadow;
    const uint32_t* hsmask;
    int32_t hshadow_off[GW_FIXED_RANGE + 1];
    int32_t hsmask_off[GW_FIXED_RANGE + 1];
    // the generic window path (observe_big, obs_side > 2 * GW_FIXED_RANGE + 1)
    int32_t obs_side;                      // S at run time
    const int32_t* sblk;                   // static blocking entities: (row << 16) | col
    int32_t n_sblk;
};

__host__ __device__ inline int mask_words(int r)
{
    const int d = 2 * r + 1;
    return (d * d + 31) >> 5;
}

// ------------------------------------------------------------ wave helpers
__device__ __forceinline__ void wave_sync()
{
    // one wavefront per env: LDS ops of a wave complete in order; this keeps
    // the compiler from moving LDS accesses across cross-lane hand-offs.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The lane id through a volatile asm: the step loop (gw_rollout) would
// otherwise let the compiler hoist every lane-derived address and mask out of
// the loop and keep them live in VGPRs across all of it (179 VGPRs and
// scratch spills instead of 124).  Recomputing it costs two VALU per use.
__device__ __forceinline__ int lane_id()
{
    int v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
    return v;
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint32_t rl(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int32_t rl(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ bool rlb(bool v, int l) { return __builtin_amdgcn_readlane((int)v, l) != 0; }

// raw buffer resource word 3 for gfx9 (data format 32, no swizzle, no stride)
#define BUF_RSRC_W3 0x00020000
// an offset past any buffer's range (< 2^31 bytes): the store is dropped
#define BUF_OOB ((int)0x80000000)
// cache policy of the observation stores: slc (streaming, non-temporal),
// measured -11..16% on the headline workload
constexpr int GW_OBS_STORE_AUX = 2;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// four observation bytes (valid values >= -2, 0x80 = skipped) -> four int32
// max(sext(byte), -2) with SDWA byte selects (one VALU per output), stored
// as one dwordx4 at voff + ioff of the buffer (voff out of range = dropped)
__device__ __forceinline__ void buf_store_i8x4(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int ioff, uint32_t w)
{
    const int m2 = -2;
    int v0, v1, v2, v3;
    asm("v_max_i32_sdwa %0, sext(%1), %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD"
        : "=v"(v0) : "v"(w), "v"(m2));
    asm("v_max_i32_sdwa %0, sext(%1), %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
        : "=v"(v1) : "v"(w), "v"(m2));
    asm("v_max_i32_sdwa %0, sext(%1), %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
        : "=v"(v2) : "v"(w), "v"(m2));
    asm("v_max_i32_sdwa %0, sext(%1), %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
        : "=v"(v3) : "v"(w), "v"(m2));
    const u32x4 v = {(uint32_t)v0, (uint32_t)v1, (uint32_t)v2, (uint32_t)v3};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)voff + ioff, 0, GW_OBS_STORE_AUX);
}

// The kernel's Params (its only / first argument, at kernarg offset 0) read
// afresh: the kernarg segment pointer passed through an empty asm, so loads
// of its fields after this point cannot be hoisted above it.  A step loop
// calls it once per iteration: the fields become scalar loads from the
// kernarg segment (scalar cache) at their use instead of loop-invariant
// values -- and the 64-bit lane masks of every loop-invariant config test --
// held live across the loop, which overflow the SGPR file and spill into
// VGPR lanes (a v_writelane / v_readlane pair per reload, VALU work).
struct Params;
__device__ __forceinline__ const Params& kernel_params()
{
    typedef const __attribute__((address_space(4))) Params KParams;
    KParams* q = (KParams*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(q));
    return *(const Params*)q;
}

__device__ __forceinline__ double rld(double v, int l)
{
    uint64_t b = __double_as_longlong(v);
    uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l);
    uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int first_lane(uint64_t m) { return (int)__builtin_ctzll(m); }

// s_setprio with a wave-uniform level (0..3; the instruction takes an immediate)
__device__ __forceinline__ void set_prio(int v)
{
    switch (v) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
    }
}

// ------------------------------------------------------------ checked build
// -DGW_CHECKS: every data-dependent LDS index and every "exactly one lane"
// ballot is validated; a violation is recorded in p.dbg and the access is
// redirected to index 0 (the build cannot fault).  Never the shipped build.
#ifdef GW_CHECKS
__device__ __noinline__ void chk_fail(uint32_t* dbg, int code, int v0, int v1)
{
    if (!dbg) return;
    if (atomicOr(&dbg[0], 1u << code) == 0u) {
        dbg[1] = (uint32_t)code; dbg[2] = (uint32_t)v0; dbg[3] = (uint32_t)v1;
        dbg[4] = blockIdx.x; dbg[5] = (uint32_t)__lane_id();
    } else {
        atomicAdd(&dbg[6], 1u);
    }
}
#define CIDX(idx, lim, code) \
    ([&](int _i, int _l) { if (_i < 0 || _i >= _l) { chk_fail(p.dbg, (code), _i, _l); return 0; } return _i; }((idx), (lim)))
#define CHECK(cond, code, v0, v1) do { if (!(cond)) chk_fail(p.dbg, (code), (v0), (v1)); } while (0)
#else
#define CIDX(idx, lim, code) (idx)
#define CHECK(cond, code, v0, v1) do { } while (0)
#endif

// DPP (GFX9 row_shr / row_bcast) wave primitives; call in uniform control flow
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWMASK, 0xf, false);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    v += dpp<0x111>(0u, v);          // row_shr:1
    v += dpp<0x112>(0u, v);          // row_shr:2
    v += dpp<0x114>(0u, v);          // row_shr:4
    v += dpp<0x118>(0u, v);          // row_shr:8
    v += dpp<0x142, 0xa>(0u, v);     // row_bcast:15 -> rows 1, 3
    v += dpp<0x143, 0xc>(0u, v);     // row_bcast:31 -> rows 2, 3
    return v;
}

__device__ __forceinline__ uint32_t wave_or(uint32_t v)
{
    v |= dpp<0x111>(0u, v);
    v |= dpp<0x112>(0u, v);
    v |= dpp<0x114>(0u, v);
    v |= dpp<0x118>(0u, v);
    v |= dpp<0x142, 0xa>(0u, v);
    v |= dpp<0x143, 0xc>(0u, v);
    return rl(v, WAVE - 1);
}

// k-th (0-based) set bit of w (k < popcount(w))
__device__ __forceinline__ int select_bit(uint64_t w, uint32_t k)
{
    int base = 0;
    uint32_t lo = (uint32_t)w;
    uint32_t pl = (uint32_t)__popc(lo);
    uint32_t x = lo;
    if (k >= pl) { k -= pl; x = (uint32_t)(w >> 32); base = 32; }
    uint32_t p16 = (uint32_t)__popc(x & 0xffffu);
    if (k >= p16) { k -= p16; x >>= 16; base += 16; }
    uint32_t p8 = (uint32_t)__popc(x & 0xffu);
    if (k >= p8) { k -= p8; x >>= 8; base += 8; }
    for (uint32_t t = 0; t < k; t++) x &= x - 1;
    return base + (int)__builtin_ctz(x);
}

// ------------------------------------------------------------ diagnostics
#define GW_STAMP_STRIDE 64   // stamps[E][64] (tools/stamps.py)
#ifdef GW_STAMPS
#define STAMP(i)                                                                  \
    do {                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                        \
        uint64_t _t = __builtin_amdgcn_s_memtime();                               \
        if (lane_id() == 0 && p.stamps) p.stamps[(size_t)e * GW_STAMP_STRIDE + (i)] = _t;      \
        __builtin_amdgcn_sched_barrier(0);                                        \
    } while (0)
// launch-level placement of the wave: [60] s_memrealtime at the start, [61]
// at the end (100 MHz, one clock for the whole device), [62] HW_ID (CU, SIMD,
// SE), [63] XCC_ID (tools/tail_probe.py)
#define STAMP_WAVE(slot, with_ids)                                                \
    do {                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                        \
        uint64_t _t = __builtin_amdgcn_s_memrealtime();                           \
        if (lane_id() == 0 && p.stamps) {                                         \
            p.stamps[(size_t)e * GW_STAMP_STRIDE + (slot)] = _t;                  \
            if (with_ids) {                                                       \
                p.stamps[(size_t)e * GW_STAMP_STRIDE + 62] =                      \
                    (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);          \
                p.stamps[(size_t)e * GW_STAMP_STRIDE + 63] =                      \
                    (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);         \
            }                                                                     \
        }                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                        \
    } while (0)
// sub-phase ticks summed in registers over the calls of one step (the
// serial attackers' phases of attack_one: att_acc[k], written once to
// stamps slots 42-48 after the attack loop, tools/stamps.py)
#define ACC_STAMP(k, t0)                                                          \
    do {                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                        \
        const uint64_t _n = __builtin_amdgcn_s_memtime();                         \
        if (att_acc) att_acc[(k) - 42] += _n - (t0);                              \
        t0 = _n;                                                                  \
        __builtin_amdgcn_sched_barrier(0);                                        \
    } while (0)
#define ACC_STAMP_T0(t0) uint64_t t0 = __builtin_amdgcn_s_memtime()
#else
#define STAMP(i) do { } while (0)
#define STAMP_WAVE(slot, with_ids) do { } while (0)
#define ACC_STAMP(k, t0) do { } while (0)
#define ACC_STAMP_T0(t0) do { } while (0)
#endif

// ------------------------------------------------------------ MT19937
__device__ __forceinline__ uint32_t temper(uint32_t y)
{
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

// The MT19937 key always lives in LDS and is always addressed through an
// LDS-typed (address space 3) pointer, so every access to it is a ds_*
// instruction whatever the surrounding code does with the pointer.
//
// Why it matters (the round-4 fault, DESIGN §4 "MT19937 key addressing"):
// in the generic-window instantiations (S = 0: observe_big is an out-of-line
// call taking the Rng / Smem by reference, so they live in scratch) a plain
// `uint32_t*` key is a generic pointer.  LLVM then lowers the twist's
// key[i], key[i + 1] pair to ONE flat_load_dwordx2 at key + 4i: legal for
// FLAT (dword alignment suffices for global memory), but for odd i the
// address is 4 mod 8 inside the LDS aperture, and a 64-bit LDS access off
// its natural alignment is a memory violation (the same pair through an
// LDS-typed pointer is a ds_read2_b32, two dword accesses).
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// mt19937.c mt19937_gen, lane-parallel in chunks of 64 (every write's
// dependency i-227 is >= 3 chunks back; i+1 is read before any lane writes)
__device__ __forceinline__ void mt_twist(lds_u32* key)
{
    const uint32_t UP = 0x80000000u, LO = 0x7fffffffu, MA = 0x9908b0dfu;
    const int l = lane_id();
    wave_sync();
    for (int b = 0; b < GW_MT_N - 1; b += WAVE) {
        const int i = b + l;
        uint32_t nv = 0;
        if (i < GW_MT_N - 1) {
            const uint32_t y = (key[i] & UP) | (key[i + 1] & LO);
            int j = i + 397; if (j >= GW_MT_N) j -= GW_MT_N;
            nv = key[j] ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
        }
        wave_sync();
        if (i < GW_MT_N - 1) key[i] = nv;
        wave_sync();
    }
    const uint32_t y = (key[GW_MT_N - 1] & UP) | (key[0] & LO);
    const uint32_t nv = key[396] ^ (y >> 1) ^ ((y & 1u) ? MA : 0u);
    wave_sync();
    if (l == 0) key[GW_MT_N - 1] = nv;
    wave_sync();
}

// The twist of a draw that crosses the key's end, as ONE out-of-line copy:
// Rng::next is inlined at every draw site, and a full twist loop at each of
// them made the kernels several times larger than the instruction cache.
__device__ __noinline__ void mt_twist_call(lds_u32* key) { mt_twist(key); }

// numpy legacy RandomState (mt19937.c).  The 624-word key stays in HBM until
// a draw needs it (a word outside the cached block, a twist, a reset); it is
// then copied to LDS.  The 64 tempered words from the stream position are
// kept per env in HBM (mt[MT_CACHE..]) and in a register, one word per lane,
// so a draw is one v_readlane and most launches never read the key.
struct Rng {
    lds_u32* key;           // LDS [624] (valid once loaded)
    const uint32_t* gkey;   // this env's key in HBM
    uint32_t cache;         // tempered key[base + lane] (lane < ccount)
    int pos;                // next index (wave-uniform)
    int base;               // cached block base (wave-uniform), -1 = none
    int ccount;             // valid words of the cached block
    bool loaded;            // key copied to LDS
    bool dirty;             // twisted since load

    __device__ __forceinline__ void ensure_key()
    {
        if (loaded) return;
        const int l = lane_id();
        constexpr int N4 = GW_MT_N / 4;                     // 156 uint4
        const uint4* src = (const uint4*)gkey;
        const bool ok2 = l + 2 * WAVE < N4;
        const uint4 a = src[l], b = src[l + WAVE], c = src[ok2 ? l + 2 * WAVE : l];
        uint4* k4 = (uint4*)key;
        k4[l] = a;
        k4[l + WAVE] = b;
        if (ok2) k4[l + 2 * WAVE] = c;
        wave_sync();
        loaded = true;
    }

    __device__ __forceinline__ void twist()
    {
        ensure_key();
        mt_twist_call(key);
        pos = 0;
        base = -1;
        dirty = true;
    }

    __device__ __forceinline__ uint32_t next()
    {
        if (pos == GW_MT_N) twist();
        if (!(base >= 0 && pos >= base && pos - base < ccount)) {
            ensure_key();
            const int b = pos & ~(WAVE - 1);
            const int i = b + lane_id();
            cache = temper(i < GW_MT_N ? key[i] : 0u);
            base = b;
            ccount = GW_MT_N - b < WAVE ? GW_MT_N - b : WAVE;
        }
        uint32_t v = rl(cache, pos - base);
        pos = pos + 1;
        return v;
    }

    // np.random.uniform(): 53-bit double from two words
    __device__ __forceinline__ double uniform()
    {
        uint32_t a = next() >> 5;
        uint32_t b = next() >> 6;
        return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
    }

    // n words consumed without looking at them (draws whose outcome is fixed:
    // uniform() > accuracy never holds for accuracy >= 1)
    __device__ __forceinline__ void skip(int n)
    {
        while (n > 0) {
            if (pos == GW_MT_N) twist();
            const int s = n < GW_MT_N - pos ? n : GW_MT_N - pos;
            pos += s;
            n -= s;
        }
    }

    // masked rejection draw on [0, max]; zero draws when max == 0
    __device__ __forceinline__ uint32_t interval(uint32_t max)
    {
        if (max == 0) return 0;
        uint32_t m = max;
        m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
        uint32_t v;
        do { v = next() & m; } while (v > max);
        return v;
    }
};

// ------------------------------------------------------------ per-env context
struct Lane {
    // constants
    int enc; uint32_t kind; int view, mrange, arange, simul;
    double strength, accuracy, init_health;
    uint32_t ov, amap;   // overlap / attack masks of this lane's encoding
    int init_r, init_c;
    // state
    int r, c; uint32_t seq; double health; bool in_grid, live, active;
    bool obs_m2;         // F_OBS_M2: the persistent obs row already holds -2
    double reward;
    int ammo;            // AmmoAgent.ammo
};

// AMMO: the lane's AmmoAgent.ammo too (the TeamBattle instantiation of the
// step kernel, whose configs hold no AmmoAgent, leaves it out)
template <bool AMMO = true>
__device__ __forceinline__ void load_lane(const Params& p, int e, Lane& L, bool valid)
{
    // unconditional loads (lanes past A read lane 0's row), then selects: a
    // branch around the loads would make its join wait for them
    const int l = lane_id();
    const int li = valid ? l : 0;
    const DevAgent s = p.spec[li];
    const size_t k = (size_t)e * p.A + li;
    const int2 q = p.pos[k];
    const uint32_t sq = p.seq[k];
    const double h = p.health[k];
    const uint8_t f = p.flags[k];
    const int32_t am = AMMO ? p.ammo[k] : 0;
    L.enc = valid ? s.enc : 0; L.kind = valid ? s.kind : 0u;
    L.view = valid ? s.view_range : 0; L.mrange = valid ? s.move_range : 0;
    L.arange = valid ? s.attack_range : 0; L.simul = valid ? s.simul : 0;
    L.strength = valid ? s.strength : 0.0; L.accuracy = valid ? s.accuracy : 0.0;
    L.init_health = valid ? s.init_health : 0.0;
    L.init_r = valid ? s.init_r : -1; L.init_c = valid ? s.init_c : -1;
    L.ov = valid ? s.ov : 0u;
    L.amap = valid ? s.amap : 0u;
    L.r = valid ? q.x : -1000; L.c = valid ? q.y : -1000;
    L.seq = valid ? sq : 0u;
    L.health = valid ? h : 0.0;
    L.in_grid = valid && (f & F_IN_GRID); L.live = valid && (f & F_LIVE); L.active = valid && (f & F_ACTIVE);
    L.obs_m2 = valid && (f & F_OBS_M2);
    L.reward = 0.0;
    L.ammo = valid ? am : 0;
}

template <bool AMMO = true>
__device__ __forceinline__ void store_lane(const Params& p, int e, const Lane& L, bool valid)
{
    if (!valid) return;
    CHECK(!L.in_grid || (L.r >= 0 && L.r < p.H && L.c >= 0 && L.c < p.W), 12, L.r, L.c);
    size_t k = (size_t)e * p.A + lane_id();
    p.pos[k] = make_int2(L.r, L.c);
    p.seq[k] = L.seq;
    p.health[k] = L.health;
    p.flags[k] = (uint8_t)((L.in_grid ? F_IN_GRID : 0) | (L.live ? F_LIVE : 0) | (L.active ? F_ACTIVE : 0) |
                           (L.obs_m2 ? F_OBS_M2 : 0));
    if (AMMO) p.ammo[k] = L.ammo;
}

// LDS carve-up per wave (dynamic shared memory, 16-B aligned pieces)
//   key  [624] u32          MT19937 state (loaded on demand)
//   tbl  [tbl_rows*pitch] u8 padded cell table: 0 empty, enc single,
//                           0x80 >= 2 occupants, 0xFF off-grid (border)
//   cnt  [ceil(HW/4)] u32   per-cell occupant counts, packed u8
//   work union: { tcnt, scnt [2][ceil(HW/4)] u32 (move isolation)
//               | stage [A*SS] i8 (observations) }
struct Smem {
    lds_u32* key;
    uint8_t* tbl;
    uint32_t* cnt;
    uint32_t* tcnt;
    uint32_t* scnt;
    int8_t* stage;
};

// Jacobi placement scratch in the work area (do_reset): stream words,
// per-lane (fresh, enc), chunk prefix counts, lane bits by cell rank, their
// prefix ORs, and a twisted copy of the key
// (sized so that the TeamBattle 32x32 env fits 10 KiB of LDS: 16 one-wave
// envs per CU, all 4096 resident at once on 256 CUs)
constexpr int JAC_WB = 160;
// the Jacobi sweeps end without a confirming sweep when at most this many
// estimates moved in the last one and none of them can change a fixpoint
constexpr int GW_JAC_CONFIRM = 16;
static_assert(JAC_WB < GW_MT_N - 397, "placement words past the twist come from the untwisted key");
constexpr int JAC_OFF_W = 0;
constexpr int JAC_OFF_PUB = JAC_OFF_W + 4 * JAC_WB;
constexpr int JAC_OFF_CP = JAC_OFF_PUB + 4 * 64;
constexpr int JAC_OFF_SB = JAC_OFF_CP + 4 * 64;
constexpr int JAC_OFF_T = JAC_OFF_SB + 8 * 64;
constexpr int JAC_OFF_KEY2 = JAC_OFF_T + 8 * 64;
constexpr size_t JAC_WORK_BYTES = JAC_OFF_KEY2 + 4 * GW_MT_N;

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

__host__ __device__ inline size_t work_bytes(int HW, int A, int S, int max_enc)
{
    size_t w = 2 * align16((size_t)((HW + 3) / 4) * 4);
    size_t s = align16((size_t)A * S * ((S + 3) & ~3));     // observation stage [A][S][SP]
    (void)max_enc;
    if (s < w) s = w;
    return s > JAC_WORK_BYTES ? s : JAC_WORK_BYTES;
}

__host__ __device__ inline size_t smem_bytes(int HW, int A, int S, int max_enc, int tbl_bytes)
{
    return align16(GW_MT_N * 4) + align16((size_t)tbl_bytes) +
           align16((size_t)((HW + 3) / 4) * 4) + work_bytes(HW, A, S, max_enc);
}

__device__ __forceinline__ Smem carve(char* base, const Params& p)
{
    const int HW = p.H * p.W;
    Smem s;
    s.key = (lds_u32*)base; base += align16(GW_MT_N * 4);
    s.tbl = (uint8_t*)base; base += align16((size_t)p.tbl_rows * p.pitch);
    s.cnt = (uint32_t*)base; base += align16((size_t)((HW + 3) / 4) * 4);
    s.tcnt = (uint32_t*)base;
    s.scnt = (uint32_t*)(base + align16((size_t)((HW + 3) / 4) * 4));
    s.stage = (int8_t*)base;
    return s;
}

__device__ __forceinline__ int tbl_idx(const Params& p, int r, int c)
{
    return CIDX((r + p.pad) * p.pitch + (c + p.pad), p.tbl_rows * p.pitch, 1);
}

// index of `cell`'s packed count word
__device__ __forceinline__ int cnt_word(const Params& p, int cell)
{
    return CIDX(cell, p.H * p.W, 3) >> 2;
}

#define cnt_get(cnt, cell) cnt_get_((cnt), (cell), p)
__device__ __forceinline__ uint32_t cnt_get_(const uint32_t* cnt, int cell, const Params& p)
{
    return (cnt[CIDX(cell, p.H * p.W, 4) >> 2] >> (8 * (cell & 3))) & 0xffu;
}

__device__ __forceinline__ uint8_t cell_byte(uint32_t count, int enc)
{
    return count == 0 ? 0 : (count == 1 ? (uint8_t)enc : (uint8_t)CELL_CROWD);
}

// Per-env state at launch start: the RNG position/counter/cached block and
// (copy_tmpl) the cell template + zero counts.  All global loads are issued
// before the first LDS write, so they share one round trip (a fence would
// stop later loads from being hoisted above it).
__device__ __forceinline__ void load_env(const Params& p, int e, Smem& sm, Rng& rng, uint32_t& ctr,
                                         bool copy_tmpl)
{
    const uint32_t* mt = p.mt + (size_t)e * GW_MT_STRIDE;
    const int l = lane_id();
    const int t16 = (p.tbl_rows * p.pitch + 15) / 16;
    const uint32_t cw = mt[MT_CACHE + l];
    const int pos = (int)uni(mt[MT_POS_SLOT]);
    const uint32_t c0 = uni(mt[MT_CTR_SLOT]);
    const uint32_t cb = uni(mt[MT_CBASE_SLOT]);
    // indices are clamped to valid addresses and the surplus is not stored
    // (a select between loads becomes a select between pointers -> FLAT)
    const bool t0ok = copy_tmpl && l < t16, t1ok = copy_tmpl && l + WAVE < t16;
    const uint4 t0 = p.tbl_tmpl[t0ok ? l : 0];
    const uint4 t1 = p.tbl_tmpl[t1ok ? l + WAVE : 0];
    if (copy_tmpl) {
        uint4* tb4 = (uint4*)sm.tbl;
        if (t0ok) tb4[l] = t0;
        if (t1ok) tb4[l + WAVE] = t1;
        for (int i = l + 2 * WAVE; i < t16; i += WAVE) tb4[i] = p.tbl_tmpl[i];
        const int nw = (p.H * p.W + 3) / 4;
        for (int i = l; i < nw; i += WAVE) sm.cnt[i] = 0u;
        wave_sync();
    }
    rng.key = sm.key;
    rng.gkey = mt;
    rng.pos = pos;
    rng.cache = cw;
    const bool cvalid = cb <= (uint32_t)GW_MT_N && (int)cb <= pos;
    rng.base = cvalid ? (int)cb : -1;
    rng.ccount = cvalid ? (GW_MT_N - (int)cb < WAVE ? GW_MT_N - (int)cb : WAVE) : 0;
    rng.loaded = false;
    rng.dirty = false;
    ctr = c0;
}

__device__ __forceinline__ void store_rng(const Params& p, int e, const Smem& sm, const Rng& rng, uint32_t ctr)
{
    uint32_t* dst = p.mt + (size_t)e * GW_MT_STRIDE;
    const int l = lane_id();
    if (rng.dirty) {
        wave_sync();
        for (int i = l; i < GW_MT_N / 4; i += WAVE) ((uint4*)dst)[i] = ((const uint4*)sm.key)[i];
    }
    if (rng.loaded) {
        // refresh the cached block at the new position (the key is in LDS)
        const int i = rng.pos + l;
        dst[MT_CACHE + l] = temper(i < GW_MT_N ? sm.key[i] : 0u);
        if (l == 0) dst[MT_CBASE_SLOT] = (uint32_t)rng.pos;
    }
    if (l == 0) { dst[MT_POS_SLOT] = (uint32_t)rng.pos; dst[MT_CTR_SLOT] = ctr; }
}

// Build the padded byte table and the counts from the lanes' positions.
// from_template: copy the per-config template (L2-resident) and zero the
// counts first; otherwise the caller already did (load_env) or cleared the
// lanes' old cells of a valid table and zeroed the counts (fused reset).
__device__ __forceinline__ void build_tables(const Params& p, Smem& sm, const Lane& L, bool from_template)
{
    const int l = lane_id();
    if (from_template) {
        const int t16 = (p.tbl_rows * p.pitch + 15) / 16;
        for (int i = l; i < t16; i += WAVE) ((uint4*)sm.tbl)[i] = p.tbl_tmpl[i];
        const int nw = (p.H * p.W + 3) / 4;
        for (int i = l; i < nw; i += WAVE) sm.cnt[i] = 0u;
        wave_sync();
    }
    int cell = L.r * p.W + L.c;
    if (L.in_grid) atomicAdd(&sm.cnt[cnt_word(p, cell)], 1u << (8 * (cell & 3)));
    wave_sync();
    if (L.in_grid) sm.tbl[tbl_idx(p, L.r, L.c)] = cell_byte(cnt_get(sm.cnt, cell), L.enc);
    wave_sync();
}

// cell table update after agent b (uniform) left cell (r, c): count-1, new byte
__device__ __forceinline__ void table_remove(const Params& p, Smem& sm, const Lane& L, int b, int r, int c)
{
    const int l = lane_id();
    const int cell = r * p.W + c;
    if (l == b) atomicSub(&sm.cnt[cnt_word(p, cell)], 1u << (8 * (cell & 3)));
    wave_sync();
    const uint32_t n = cnt_get(sm.cnt, cell);
    int enc = 0;
    if (n == 1) {
        const uint64_t m = __ballot(L.in_grid && L.r == r && L.c == c);
        CHECK(__popcll(m) == 1, 10, r * 1000 + c, (int)n);
        enc = rl(L.enc, first_lane(m));
    }
    if (l == 0) sm.tbl[tbl_idx(p, r, c)] = cell_byte(n, enc);
    wave_sync();
}

// ------------------------------------------------------------ observation
// Observation stage: A*SS compact bytes (the env's outputs in order), then
// the crowded-cell pair list; sized as int8 [A][S][SP], SP = 4*ceil(S/4)
// (a window row as whole table dwords).
__host__ __device__ constexpr int stage_pitch(int S) { return (S + 3) & ~3; }

// Lane l's window rows, row-padded [S][NW] dwords in registers, -> SS
// consecutive bytes at byte l*SS of the stage (the compact layout the store
// reads: output m of the env is stage byte m).  Byte i of the row stream is
// window row i / S, column i % S.  Lanes share the dwords at their span's
// ends, written byte by byte.
template <int S>
__device__ __forceinline__ void write_compact(Smem& sm, int l, const uint32_t* rw)
{
    constexpr int NW = (S + 3) / 4;
    constexpr int SS = S * S;
    constexpr int CW = (SS + 3) / 4;            // stream dwords
    uint32_t seg[CW];
#pragma unroll
    for (int g = 0; g < CW; g++) {
        // stream bytes 4g..4g+3 from at most two row dwords (one perm), or
        // assembled byte by byte when they span three
        int src[4], sb[4];
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int i = 4 * g + b < SS ? 4 * g + b : SS - 1;
            const int r = i / S, c = i % S;
            src[b] = r * NW + (c >> 2);
            sb[b] = c & 3;
        }
        const int s0 = src[0];
        int s1 = s0;
#pragma unroll
        for (int b = 1; b < 4; b++) if (src[b] != s0) s1 = src[b];
        bool two = true;
#pragma unroll
        for (int b = 0; b < 4; b++) two = two && (src[b] == s0 || src[b] == s1);
        if (two) {
            // v_perm_b32(hi, lo, sel): selector byte k picks byte k of lo
            // (0-3) or of hi (4-7)
            uint32_t sel = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) sel |= (uint32_t)((src[b] == s0 ? 0 : 4) + sb[b]) << (8 * b);
            seg[g] = __builtin_amdgcn_perm(rw[s1], rw[s0], sel);
        } else {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) v |= ((rw[src[b]] >> (8 * sb[b])) & 0xffu) << (8 * b);
            seg[g] = v;
        }
    }
    // memory dword k of this lane's span holds stream bytes [4k - s, 4k - s + 4)
    const int s = (l * SS) & 3;
    uint32_t* dst = (uint32_t*)sm.stage + ((l * SS) >> 2);
#pragma unroll
    for (int k = 0; k <= CW; k++) {
        const uint32_t lo_w = k == 0 ? 0u : seg[k - 1];
        const uint32_t hi_w = k < CW ? seg[k] : 0u;
        const uint32_t val = (uint32_t)((((uint64_t)hi_w << 32) | lo_w) >> (32 - 8 * s));
        if (k >= 1 && 4 * k + 4 <= SS) {            // full for every s
            dst[k] = val;
        } else {
            const int lo = k == 0 ? s : 0;
            const int hi = s + SS - 4 * k < 4 ? s + SS - 4 * k : 4;
            if (lo == 0 && hi == 4) {
                dst[k] = val;
            } else {
                uint8_t* d8 = (uint8_t*)(dst + k);
#pragma unroll
                for (int b = 0; b < 4; b++)
                    if (b >= lo && b < hi) d8[b] = (uint8_t)(val >> (8 * b));
            }
        }
    }
}

// PositionCenteredEncodingObserver.get_obs for every live lane; S = 2R+1.
template <int S, bool PLAIN = false>
__device__ __forceinline__ void observe_fixed(const Params& p, int e, Smem& sm, Rng& rng, Lane& L,
                                              int32_t* obs, int stamp_base = 8)
{
    // PLAIN (step_kernel<S, 1>): no blocking entities, one view range, every observer
    const bool HV = !PLAIN && p.hetero_view, BL = !PLAIN && p.blockers, LB = !PLAIN && p.lane_blockers;
    const int OO = PLAIN ? -1 : p.obs_only;
    (void)stamp_base;
    constexpr int SS = S * S;
    constexpr int R = S / 2;
    constexpr int NW = (S + 3) / 4;           // stage dwords per window row
    constexpr int ND = NW + 1;                // table dwords covering S bytes at any alignment
    constexpr int SSP = S * stage_pitch(S);
    const int l = lane_id();
    const int A = p.A;
    // (gw_component OBSERVE: the one lane OO, whatever its done state)
    const bool obs_me = (OO >= 0 ? l == OO : (l < A && L.live)) &&
                        (L.kind & GW_K_GRID_OBSERVER);
    // persistent obs buffer (gw_config.persistent_obs): rows that already
    // hold -2 and stay -2 (done entities, non-observers) are not rewritten
    // (gw_rollout with skip_done_obs: rows of lanes without an observation
    // this step are not written at all)
    const uint64_t skip = p.persistent_obs ? __ballot(l < A && L.obs_m2 && !obs_me)
                        : (p.skip_done_obs ? __ballot(l < A && !obs_me) : 0ull);
    if (l < A) L.obs_m2 = p.persistent_obs && !obs_me;
    // observers with different view ranges (HV): lane l's window
    // of range vw <= R sits in the top-left (2vw+1)^2 of its S x S slot, the
    // rest of the slot is -2 (the reference's per-agent (2v+1)^2 obs,
    // observer.py:162-174, in one tensor shape)
    const int vw = HV ? (obs_me ? L.view : 0) : R;

    // cells hidden by blocking entities (create_grid_and_mask, utils.py:46-115):
    // static blockers precomputed per cell, blocking lanes from the shadow LUT
    constexpr int MW = (SS + 31) / 32;
    uint32_t hid[MW];
#pragma unroll
    for (int w = 0; w < MW; w++) hid[w] = 0u;
    if (BL && HV) {
        // slot-geometry LUTs per range (bit wr * S + wc)
        if (obs_me && p.hsmask_off[vw] >= 0) {
            const uint32_t* src = p.hsmask + p.hsmask_off[vw] + (size_t)(L.r * p.W + L.c) * MW;
#pragma unroll
            for (int w = 0; w < MW; w++) hid[w] = src[w];
        }
        if (LB) {
            for (uint64_t bl = __ballot(l < A && L.active && (L.kind & GW_K_BLOCKING)); bl; bl &= bl - 1) {
                const int b = first_lane(bl);
                const int dr = rl(L.r, b) - L.r, dc = rl(L.c, b) - L.c;
                if (obs_me && dr >= -vw && dr <= vw && dc >= -vw && dc <= vw && (dr != 0 || dc != 0)) {
                    const uint32_t* src = p.hshadow + p.hshadow_off[vw] +
                                          ((dr + vw) * (2 * vw + 1) + (dc + vw)) * MW;
#pragma unroll
                    for (int w = 0; w < MW; w++) hid[w] |= src[w];
                }
            }
        }
    } else if (BL) {
        if (obs_me && p.smask_off[R] >= 0) {
            const uint32_t* src = p.smask + p.smask_off[R] + (size_t)(L.r * p.W + L.c) * MW;
#pragma unroll
            for (int w = 0; w < MW; w++) hid[w] = src[w];
        }
        if (LB) {
            for (uint64_t bl = __ballot(l < A && L.active && (L.kind & GW_K_BLOCKING)); bl; bl &= bl - 1) {
                const int b = first_lane(bl);
                const int dr = rl(L.r, b) - L.r, dc = rl(L.c, b) - L.c;
                if (obs_me && dr >= -R && dr <= R && dc >= -R && dc <= R && (dr != 0 || dc != 0)) {
                    const uint32_t* src = p.shadow + p.shadow_off[R] + ((dr + R) * S + (dc + R)) * MW;
#pragma unroll
                    for (int w = 0; w < MW; w++) hid[w] |= src[w];
                }
            }
        }
    }

    // window rows -> stage: every row's dwords first (independent LDS reads),
    // then decoded with alignbyte and written as dwords.  Table bytes are the
    // observation values (0 empty, enc, 0xFF = -1 off-grid); 0x80 marks a
    // crowded cell, resolved below; hidden cells become 0xFE = -2.
    uint32_t nev = 0;                         // crowded visible cells of this observer
    uint32_t rw[S * NW];                      // this lane's window rows, row-padded
    auto stage_rows = [&](auto masked, auto hetero) {
        constexpr bool MASKED = decltype(masked)::value;
        constexpr bool HETERO = decltype(hetero)::value;
        const uint32_t* t32 = (const uint32_t*)sm.tbl;
        uint32_t rows[S][ND];
        const int o0 = HETERO ? tbl_idx(p, L.r - vw, L.c - vw) : tbl_idx(p, L.r - R, L.c - R);
        const int D = 2 * vw + 1;                   // HETERO: this lane's window side
#pragma unroll
        for (int wr = 0; wr < S; wr++) {
            // HETERO: rows past the window re-read its last row (in the table), then masked
            const int o = o0 + (HETERO ? min(wr, D - 1) : wr) * p.pitch;
#pragma unroll
            for (int d = 0; d < ND; d++)
                rows[wr][d] = t32[CIDX((o >> 2) + d, (p.tbl_rows * p.pitch + 3) / 4, 2)];
        }
        const int sh = o0 & 3;
        const bool self_fix = !p.observe_self && L.in_grid;
#pragma unroll
        for (int wr = 0; wr < S; wr++) {
#pragma unroll
            for (int d = 0; d < NW; d++) {
                uint32_t w = __builtin_amdgcn_alignbyte(rows[wr][d + 1], rows[wr][d], sh);
                if constexpr (HETERO) {
                    if (wr == vw && d == (vw >> 2) && self_fix) {   // my cell at (vw, vw)
                        const int bs = 8 * (vw & 3);
                        if (((w >> bs) & 0xffu) != CELL_CROWD) w &= ~(0xffu << bs);
                    }
                    // slot cells outside the window: -2
                    const int nb = wr < D ? (D - 4 * d) : 0;
                    const uint32_t keep = nb >= 4 ? 0xffffffffu : (nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u));
                    w = (w & keep) | (0xFEFEFEFEu & ~keep);
                } else if (wr == R && d == R / 4 && self_fix) {  // alone on my cell, not observing myself
                    constexpr int bs = 8 * (R & 3);
                    if (((w >> bs) & 0xffu) != CELL_CROWD) w &= ~(0xffu << bs);
                }
                if constexpr (MASKED) {
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        const int kk = wr * S + d * 4 + b;
                        if (d * 4 + b < S && ((hid[kk >> 5] >> (kk & 31)) & 1u))
                            w = (w & ~(0xffu << (8 * b))) | (0xFEu << (8 * b));
                    }
                }
                // valid bytes of this dword (the last one of a row is padded)
                const uint32_t vm = (S - 4 * d >= 4) ? 0x80808080u
                                        : (0x80808080u & ((1u << (8 * (S - 4 * d))) - 1u));
                nev += (uint32_t)__popc(w & vm & ~(w << 1));
                rw[wr * NW + d] = w;
            }
        }
    };
    if (l < A) {
        if (obs_me) {
            using T = std::integral_constant<bool, true>;
            using F = std::integral_constant<bool, false>;
            if (HV) {
                if (BL) stage_rows(T(), T());
                else stage_rows(F(), T());
            } else if (BL) {
                stage_rows(T(), F());
            } else {
                stage_rows(F(), F());
            }
        } else {
            // -2 rows; a row the store skips holds the 0x80 sentinel instead
            const uint32_t fill = ((skip >> l) & 1ull) ? 0x80808080u : 0xFEFEFEFEu;
#pragma unroll
            for (int k = 0; k < S * NW; k++) rw[k] = fill;
        }
        write_compact<S>(sm, l, rw);
    }
    wave_sync();
    STAMP(stamp_base);

    // crowded cells draw np.random.choice in (agent, row, col) order
    // (observer.py:224-246): one bounded draw over the cell's encodings in
    // insertion (seq) order, without the observer when observe_self=False.
    const uint64_t ev_lanes = __ballot(nev != 0);
    uint32_t ev_scan = 0;
    int P = 0;
    if (ev_lanes && (ev_lanes & (ev_lanes - 1))) {          // two or more observers
        ev_scan = wave_incl_scan(nev);
        P = (int)rl(ev_scan, WAVE - 1);
    }
    if (P >= 6 && P <= p.pair_cap) {
        rng.ensure_key();
        // Parallel form: every (observer, cell) pair knows its member count
        // up front, so the stream offset of its draw is the exclusive scan
        // of the words the earlier pairs use (iterated to consistency, as in
        // the reset placement); the value is the j-th member by seq.
        uint16_t* pairs = (uint16_t*)(sm.stage + A * SSP);
        if (nev) {
            // this lane's compact span: dword k holds stream bytes 4k - s ..
            int q = (int)(ev_scan - nev);
            constexpr int CW = (SS + 3) / 4;
            const int s = (l * SS) & 3;
            const uint32_t* st32 = (const uint32_t*)sm.stage + ((l * SS) >> 2);
#pragma unroll
            for (int k = 0; k <= CW; k++) {
                const uint32_t w = st32[k];
                // bytes b with 0 <= 4k + b - s < SS
                const int lo = s - 4 * k, hi = SS + s - 4 * k;
                uint32_t vm = 0x80808080u;
                if (lo > 0) vm &= 0xffffffffu << (8 * lo);
                if (hi < 4) vm &= hi <= 0 ? 0u : ((1u << (8 * hi)) - 1u);
                for (uint32_t m = w & vm & ~(w << 1); m; m &= m - 1) {
                    const int i = 4 * k + (int)(__builtin_ctz(m) >> 3) - s;
                    pairs[CIDX(q++, p.pair_cap, 20)] = (uint16_t)((l << 8) | i);
                }
            }
        }
        // rank of every lane inside its cell by seq (lanes in crowded cells only)
        const int my_cell = L.r * p.W + L.c;
        const bool in_crowd = l < A && L.in_grid && cnt_get(sm.cnt, my_cell) >= 2;
        const uint64_t crowd_lanes = __ballot(in_crowd);
        int my_rank = 0;
        for (uint64_t it = crowd_lanes; it; it &= it - 1) {
            const int m = first_lane(it);
            const int cm = rl(my_cell, m);
            const uint32_t sq = rl(L.seq, m);
            my_rank += (in_crowd && cm == my_cell && sq < L.seq) ? 1 : 0;
        }
        wave_sync();
        bool abort = false;
        for (int c0 = 0; c0 < P && !abort; c0 += WAVE) {
            const int q = c0 + l;
            const bool act = q < P;
            const int pv = act ? (int)pairs[q] : 0;
            const int o = pv >> 8, pi = pv & 255, pwr = pi / S, pwc = pi - pwr * S;
            const int orr = __shfl(L.r, o), occ = __shfl(L.c, o);
            const uint32_t oseq = __shfl(L.seq, o);
            const bool o_in = __shfl((int)L.in_grid, o) != 0;
            const int ov = HV ? __shfl(vw, o) : R;     // the observer's window origin
            const int gr = orr - ov + pwr, gc = occ - ov + pwc;
            const int gcell = gr * p.W + gc;
            const bool self_in = !p.observe_self && o_in && orr == gr && occ == gc;
            uint32_t n = act ? cnt_get(sm.cnt, gcell) : 1u;
            if (self_in) n -= 1;
            const uint32_t mx = n - 1u;
            uint32_t mk = mx;
            mk |= mk >> 1; mk |= mk >> 2; mk |= mk >> 4;
            int used = (act && mx > 0) ? 1 : 0;
            uint32_t j = 0;
            bool past = false;
            for (int it = 0; it <= WAVE; it++) {
                const int st0 = (int)(wave_incl_scan((uint32_t)used) - (uint32_t)used);
                int nu = 0;
                j = 0;
                past = false;
                if (act && mx > 0) {
                    int k = rng.pos + st0;
                    for (;;) {
                        if (k >= GW_MT_N) { past = true; break; }   // a twist inside: serial
                        const uint32_t w = temper(rng.key[k]) & mk;
                        k++;
                        if (w <= mx) { j = w; break; }
                    }
                    nu = k - (rng.pos + st0);
                }
                const bool ch = __ballot(nu != used) != 0;
                used = nu;
                if (!ch) break;
            }
            if (__ballot(past)) { abort = true; break; }
            // the j-th member of the cell in seq order (minus the observer)
            int val = 0;
            for (uint64_t it = crowd_lanes; it; it &= it - 1) {
                const int m = first_lane(it);
                const int cm = rl(my_cell, m);
                const int rk = rl(my_rank, m);
                const uint32_t sq = rl(L.seq, m);
                const int enc = rl(L.enc, m);
                if (act && cm == gcell && !(self_in && m == o)) {
                    const int r2 = rk - ((self_in && oseq < sq) ? 1 : 0);
                    if (r2 == (int)j) val = enc;
                }
            }
            if (act) sm.stage[o * SS + pi] = (int8_t)val;
            rng.pos += (int)rl(wave_incl_scan((uint32_t)used), WAVE - 1);
            rng.base = -1;
        }
        wave_sync();
        if (!abort) nev = 0;
    }
    // serial form (few pairs, or a twist inside the batch): whatever is
    // still crowded in the stage, in the same order
    uint64_t olanes = __ballot(nev != 0);
    while (olanes) {
        const int o = first_lane(olanes);
        olanes &= olanes - 1;
        const int orr = rl(L.r, o), oc = rl(L.c, o);
        const int ov = HV ? rl(vw, o) : R;
        for (int k0 = 0; k0 < SS; k0 += WAVE) {
            const int k = k0 + l;
            const bool crowd = k < SS && (uint8_t)sm.stage[o * SS + k] == CELL_CROWD;
            uint64_t bits = __ballot(crowd);
            while (bits) {
                const int kk = k0 + (int)__builtin_ctzll(bits);
                bits &= bits - 1;
                const int gr = orr - ov + kk / S, gc = oc - ov + kk % S;
                const bool mem = l < A && L.in_grid && L.r == gr && L.c == gc && (p.observe_self || l != o);
                const uint64_t mm = __ballot(mem);
                const int n = __popcll(mm);
                CHECK(n >= 1, 11, gr * 1000 + gc, o);
                const uint32_t j = rng.interval((uint32_t)(n - 1));
                // the j-th member in insertion (seq) order
                int sel = first_lane(mm);
                for (uint64_t it = mm; it; it &= it - 1) {
                    const int m = first_lane(it);
                    const uint32_t sq = rl(L.seq, m);
                    const uint32_t rank = (uint32_t)__popcll(__ballot(mem && L.seq < sq));
                    if (rank == j) { sel = m; break; }
                }
                const int val = rl(L.enc, sel);
                if (l == 0) sm.stage[o * SS + kk] = (int8_t)val;
            }
        }
    }
    wave_sync();
    STAMP(stamp_base + 1);

    // stage (int8, compact: output m is stage byte m) -> obs (int32):
    // lane-contiguous int4 stores of 4 consecutive outputs from one aligned
    // stage dword each.  Rows the store skips hold the 0x80 sentinel: a
    // dword of four sentinels is not stored, a mixed one stores -2 for them
    // (max(v, -2): valid bytes are >= -2).
    const int total = A * SS;
    int32_t* out = obs + (size_t)e * total;
    const uint32_t* cs = (const uint32_t*)sm.stage;
    if ((total & 3) == 0) {
        // raw buffer stores on the env's obs row: the range check drops the
        // tail past A*SS (no per-store bound test) and a skipped dword is sent
        // out of range instead of branched around; offsets are immediates
        constexpr int NIT = (GW_MAX_AGENTS * SS + 4 * WAVE - 1) / (4 * WAVE);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, total * 4, BUF_RSRC_W3);
        const uint32_t base = (uint32_t)l * 16u;
        auto put = [&](int k, uint32_t w) {
            uint32_t voff = (skip && w == 0x80808080u) ? 0x80000000u : base;
            asm volatile("" : "+v"(voff));      // keeps k * 1024 an immediate offset
            buf_store_i8x4(rs, voff, k * 4 * WAVE * 4, w);
        };
        if (total > (NIT - 1) * 4 * WAVE) {
            // every iteration has live bytes: batches of LDS reads in flight
            constexpr int B = NIT < 7 ? NIT : 7;
#pragma unroll
            for (int k0 = 0; k0 < NIT; k0 += B) {
                uint32_t w[B];
#pragma unroll
                for (int k = 0; k < B; k++) if (k0 + k < NIT) w[k] = cs[(k0 + k) * WAVE + l];
#pragma unroll
                for (int k = 0; k < B; k++) if (k0 + k < NIT) put(k0 + k, w[k]);
            }
        } else {
            for (int k = 0; k * 4 * WAVE < total; k++) put(k, cs[k * WAVE + l]);
        }
    } else {
        for (int m = l; m < total; m += WAVE) {
            const int v = sm.stage[m];
            if (!((skip >> (m / SS)) & 1ull)) out[m] = v < -2 ? -2 : v;
        }
    }
}

// PositionCenteredEncodingObserver.get_obs (observer.py:204-250) for windows
// wider than the compiled parts (S = p.obs_side > 2 * GW_FIXED_RANGE + 1, a
// view range up to the grid's size and beyond): one observer at a time, in
// lane (= agents dict) order, the wave covering its S x S slot 64 cells at a
// time in row-major order, each cell's value computed straight from the cell
// table and stored (no stage): -1 off the grid, -2 outside the observer's own
// range (hetero view: its window sits top-left in the slot) and behind
// blocking entities (create_grid_and_mask, utils.py:46-115, via
// shadow_hides for every blocking lane and static blocker in range), 0 for
// the observer's own cell when it is alone there and observe_self is off,
// and for a crowded cell np.random.choice over the occupants' encodings in
// insertion (seq) order without the observer when observe_self is off --
// the draws in (observer, row, col) order as in the reference's loops.
__device__ __forceinline__ void observe_big(const Params& p, int e, Smem& sm, Rng& rng, Lane& L, int32_t* obs)
{
    const int S = p.obs_side, R = S / 2, SS = S * S;
    const int l = lane_id(), A = p.A;
    const int OO = p.obs_only;
    const bool obs_me = (OO >= 0 ? l == OO : (l < A && L.live)) && (L.kind & GW_K_GRID_OBSERVER);
    const uint64_t skip = p.persistent_obs ? __ballot(l < A && L.obs_m2 && !obs_me)
                        : (p.skip_done_obs ? __ballot(l < A && !obs_me) : 0ull);
    if (l < A) L.obs_m2 = p.persistent_obs && !obs_me;
    const uint64_t observers = __ballot(obs_me);
    const uint64_t blk = p.lane_blockers ? __ballot(l < A && L.active && (L.kind & GW_K_BLOCKING)) : 0ull;
    for (int o = 0; o < A; o++) {
        int32_t* out = obs + ((size_t)e * A + o) * SS;
        if (!((observers >> o) & 1ull)) {
            if (!((skip >> o) & 1ull))
                for (int k = l; k < SS; k += WAVE) __builtin_nontemporal_store(-2, out + k);
            continue;
        }
        const int orr = rl(L.r, o), oc = rl(L.c, o);
        const bool o_in = rlb(L.in_grid, o);
        const int vw = p.hetero_view ? rl(L.view, o) : R;
        const int D = 2 * vw + 1;
        const int ocell = orr * p.W + oc;
        for (int k0 = 0; k0 < SS; k0 += WAVE) {
            const int k = k0 + l;
            const int wr = k / S, wc = k - wr * S;
            const bool inwin = k < SS && wr < D && wc < D;
            const int dr = wr - vw, dc = wc - vw;             // the cell's offset from the observer
            const int gr = orr + dr, gc = oc + dc;
            // create_grid_and_mask: a hidden cell is -2 on or off the grid.
            // (the blockers' readlanes run under the full wave: a readlane
            // inside the divergent branch could read a lane the branch left
            // inactive)
            bool hid = false;
            for (uint64_t it = blk; it; it &= it - 1) {
                const int b = first_lane(it);
                const int br = rl(L.r, b) - orr, bc = rl(L.c, b) - oc;
                if (br >= -vw && br <= vw && bc >= -vw && bc <= vw && (br != 0 || bc != 0))
                    hid = hid || (inwin && shadow_hides(br, bc, dr, dc));
            }
            for (int q = 0; q < p.n_sblk; q++) {
                const int32_t sc = p.sblk[q];
                const int br = (sc >> 16) - orr, bc = (sc & 0xffff) - oc;
                if (br >= -vw && br <= vw && bc >= -vw && bc <= vw && (br != 0 || bc != 0))
                    hid = hid || (inwin && shadow_hides(br, bc, dr, dc));
            }
            int val = -2;
            bool crowd = false;
            if (inwin && !hid) {
                if (gr < 0 || gr >= p.H || gc < 0 || gc >= p.W) {
                    val = -1;
                } else {
                    const uint32_t b = sm.tbl[tbl_idx(p, gr, gc)];
                    if (b == CELL_CROWD) crowd = true;
                    else if (!p.observe_self && o_in && gr * p.W + gc == ocell) val = 0;
                    else val = (int)(int8_t)b;
                }
            }
            for (uint64_t it = __ballot(crowd); it; it &= it - 1) {
                const int kl = first_lane(it);
                const int cr = rl(gr, kl), cc = rl(gc, kl);
                const bool mem = l < A && L.in_grid && L.r == cr && L.c == cc && (p.observe_self || l != o);
                const uint64_t mm = __ballot(mem);
                const int n = __popcll(mm);
                CHECK(n >= 1, 11, cr * 1000 + cc, o);
                const uint32_t j = rng.interval((uint32_t)(n - 1));
                // the j-th member in insertion (seq) order
                int sel = first_lane(mm);
                for (uint64_t jt = mm; jt; jt &= jt - 1) {
                    const int m = first_lane(jt);
                    const uint32_t sq = rl(L.seq, m);
                    const uint32_t rank = (uint32_t)__popcll(__ballot(mem && L.seq < sq));
                    if (rank == j) { sel = m; break; }
                }
                const int v = rl(L.enc, sel);
                if (l == kl) val = v;
            }
            if (k < SS) __builtin_nontemporal_store(val, out + k);
        }
    }
}

template <int S, bool PLAIN = false>
__device__ __forceinline__ void observe_all(const Params& p, int e, Smem& sm, Rng& rng, Lane& L,
                                            int32_t* obs, int stamp_base = 8)
{
    if constexpr (S == 0) observe_big(p, e, sm, rng, L, obs);
    else observe_fixed<S, PLAIN>(p, e, sm, rng, L, obs, stamp_base);
}

// ------------------------------------------------------------ attack
// Window scan of this lane's attack: could any agent be a candidate?
// (superset test on the cell table; crowded cells count as possible)
__device__ __forceinline__ bool attack_precheck(const Params& p, const Smem& sm, const Lane& L)
{
    const int R = L.arange;
    bool any = false;
    if (R == 1) {
        // three window rows, one aligned dword each (independent LDS reads)
        const uint32_t* t32 = (const uint32_t*)sm.tbl;
        const int o0 = tbl_idx(p, L.r - 1, L.c - 1);
        uint32_t w[3];
#pragma unroll
        for (int wr = 0; wr < 3; wr++) {
            const int o = o0 + wr * p.pitch;
            w[wr] = __builtin_amdgcn_alignbyte(t32[(o >> 2) + 1], t32[o >> 2], o & 3);
        }
#pragma unroll
        for (int wr = 0; wr < 3; wr++) {
#pragma unroll
            for (int b = 0; b < 3; b++) {
                const uint32_t v = (w[wr] >> (8 * b)) & 0xffu;
                if (v == CELL_OFF || v == 0) continue;
                if (wr == 1 && b == 1 && v != CELL_CROWD) continue;    // just me
                if (v == CELL_CROWD || ((L.amap >> (v & 31u)) & 1u)) any = true;
            }
        }
        return any;
    }
    for (int dr = -R; dr <= R; dr++) {
        for (int dc = -R; dc <= R; dc++) {
            const uint32_t b = sm.tbl[tbl_idx(p, L.r + dr, L.c + dc)];
            if (b == CELL_OFF || b == 0) continue;
            if (dr == 0 && dc == 0 && b != CELL_CROWD) continue;   // just me
            if (b == CELL_CROWD || ((L.amap >> b) & 1u)) any = true;
        }
    }
    return any;
}

// AttackActorBaseComponent.process_action's ammo filter (actor.py:343-351)
// for AmmoAgent attacker a (uniform): more attacked entries than ammo keeps
// np.random.choice(attacked, ammo, replace=False) = entries permutation(n)[:ammo]
// in that order (n - 1 interval draws, also for ammo 0); then ammo -= the
// kept count.  list: lane t holds entry t.  Returns whether it chose (its
// result is a list: .tolist(), actor.py:347-351).
__device__ __forceinline__ bool ammo_filter(Rng& rng, Lane& L, int a, int& nlist, int& list)
{
    const int l = lane_id();
    const int am = rl(L.ammo, a);
    const bool chose = nlist > am;
    if (chose) {
        int perm = l;
        for (int i = nlist - 1; i >= 1; i--) {
            const int j = (int)rng.interval((uint32_t)i);
            const int pi = rl(perm, i), pj = rl(perm, j);
            if (l == i) perm = pj;
            if (l == j) perm = pi;
        }
        const int kept = __shfl(list, l < am ? perm : 0);
        list = l < am ? kept : -1;
        nlist = am;
    }
    if (l == a) L.ammo = am - nlist;
    return chose;
}

// BinaryAttackActor.process_action for attacker a with k attacks.
// Returns status (attempted); list (register of lane t) = attacked lanes in
// list order; applies damage and updates the cell table for kills.
// *ndarray (optional): the attacked agents are the numpy array
// _subset_attackables' np.random.choice returns (actor.py:412-414) and no
// ammo filter turned them into a list (actor.py:347-351).
template <bool PLAIN = false>
__device__ __forceinline__ bool attack_one(const Params& p, Smem& sm, Rng& rng, Lane& L, int a,
                                           int k, int& nlist, int& list, bool* ndarray = nullptr,
                                           uint64_t* att_acc = nullptr)
{
    (void)att_acc;
    if (ndarray) *ndarray = false;
    ACC_STAMP_T0(t0);
    const bool BL = !PLAIN && p.blockers, LB = !PLAIN && p.lane_blockers;
    const int l = lane_id();
    nlist = 0;
    list = -1;
    const uint32_t akind = rl(L.kind, a);
    if (!(akind & GW_K_ATTACKING)) return false;
    if (k == 0) return false;
    const int ar = rl(L.r, a), ac = rl(L.c, a);
    const int R = rl(L.arange, a);
    const double acc = rld(L.accuracy, a);
    const uint32_t amap = rl(L.amap, a);
    const int D = 2 * R + 1;
    const int dr = L.r - ar, dc = L.c - ac;
    bool cand = l < p.A && L.in_grid && l != a && L.active && ((amap >> L.enc) & 1u) &&
                dr >= -R && dr <= R && dc >= -R && dc <= R;
    if (BL) {                                       // attack mask (actor.py:483-494)
        const int k = (dr + R) * D + (dc + R), mw = mask_words(R);
        bool hidden = false;
        if (cand && p.smask_off[R] >= 0)
            hidden = (p.smask[p.smask_off[R] + (size_t)(ar * p.W + ac) * mw + (k >> 5)] >> (k & 31)) & 1u;
        if (LB) {
            for (uint64_t bl = __ballot(l < p.A && L.active && (L.kind & GW_K_BLOCKING)); bl; bl &= bl - 1) {
                const int b = first_lane(bl);
                const int bdr = rl(L.r, b) - ar, bdc = rl(L.c, b) - ac;
                if (bdr < -R || bdr > R || bdc < -R || bdc > R || (bdr == 0 && bdc == 0)) continue;
                if (cand) {
                    const uint32_t* src = p.shadow + p.shadow_off[R] + ((bdr + R) * D + (bdc + R)) * mw;
                    hidden = hidden || ((src[k >> 5] >> (k & 31)) & 1u);
                }
            }
        }
        cand = cand && !hidden;
    }
    const uint32_t ckey = ((uint32_t)((dr + R) * D + (dc + R)) << 24) | L.seq;
    const uint64_t cm = __ballot(cand);
    // rank of every candidate in (window cell, insertion) order
    int crank = -1;
    for (uint64_t it = cm; it; it &= it - 1) {
        const int j = first_lane(it);
        const uint32_t kj = rl(ckey, j);
        const int rk = __popcll(__ballot(cand && ckey < kj));
        if (l == j) crank = rk;
    }
    const int ncand = __popcll(cm);
    ACC_STAMP(42, t0);                                     // window scan + candidate ranks
    int rank = -1;                                         // rank among accepted
    int n = 0;
    if (acc >= 1.0) {
        // uniform() is < 1: every candidate passes its accuracy draw
        rng.skip(2 * ncand);
        rank = crank;
        n = ncand;
    } else {
        for (int r = 0; r < ncand; r++) {
            const uint64_t jm = __ballot(crank == r);
            CHECK(__popcll(jm) == 1, 8, r, ncand);
            const int j = first_lane(jm);
            const double u = rng.uniform();                 // _basic_criteria draw
            if (u > acc) continue;
            if (l == j) rank = n;
            n++;
        }
    }
    ACC_STAMP(43, t0);                                     // accuracy draws
    if (n == 0) return true;                                // (True, [])
    // _subset_attackables: pick (lane t) = accepted rank of list[t]
    int pick = -1;
    if (!p.stacked && k > n) {
        pick = l < n ? l : -1;
        nlist = n;
    } else if (p.stacked) {
        for (int t = 0; t < k; t++) {
            int idx = (int)rng.interval((uint32_t)(n - 1));
            if (l == t) pick = idx;
        }
        nlist = k;
        if (ndarray) *ndarray = true;
    } else {
        int perm = l;                                       // permutation(n)[:k]
        for (int i = n - 1; i >= 1; i--) {
            int j = (int)rng.interval((uint32_t)i);
            int pi = rl(perm, i), pj = rl(perm, j);
            if (l == i) perm = pj;
            if (l == j) perm = pi;
        }
        pick = l < k ? perm : -1;
        nlist = k;
        if (ndarray) *ndarray = true;
    }
    ACC_STAMP(44, t0);                                     // subset draws
    for (int t = 0; t < nlist; t++) {
        const int pr = rl(pick, t);
        const uint64_t tm = __ballot(rank == pr);
        CHECK(__popcll(tm) == 1, 9, pr, n);
        const int lane_t = first_lane(tm);
        if (l == t) list = lane_t;
    }
    if (!PLAIN && (akind & GW_K_AMMO) && ammo_filter(rng, L, a, nlist, list) && ndarray) *ndarray = false;
    ACC_STAMP(45, t0);                                     // attacked list
    // apply damage in list order (actor.py:353-358)
    const double strength = rld(L.strength, a);
    for (int t = 0; t < nlist; t++) {
        const int b = rl(list, t);
        if (!rlb(L.active, b)) continue;                    // already dead: skipped
        if (l == b) {
            double h = L.health - strength;
            if (0.0 > h) h = 0.0;
            if (1.0 < h) h = 1.0;
            L.health = h;
            L.active = h > 0.0;
        }
        if (!rlb(L.active, b)) {                            // grid.remove
            const int br = rl(L.r, b), bc = rl(L.c, b);
            if (l == b) L.in_grid = false;
            table_remove(p, sm, L, b, br, bc);
        }
    }
    ACC_STAMP(46, t0);                                     // damage + cell table
    return true;
}

// SelectiveAttackActor._determine_attack (actor.py:689-728) for attacker a,
// then the damage of AttackActorBaseComponent.process_action (:343-361).
// `cells`: the attacker's row-major (2R+1)^2 attack counts (HBM, uniform).
// Cells are visited in (r, c) order; each attacked cell's candidates (by
// seq) draw for accuracy, then _subset_attackables picks that cell's share.
// Returns the attack status; lane t holds attacked-list entry t.
__device__ __forceinline__ bool attack_selective(const Params& p, Smem& sm, Rng& rng, Lane& L, int a,
                                                 const int32_t* cells, int& nlist, int& list)
{
    const int l = lane_id();
    nlist = 0;
    list = -1;
    const uint32_t akind = rl(L.kind, a);
    if (!(akind & GW_K_ATTACKING)) return false;
    const int R = rl(L.arange, a);
    const int D = 2 * R + 1;
    bool any = false;
    for (int q = 0; q < D * D; q++) any |= cells[q] != 0;
    if (!any) return false;                                 // (False, [])
    const int ar = rl(L.r, a), ac = rl(L.c, a);
    const double acc = rld(L.accuracy, a);
    const uint32_t amap = rl(L.amap, a);
    const int dr = L.r - ar, dc = L.c - ac;
    bool cand = l < p.A && L.in_grid && l != a && L.active && ((amap >> L.enc) & 1u) &&
                dr >= -R && dr <= R && dc >= -R && dc <= R;
    const int myq = (dr + R) * D + (dc + R);
    if (p.blockers) {                                       // attack mask (create_grid_and_mask)
        const int mw = mask_words(R);
        bool hidden = false;
        if (cand && p.smask_off[R] >= 0)
            hidden = (p.smask[p.smask_off[R] + (size_t)(ar * p.W + ac) * mw + (myq >> 5)] >> (myq & 31)) & 1u;
        if (p.lane_blockers) {
            for (uint64_t bl = __ballot(l < p.A && L.active && (L.kind & GW_K_BLOCKING)); bl; bl &= bl - 1) {
                const int b = first_lane(bl);
                const int bdr = rl(L.r, b) - ar, bdc = rl(L.c, b) - ac;
                if (bdr < -R || bdr > R || bdc < -R || bdc > R || (bdr == 0 && bdc == 0)) continue;
                if (cand) {
                    const uint32_t* src = p.shadow + p.shadow_off[R] + ((bdr + R) * D + (bdc + R)) * mw;
                    hidden = hidden || ((src[myq >> 5] >> (myq & 31)) & 1u);
                }
            }
        }
        cand = cand && !hidden;
    }
    const uint64_t cm = __ballot(cand);
    for (int q = 0; q < D * D && cm; q++) {
        const int k = cells[q];
        if (k == 0) continue;                               // no attack on this cell
        const bool here = cand && myq == q;
        uint64_t mm = __ballot(here);
        if (!mm) continue;
        // _basic_criteria in cell (seq) order: accuracy draws
        int arank = -1;                                     // rank among this cell's accepted
        int n = 0;
        if (acc >= 1.0) {                                   // every draw passes: ranks by seq
            const int nm = __popcll(mm);
            rng.skip(2 * nm);
            int rk = 0;
            for (uint64_t it = mm; it; it &= it - 1) {
                const uint32_t sqm = rl(L.seq, first_lane(it));
                rk += (here && sqm < L.seq) ? 1 : 0;
            }
            if (here) arank = rk;
            n = nm;
            mm = 0;
        }
        while (mm) {
            uint32_t best = 0xFFFFFFFFu;
            int j = -1;
            for (uint64_t it = mm; it; it &= it - 1) {      // lowest seq left
                const int m = first_lane(it);
                const uint32_t sq = rl(L.seq, m);
                if (sq < best) { best = sq; j = m; }
            }
            mm &= ~(1ull << j);
            const double u = rng.uniform();
            if (u > acc) continue;
            if (l == j) arank = n;
            n++;
        }
        if (n == 0) continue;
        // _subset_attackables (actor.py:394-414)
        int pick = -1, take;
        if (!p.stacked && k > n) {
            pick = l < n ? l : -1;
            take = n;
        } else if (p.stacked) {
            for (int t = 0; t < k; t++) {
                const int idx = (int)rng.interval((uint32_t)(n - 1));
                if (l == t) pick = idx;
            }
            take = k;
        } else {
            int perm = l;                                   // permutation(n)[:k]
            for (int i = n - 1; i >= 1; i--) {
                const int j = (int)rng.interval((uint32_t)i);
                const int pi = rl(perm, i), pj = rl(perm, j);
                if (l == i) perm = pj;
                if (l == j) perm = pi;
            }
            pick = l < k ? perm : -1;
            take = k;
        }
        if (nlist + take > WAVE) take = WAVE - nlist;      // counts beyond the action space
        for (int t = 0; t < take; t++) {
            const int pr = rl(pick, t);
            const uint64_t tm = __ballot(arank == pr && here);
            CHECK(__popcll(tm) == 1, 9, pr, n);
            if (l == nlist + t) list = first_lane(tm);
        }
        nlist += take;
    }
    if (akind & GW_K_AMMO) ammo_filter(rng, L, a, nlist, list);
    // apply damage in list order (actor.py:353-358)
    const double strength = rld(L.strength, a);
    for (int t = 0; t < nlist; t++) {
        const int b = rl(list, t);
        if (!rlb(L.active, b)) continue;                    // already dead: skipped
        if (l == b) {
            double h = L.health - strength;
            if (0.0 > h) h = 0.0;
            if (1.0 < h) h = 1.0;
            L.health = h;
            L.active = h > 0.0;
        }
        if (!rlb(L.active, b)) {                            // grid.remove
            const int br = rl(L.r, b), bc = rl(L.c, b);
            if (l == b) L.in_grid = false;
            table_remove(p, sm, L, b, br, bc);
        }
    }
    return true;
}

// MoveActor.process_action, serial form (Grid.query as a ballot)
__device__ __forceinline__ bool move_one(const Params& p, Lane& L, int a, int mr, int mc, uint32_t newseq)
{
    const int l = lane_id();
    const uint32_t akind = rl(L.kind, a);
    if (!(akind & GW_K_MOVING)) return false;               // returns None
    const int ar = rl(L.r, a), ac = rl(L.c, a);
    const int nr = ar + mr, nc = ac + mc;
    if (!(0 <= nr && nr < p.H && 0 <= nc && nc < p.W)) return false;
    if (nr == ar && nc == ac) return true;
    if (p.static_bits) {                                    // a static entity: overlaps nothing
        const int cell = nr * p.W + nc;
        if ((p.static_bits[cell >> 5] >> (cell & 31)) & 1u) return false;
    }
    const uint32_t aov = rl(L.ov, a);
    const bool blocks = l < p.A && L.in_grid && L.r == nr && L.c == nc && !((aov >> L.enc) & 1u);
    if (__ballot(blocks)) return false;                     // Grid.query
    if (l == a) { L.r = nr; L.c = nc; L.seq = newseq; }     // remove + place (appended)
    return true;
}

__device__ __forceinline__ void renorm_seq(const Params& p, Lane& L, uint32_t& ctr)
{
    // keep seq < 2^24 (attack keys use 24 bits): rank-compress, order preserved
    const int l = lane_id();
    uint32_t rank = 0;
    for (int i = 0; i < p.A; i++) {
        uint32_t si = rl(L.seq, i);
        bool gi = rlb(L.in_grid, i);
        if (gi && si < L.seq) rank++;
    }
    if (l < p.A && L.in_grid) L.seq = rank;
    ctr = (uint32_t)p.A;
}

// ------------------------------------------------------------ done components
// SmartGridWorldSimulation.get_done (smart.py:106-111): the AND of the done
// components, all([]) = True.  ActiveDone / OneTeamRemainingDone: not active
// (done.py:44-48); TargetAgentDone: on the target's position (np.array_equal,
// done.py:91-95; a removed agent keeps its last position); TargetDestroyedDone:
// the target is inactive (done.py:131-132).  Targets are read from the spec
// table on demand (only the target programs pay for them).
__device__ __forceinline__ void target_of(const Params& p, const Lane& L, int32_t& tl, int32_t& tpos,
                                          int32_t& dl)
{
    const int l = lane_id();
    const DevAgent* s = p.spec + (l < p.A ? l : 0);
    tl = l < p.A ? s->tgt_lane : -1;
    tpos = s->tgt_pos;
    dl = l < p.A ? s->dtgt_lane : -1;
}

// this lane's get_done (every lane at once)
__device__ __forceinline__ bool lane_done(const Params& p, const Lane& L)
{
    const uint32_t dk = p.done_kind;
    bool d = true;
    if (dk & (GW_DONE_ACTIVE | GW_DONE_ONE_TEAM)) d = d && !L.active;
    if (dk & (GW_DONE_TARGET_AGENT | GW_DONE_TARGET_DESTROYED)) {
        int32_t tl, tpos, dl;
        target_of(p, L, tl, tpos, dl);
        const int ti = tl >= 0 ? tl : lane_id(), di = dl >= 0 ? dl : lane_id();
        const int tr = __shfl(L.r, ti), tc = __shfl(L.c, ti);
        const bool da = __shfl((int)L.active, di) != 0;
        if (dk & GW_DONE_TARGET_AGENT) {
            const int rr = tl == -2 ? (tpos >> 16) : tr, cc = tl == -2 ? (tpos & 0xffff) : tc;
            d = d && tl != -1 && L.r == rr && L.c == cc;
        }
        if (dk & GW_DONE_TARGET_DESTROYED) d = d && dl >= 0 && !da;   // a static target never dies
    }
    return d;
}

// get_done of lane a (uniform), at this point of the step
__device__ __forceinline__ bool lane_done_uniform(const Params& p, const Lane& L, int a)
{
    const uint32_t dk = p.done_kind;
    bool d = true;
    if (dk & (GW_DONE_ACTIVE | GW_DONE_ONE_TEAM)) d = d && !rlb(L.active, a);
    if (dk & (GW_DONE_TARGET_AGENT | GW_DONE_TARGET_DESTROYED)) {
        const DevAgent* s = p.spec + a;
        const int tl = uni(s->tgt_lane), tpos = uni(s->tgt_pos), dl = uni(s->dtgt_lane);
        if (dk & GW_DONE_TARGET_AGENT) {
            const int ar = rl(L.r, a), ac = rl(L.c, a);
            const int tr = tl >= 0 ? rl(L.r, tl) : (tpos >> 16), tc = tl >= 0 ? rl(L.c, tl) : (tpos & 0xffff);
            d = d && tl != -1 && ar == tr && ac == tc;
        }
        if (dk & GW_DONE_TARGET_DESTROYED) d = d && dl >= 0 && !rlb(L.active, dl);
    }
    return d;
}

// the target components' get_all_done: every MAPPED entity done (done.py:97-99,134-137)
__device__ __forceinline__ bool targets_all_done(const Params& p, const Lane& L)
{
    const uint32_t dk = p.done_kind;
    int32_t tl, tpos, dl;
    target_of(p, L, tl, tpos, dl);
    const int ti = tl >= 0 ? tl : lane_id(), di = dl >= 0 ? dl : lane_id();
    const int tr = __shfl(L.r, ti), tc = __shfl(L.c, ti);
    const bool da = __shfl((int)L.active, di) != 0;
    bool bad = false;
    if (dk & GW_DONE_TARGET_AGENT) {
        const int rr = tl == -2 ? (tpos >> 16) : tr, cc = tl == -2 ? (tpos & 0xffff) : tc;
        bad = bad || (tl != -1 && !(L.r == rr && L.c == cc));
    }
    if (dk & GW_DONE_TARGET_DESTROYED) bad = bad || (dl == -2 || (dl >= 0 && da));
    return __ballot(lane_id() < p.A && bad) == 0;
}

// ------------------------------------------------------------ reset
// AllStepManager.reset (all_step_manager.py:37-49) -> SmartGWS.reset ->
// PositionState.reset (state.py:88-166) / HealthState.reset (:629-641) in the
// pinned order.  Returns false on the reference's placement exceptions.
// what: 1 PositionState only, 2 HealthState only (the component-level
// gw_component ops), 3 both in the pinned state order (SmartGWS.reset)
__device__ __forceinline__ bool do_reset(const Params& p, Smem& sm, Rng& rng, Lane& L, uint32_t& ctr, uint32_t& err,
                                         int what = 3)
{
    const int l = lane_id();
    const int A = p.A;
    const bool valid = l < A;
    // placement works in free-cell space: the cells no static entity holds
    // (every list lost them before the first draw); NF = p.n_free
    const int NF = p.n_free;
    auto to_cell = [&](int f) -> int { return p.free_cell ? (int)p.free_cell[CIDX(f, NF, 19)] : f; };
    auto to_free = [&](int cell) -> int { return p.cell_free ? (int)p.cell_free[CIDX(cell, p.H * p.W, 19)] : cell; };
    if (what == 3) {
        L.live = valid && (L.kind & GW_K_OBSERVING) && (L.kind & GW_K_ACTING);
        L.reward = 0.0;
    }
    if (what & 1) {                         // Grid.reset (state.py:97): every cell empty
        L.in_grid = false;
        ctr = 0;
    }
    rng.ensure_key();                       // placement / health read the key directly
    const bool has_health = __ballot(valid && (L.kind & GW_K_HEALTH)) != 0;

    auto health_reset = [&]() {
        // one uniform() per HealthAgent without initial_health, in agent order:
        // consecutive word pairs of the stream, drawn lane-parallel when no
        // twist falls inside the batch
        const bool hl = valid && (L.kind & GW_K_HEALTH);
        const bool randh = hl && !(L.init_health >= 0.0);
        const uint64_t rm = __ballot(randh);
        const int nrand = __popcll(rm);
#ifdef GW_STAMPS
        if (l == 0 && p.stamps) {
            p.stamps[(size_t)blockIdx.x * GW_STAMP_STRIDE + 40] = (uint64_t)rng.pos;
            p.stamps[(size_t)blockIdx.x * GW_STAMP_STRIDE + 41] = (uint64_t)nrand;
        }
#endif
        if (rng.pos + 2 * nrand <= 2 * GW_MT_N) {
            // the lane of random-health rank k takes stream words pos + 2k and
            // pos + 2k + 1; words past the key's end come from the twisted
            // key (numpy twists when the position reaches 624, mt19937.c)
            const int k = __popcll(rm & ((1ull << l) - 1));
            const int i0 = rng.pos + 2 * k;
            uint32_t w[2] = {0u, 0u};
#pragma unroll
            for (int q = 0; q < 2; q++)
                if (randh && i0 + q < GW_MT_N) w[q] = temper(rng.key[CIDX(i0 + q, GW_MT_N, 5)]);
            const int np = rng.pos + 2 * nrand;
            if (np > GW_MT_N) {
                mt_twist(rng.key);
#pragma unroll
                for (int q = 0; q < 2; q++)
                    if (randh && i0 + q >= GW_MT_N) w[q] = temper(rng.key[CIDX(i0 + q - GW_MT_N, GW_MT_N, 5)]);
                rng.pos = np - GW_MT_N;
                rng.dirty = true;
                rng.base = -1;
            } else {
                rng.pos = np;
            }
            if (hl) {
                double h = L.init_health;
                if (randh) h = ((double)(w[0] >> 5) * 67108864.0 + (double)(w[1] >> 6)) / 9007199254740992.0;
                if (0.0 > h) h = 0.0;
                if (1.0 < h) h = 1.0;
                L.health = h;
                L.active = h > 0.0;
            }
            return;
        }
        for (int a = 0; a < A; a++) {
            const uint32_t k = rl(L.kind, a);
            if (!(k & GW_K_HEALTH)) continue;
            const double ih = rld(L.init_health, a);
            double h = ih >= 0.0 ? ih : rng.uniform();
            if (0.0 > h) h = 0.0;
            if (1.0 < h) h = 1.0;
            if (l == a) { L.health = h; L.active = h > 0.0; }
        }
    };

    // PositionState (state.py:88-166) without availability bitmaps: list e
    // is "every cell except the distinct cells removed from it", and the
    // removed cells are the placed lanes' own cells.  Lane j carries its
    // cell and remeff_j = the lists its placement removed a NEW cell from
    // (a cell already removed is not counted twice, as list.remove raising
    // ValueError in the reference).  The idx-th listed cell is the least
    // fixpoint of c = idx + #{removed cells <= c}; list lengths are one
    // register, lane e holding |list e|.
#ifdef GW_STAMPS
    uint64_t acc_t[5] = {0, 0, 0, 0, 0};
#define ACC_T(k, t0) do { __builtin_amdgcn_sched_barrier(0); uint64_t _n = __builtin_amdgcn_s_memtime(); acc_t[k] += _n - (t0); t0 = _n; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define ACC_T(k, t0) do { } while (0)
#endif
    auto position_reset_lanes = [&]() -> bool {
        int cell_l = -1;                 // this lane's cell once placed
        uint32_t remeff = 0;             // lists this lane's placement shortened
        uint32_t lens = (l >= 1 && l <= p.max_enc) ? (uint32_t)NF : 0u;
        const uint32_t all_encs = ((2u << p.max_enc) - 1u) & ~1u;
        // randomize_placement_order: the shuffled agents dict's order
        const int32_t* order = p.place_order ? p.place_order + (size_t)blockIdx.x * A : nullptr;
        for (int pass = 0; pass < 2; pass++) {
            for (int k = 0; k < A; k++) {
                const int a = order ? (int)uni(order[k]) : k;
#ifdef GW_STAMPS
                uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
                const int ir = rl(L.init_r, a);
                const bool has_ip = ir >= 0;
                if ((pass == 0) != has_ip) continue;
                const int aenc = rl(L.enc, a);
                const uint32_t aov = rl(L.ov, a);
                int cell;
                ACC_T(0, t0);
                if (has_ip) {
                    const int ic = rl(L.init_c, a);
                    cell = to_free(ir * p.W + ic);
                    // Grid.place -> query (grid.py:81-129), asserted by the reference
                    const bool blocks = valid && L.in_grid && cell_l == cell && !((aov >> L.enc) & 1u);
                    if (__ballot(blocks)) { err |= GW_ERR_INIT_POSITION; return false; }
                } else {
                    const uint32_t n = rl(lens, aenc);
                    if (n == 0) { err |= GW_ERR_NO_CELL; return false; }
                    const uint32_t idx = rng.interval(uni(n - 1));   // np.random.choice(list, 1)
                    ACC_T(1, t0);
                    const bool inlist = L.in_grid && ((remeff >> aenc) & 1u);
                    int c = (int)idx;
                    for (;;) {
                        const int c2 = (int)idx + __popcll(__ballot(inlist && cell_l <= c));
                        if (c2 == c) break;
                        c = c2;
                    }
                    cell = uni(c);
                    CHECK(cell >= 0 && cell < NF, 7, cell, a);
                    // a cell taken from list aenc always passes Grid.query
                    ACC_T(2, t0);
                }
                // _update_available_positions (state.py:126-141)
                const uint32_t rem = p.no_overlap_at_reset ? all_encs : (all_encs & ~aov);
                uint32_t fresh = 0;
                for (uint32_t m = rem; m; m &= m - 1) {
                    const int f = __builtin_ctz(m);
                    if (!__ballot(L.in_grid && cell_l == cell && ((remeff >> f) & 1u))) fresh |= 1u << f;
                }
                if (l >= 1 && l <= p.max_enc && ((fresh >> l) & 1u)) lens -= 1;
                if (l == a) {
                    cell_l = cell; remeff = fresh; L.in_grid = true; L.seq = ctr;
                }
                ctr++;
                ACC_T(3, t0);
            }
        }
        if (L.in_grid) { const int gc = to_cell(cell_l); L.r = gc / p.W; L.c = gc % p.W; }
#ifdef GW_STAMPS
        if (l == 0 && p.stamps)
            for (int k = 0; k < 4; k++) p.stamps[(size_t)blockIdx.x * GW_STAMP_STRIDE + 16 + k] = acc_t[k];
#endif
        return true;
    };

    // The same placement solved for all lanes at once: every unknown of the
    // sequential loop above (|list|, the stream offset and index of the draw,
    // the cell, which lists the cell was freshly removed from) is re-derived
    // each sweep from the other lanes' current estimates, until a sweep
    // changes nothing.  Lane i only depends on lanes placed before it, so the
    // fixed point is the sequential result.  Per sweep the estimates are
    // ranked by cell (histogram in the count table + chunk prefix sums), and
    // T[r] = the lanes holding the r+1 lowest cells, so "removed cells <= c"
    // is popc(T[rank(c)-1] & removers-before-me): the least fixpoint of
    // c = idx + #{removed <= c} costs a few LDS reads (a fixpoint on a
    // removed cell is not the least: restart from idx).  Returns 0 placed,
    // 1 placement exception (err set), 2 unresolved (word buffer / sweep
    // cap / a full list): run the serial loop.
    auto position_reset_jacobi = [&]() -> int {
        constexpr int MAX_SWEEPS = 48;
#ifdef GW_STAMPS
        uint64_t acc_t[5] = {0, 0, 0, 0, 0};
        uint64_t t0 = __builtin_amdgcn_s_memtime();
        int nsw = 0;
#endif
        const uint32_t all_encs = ((2u << p.max_enc) - 1u) & ~1u;
        const bool ip = valid && L.init_r >= 0;
        const bool rnd = valid && !ip;
        const uint64_t ipm = __ballot(ip), rndm = __ballot(rnd);
        const int nrnd = __popcll(rndm);
        if (nrnd + 8 > JAC_WB) return 2;
        const uint64_t lt_l = (1ull << l) - 1ull;
        const uint64_t before = ip ? (ipm & lt_l) : (rnd ? (ipm | (rndm & lt_l)) : 0ull);
        const uint32_t rem = valid ? (p.no_overlap_at_reset ? all_encs : (all_encs & ~L.ov)) : 0u;
        uint32_t* wbuf = (uint32_t*)(sm.stage + JAC_OFF_W);
        uint32_t* pub = (uint32_t*)(sm.stage + JAC_OFF_PUB);   // fresh | enc << 16
        uint32_t* cpa = (uint32_t*)(sm.stage + JAC_OFF_CP);
        uint2* sb = (uint2*)(sm.stage + JAC_OFF_SB);
        uint2* tb = (uint2*)(sm.stage + JAC_OFF_T);
        uint32_t* hist = sm.cnt;   // rebuilt by build_tables afterwards
        const int nw = (NF + 3) >> 2;
        int chs = 4;               // chunk of 1 << chs cells per lane (>= 16)
        while ((WAVE << chs) < NF) chs++;
        const int cw4 = 1 << (chs - 4);   // uint4 per chunk (1, 2 or 4)
        const int nw4 = (nw + 3) >> 2;
        const uint4* h4 = (const uint4*)hist;
        // count bytes of chunk k: the sum below byte `off` and (at) the byte
        // at `off` (off == chunk size: the whole chunk).  One uint4 per
        // iteration; a 1024-cell grid has one-uint4 chunks (one LDS trip).
        auto chunk_sum = [&](int k, int off, uint32_t& at) -> uint32_t {
            uint32_t sum = 0;
            at = 0;
            for (int q = 0; q < cw4; q++) {
                const int i = k * cw4 + q;
                const bool ok = i < nw4;
                const uint4 v = h4[ok ? i : 0];
                const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const int b0 = (q * 4 + t) * 4;          // first chunk byte of this dword
                    const int nb = off - b0;                  // bytes of it below `off`
                    uint32_t m = nb >= 4 ? 0xffffffffu : (nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u));
                    const bool live = ok && i * 4 + t < nw;
                    if (!live) m = 0u;
                    sum = __builtin_amdgcn_sad_u8(d[t] & m, 0u, sum);
                    if (live && nb >= 0 && nb < 4) at = (d[t] >> (8 * nb)) & 0xffu;
                }
            }
            return sum;
        };
        // #cells <= c among this sweep's estimates (lt: < c)
        auto rank_le = [&](int c, uint32_t& lt) -> uint32_t {
            const int k = c >> chs;
            const uint32_t base = cpa[CIDX(k, WAVE, 14)];
            uint32_t at;
            lt = base + chunk_sum(k, c - (k << chs), at);
            return lt + at;
        };
        const int pos0 = rng.pos;
        const bool crosses = pos0 + JAC_WB > GW_MT_N;
        wave_sync();
        if (nrnd > 0) {
            // the next JAC_WB tempered words of the stream, across a twist
            // into a copy of the key (the live key changes only if used)
            for (int t = l; t < JAC_WB; t += WAVE) {
                const int k = pos0 + t;
                if (k < GW_MT_N) wbuf[t] = temper(rng.key[k]);
            }
            if (crosses) {
                // word j < 227 of the next key needs only the current one
                // (mt19937's twist rewrites key[j] from key[j], key[j + 1]
                // and key[j + 397], none rewritten yet for j < 227): the
                // words past the twist without twisting (JAC_WB < 227).
                // Indices clamped, every read in range for every lane.
                for (int t = l; t < JAC_WB; t += WAVE) {
                    const int j = pos0 + t - GW_MT_N;
                    const int jj = j < 0 ? 0 : j;
                    const uint32_t k0 = rng.key[CIDX(jj, GW_MT_N, 21)], k1 = rng.key[CIDX(jj + 1, GW_MT_N, 21)];
                    const uint32_t k397 = rng.key[CIDX(jj + 397, GW_MT_N, 21)];
                    const uint32_t y = (k0 & 0x80000000u) | (k1 & 0x7fffffffu);
                    if (j >= 0) wbuf[t] = temper(k397 ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
                }
            }
            wave_sync();
        }
        ACC_T(0, t0);
        // interval(n - 1) draws: stream offsets = exclusive scan of words
        // used; iterate until consistent (each pass fixes the first lane)
        auto draw_all = [&](uint32_t n, int& used, int& nidx, bool& bad_) {
            const bool draws = rnd && n > 1;
            const uint32_t mx = n - 1u;
            uint32_t mk = mx;
            mk |= mk >> 1; mk |= mk >> 2; mk |= mk >> 4; mk |= mk >> 8; mk |= mk >> 16;
            for (int it = 0; it <= WAVE; it++) {
                const int st = (int)(wave_incl_scan((uint32_t)used) - (uint32_t)used);
                int nu = 0;
                nidx = 0;
                bad_ = false;
                if (draws) {
                    int q = st;
                    for (;;) {
                        if (q >= JAC_WB) { bad_ = true; break; }
                        const uint32_t w = wbuf[CIDX(q, JAC_WB, 13)] & mk;
                        q++;
                        if (w <= mx) { nidx = (int)w; break; }
                    }
                    nu = q - st;
                }
                const bool ch = __ballot(nu != used) != 0;
                used = nu;
                if (!ch) break;
            }
        };
        // every cell placed leaves every list (no initial positions, no
        // overlap at reset, every encoding listed): one shared list, |list|
        // = NF - #placed before, and the cells are the decoded Lehmer code of
        // the draws -- backwards over the lanes, each later lane's rank moves
        // past the cell of the lane before it (the rank of c_j among the cells
        // c_j, ..., c_k is fixed once the lanes after j are decoded).  No
        // ranking tables, no sweeps: one readlane + compare per placed lane.
        const bool shared = !valid || (rnd && rem == all_encs && ((all_encs >> L.enc) & 1u));
        if (nrnd > 0 && __ballot(!shared) == 0) {
            const uint32_t n = (uint32_t)NF - (uint32_t)__popcll(rndm & lt_l);
            if (__ballot(rnd && n == 0)) return 2;   // the serial loop raises at the right point
            int used = rnd ? 1 : 0, nidx = 0;
            bool bad_ = false;
            draw_all(n, used, nidx, bad_);
            if (__ballot(bad_)) return 2;
            ACC_T(2, t0);
            int v = nidx;
            for (uint64_t m = rndm & ~(1ull << (63 - __builtin_clzll(rndm))); m;) {
                const int j = 63 - __builtin_clzll(m);
                m &= ~(1ull << j);
                const int vj = rl(v, j);
                if (rnd && l > j && v >= vj) v++;
            }
            ACC_T(3, t0);
            const int total = (int)rl(wave_incl_scan((uint32_t)used), WAVE - 1);
            const int np = pos0 + total;
            if (np > GW_MT_N) {
                mt_twist_call(rng.key);
                rng.pos = np - GW_MT_N;
                rng.dirty = true;
            } else {
                rng.pos = np;
            }
            rng.base = -1;
            CHECK(!valid || (v >= 0 && v < NF), 7, v, l);
            if (valid) {
                L.in_grid = true;
                const int gc = to_cell(v);
                L.r = gc / p.W; L.c = gc % p.W;
                L.seq = (uint32_t)__popcll(rndm & lt_l);
            }
            ctr = (uint32_t)nrnd;
            ACC_T(4, t0);
#ifdef GW_STAMPS
            if (l == 0 && p.stamps) {
                for (int k = 0; k < 5; k++) p.stamps[(size_t)blockIdx.x * GW_STAMP_STRIDE + 20 + k] = acc_t[k];
                p.stamps[(size_t)blockIdx.x * GW_STAMP_STRIDE + 25] = 0;
            }
#endif
            return 0;
        }
        auto lanes_upto = [&](uint32_t r) -> uint64_t {   // lanes of the r lowest cells
            if (r == 0) return 0ull;
            const uint2 t = tb[CIDX((int)r - 1, WAVE, 16)];
            return ((uint64_t)t.y << 32) | t.x;
        };
        int cell = ip ? to_free(L.init_r * p.W + L.init_c) : 0;
        uint32_t fresh = rem;
        int used = rnd ? 1 : 0;
        int idx = rnd ? -1 : 0;
        uint32_t n = 0;
        bool bad = false, qbad = false;
        // the list lengths and the draws depend on the other lanes' fresh
        // sets only: a sweep that changed no fresh set leaves them as they are
        // (after the first sweep only a shared cell changes one)
        uint64_t rm = 0;
        bool fresh_dirty = true;
        for (int sweep = 0;; sweep++) {
            if (sweep == MAX_SWEEPS) return 2;
            int nidx = idx;
            if (fresh_dirty) {
                // |list enc| when this lane is placed, and who shortened it
                uint64_t mym = 0;
                for (int f = 1; f <= p.max_enc; f++) {
                    const uint64_t m = __ballot((fresh >> f) & 1u);
                    if (L.enc == f) mym = m;
                }
                rm = mym & before;
                n = (uint32_t)NF - (uint32_t)__popcll(rm);
                ACC_T(1, t0);
                nidx = 0;
                draw_all(n, used, nidx, bad);
            }
            ACC_T(2, t0);
            // rank this sweep's cell estimates
            // a new draw starts from its expected cell, the idx-th of n listed
            // cells spread over NF (the fixpoint below is exact from any start)
            int ce0 = cell;
            // (placement 28.3 k -> 26.6 k ticks median, 47 k -> 34 k max, at most 5
            // sweeps instead of 7: profiles/r04/stamps_tb_expected_cell.txt)
            if (rnd && nidx != idx) {
                const int g = (int)((float)nidx * ((float)NF / (float)(n > 0 ? n : 1)));
                ce0 = g < nidx ? nidx : (g >= NF ? NF - 1 : g);
            }
            for (int i = l; i < nw; i += WAVE) hist[i] = 0u;
            if (valid) pub[l] = fresh | ((uint32_t)L.enc << 16);
            sb[l] = make_uint2(0u, 0u);
            wave_sync();
            uint32_t tie = 0;
            if (valid) {
                const int sh = 8 * (ce0 & 3);
                tie = (atomicAdd(&hist[CIDX(ce0 >> 2, nw, 17)], 1u << sh) >> sh) & 0xffu;
            }
            wave_sync();
            uint32_t dummy;
            const uint32_t csum = chunk_sum(l, 1 << chs, dummy);
            cpa[l] = wave_incl_scan(csum) - csum;
            wave_sync();
            if (valid) {
                uint32_t lt0;
                rank_le(ce0, lt0);
                sb[CIDX((int)(lt0 + tie), WAVE, 18)] = l < 32 ? make_uint2(1u << l, 0u) : make_uint2(0u, 1u << (l - 32));
            }
            wave_sync();
            {
                const uint2 sv = sb[l];
                tb[l] = make_uint2(wave_incl_scan(sv.x), wave_incl_scan(sv.y));
            }
            wave_sync();
            // least fixpoint of c = idx + #{removed cells <= c}
            int c = ce0;
            bool fin = !rnd, ovf = false;
            uint64_t eqm = 0;
            for (int it = 0;; it++) {
                uint32_t lt;
                const uint32_t le = rank_le(c, lt);
                const uint64_t mle = lanes_upto(le);
                eqm = mle & ~lanes_upto(lt);
                if (!fin) {
                    const int c2 = nidx + __popcll(mle & rm);
                    if (c2 >= NF) { ovf = true; fin = true; }
                    else if (c2 != c) c = c2;
                    else if (eqm & rm) c = nidx;   // on a removed cell: not the least
                    else fin = true;
                }
                if (__ballot(!fin) == 0) break;
                if (it == 2 * WAVE) { ovf = ovf || !fin; break; }
            }
            // earlier placements on the same cell: lists already shortened
            // by it, and Grid.query for initial positions
            uint64_t dm = valid ? (eqm & before) : 0ull;
            uint32_t dup = 0;
            bool qb = false;
            while (dm) {
                const int j = __builtin_ctzll(dm);
                dm &= dm - 1ull;
                const uint32_t pw = pub[j];
                const uint2 pj = make_uint2(pw & 0xffffu, pw >> 16);
                dup |= pj.x;
                qb |= !((L.ov >> pj.y) & 1u);
            }
            wave_sync();
            const uint32_t nf = rem & ~dup;
            const bool lane_ch = valid && (ovf || c != ce0 || nf != fresh || nidx != idx);
            const bool any = __ballot(lane_ch) != 0;
            fresh_dirty = __ballot(valid && nf != fresh) != 0;
            cell = c; fresh = nf; idx = nidx; qbad = qb;
            ACC_T(3, t0);
#ifdef GW_STAMPS
            nsw++;
#endif
            if (!any) break;
            // Would the next sweep change anything?  Each lane's fixpoint of this
            // sweep is exact against the estimates it ranked (c = idx + #{rm
            // estimates <= c}, none of them on c), and so is its duplicate set.
            // With no fresh set changed (same rm, n and draws) they stay exact
            // against the new estimates unless an estimate that moved crossed c
            // (an rm lane) or left or landed on c (any earlier lane): then the
            // confirming sweep is not needed.
            if (!fresh_dirty && __ballot(ovf) == 0) {
                const uint64_t mv = __ballot(valid && c != ce0);
                if (__popcll(mv) <= GW_JAC_CONFIRM) {
                    bool aff = false;
                    const uint32_t xy = (uint32_t)ce0 << 16 | (uint32_t)c;   // cells < 2^16
                    for (uint64_t m = mv; m; m &= m - 1ull) {
                        const int j = first_lane(m);
                        const uint32_t xyj = rl(xy, j);
                        const int x = (int)(xyj >> 16), y = (int)(xyj & 0xffffu);
                        if ((before >> j) & 1ull) {
                            aff = aff || x == c || y == c;
                            if (rnd && ((rm >> j) & 1ull)) aff = aff || ((x < c) != (y < c));
                        }
                    }
                    if (__ballot(valid && aff) == 0) break;
                }
            }
        }
        if (__ballot(bad)) return 2;
        if (__ballot(ip && qbad)) { err |= GW_ERR_INIT_POSITION; return 1; }   // grid.py:81-129
        if (__ballot(rnd && n == 0)) return 2;   // the serial loop raises at the right point
        const int total = (int)rl(wave_incl_scan((uint32_t)used), WAVE - 1);
        const int np = pos0 + total;
        if (np > GW_MT_N) {   // the draws crossed the twist: twist the live key
            mt_twist_call(rng.key);
            rng.pos = np - GW_MT_N;
            rng.dirty = true;
        } else {
            rng.pos = np;
        }
        rng.base = -1;
        CHECK(!valid || (cell >= 0 && cell < NF), 7, cell, l);
        if (valid) {
            L.in_grid = true;
            const int gc = to_cell(cell);
            L.r = gc / p.W; L.c = gc % p.W;
            L.seq = ip ? (uint32_t)__popcll(ipm & lt_l) : (uint32_t)(__popcll(ipm) + __popcll(rndm & lt_l));
        }
        ctr = (uint32_t)__popcll(ipm | rndm);
        ACC_T(4, t0);
#ifdef GW_STAMPS
        if (l == 0 && p.stamps) {
            for (int k = 0; k < 5; k++) p.stamps[(size_t)blockIdx.x * GW_STAMP_STRIDE + 20 + k] = acc_t[k];
            p.stamps[(size_t)blockIdx.x * GW_STAMP_STRIDE + 25] = nsw;
        }
#endif
        return 0;
    };

    auto place = [&]() -> bool {
        // the Jacobi form solves lane order only: a shuffled order runs serially
        if (p.place_order) return position_reset_lanes();
        const int r = position_reset_jacobi();
        if (r == 2) return position_reset_lanes();
        return r == 0;
    };
#ifdef GW_STAMPS
    const int e = blockIdx.x;
#endif
    bool ok = true;
    if (what == 1) {
        ok = place();
    } else if (what == 2) {
        if (has_health) health_reset();
    } else if (p.state_order == GW_ORDER_POSITION_HEALTH) {
        ok = place();
        STAMP(11);
        if (ok && has_health) health_reset();
        STAMP(15);
    } else {
        if (has_health) health_reset();
        STAMP(11);
        ok = place();
        STAMP(15);
    }
    if (what == 3 && valid && !(L.kind & GW_K_HEALTH)) L.active = true;   // PrincipleAgent.active
    // AmmoState.reset (state.py:644-656): no draw, any place in the state order
    if (what == 3 && valid && (L.kind & GW_K_AMMO)) L.ammo = p.spec[l].init_ammo;
    return ok;
}

template <int S, bool PLAIN = false>
__device__ __forceinline__ void reset_env(const Params& p, int e, Smem& sm, Rng& rng, Lane& L, uint32_t& ctr,
                                          bool fused, int32_t* obs)
{
    const int SS = S ? S * S : p.obs_side * p.obs_side;
    uint32_t err = 0;
    // fused: the LDS table holds the end-of-step grid; empty the lanes' cells
    // (static entities stay) instead of re-reading the template
    if (fused && L.in_grid) sm.tbl[tbl_idx(p, L.r, L.c)] = 0;
    const bool ok = do_reset(p, sm, rng, L, ctr, err);
    STAMP(13);
    if (ok) {
        if (fused) {
            const int nw = (p.H * p.W + 3) / 4;      // the placement used the counts as scratch
            wave_sync();
            for (int i = lane_id(); i < nw; i += WAVE) sm.cnt[i] = 0u;
            wave_sync();
        }
        build_tables(p, sm, L, !fused);
        observe_all<S, PLAIN>(p, e, sm, rng, L, obs, 26);
    } else {
        int32_t* out = obs + (size_t)e * p.A * SS;
        for (int i = lane_id(); i < p.A * SS; i += WAVE) out[i] = -2;
        if (lane_id() < p.A) L.obs_m2 = p.persistent_obs != 0;
    }
    if (lane_id() == 0 && p.err) p.err[e] |= err;
}

// the per-config template (static entities, off-grid border) in the LDS
// table without any lane, counts zeroed
__device__ __forceinline__ void table_template(const Params& p, Smem& sm)
{
    const int l = lane_id();
    wave_sync();
    const int t16 = (p.tbl_rows * p.pitch + 15) / 16;
    for (int i = l; i < t16; i += WAVE) ((uint4*)sm.tbl)[i] = p.tbl_tmpl[i];
    const int nw = (p.H * p.W + 3) / 4;
    for (int i = l; i < nw; i += WAVE) sm.cnt[i] = 0u;
    wave_sync();
}

// ------------------------------------------------------------ kernels
// AllStepManager.step for p.nsteps consecutive steps of one env (one wave):
// the single-step calls run one; gw_rollout runs a whole fragment of a
// rollout in one launch, so each env goes on to its next step as soon as it
// has finished one (no launch-wide barrier between steps: the launch lasts
// the slowest env's SUM of steps, not the sum of every step's slowest env).
// Lane state, the RNG (key in LDS once loaded) and the LDS cell table stay
// on the chip between steps; step t reads actions[t] and writes obs[t],
// reward[t], done[t], all_done[t] (strides E*A*act_dim, E*A*SS, E*A, E).
// waves per SIMD the step kernel is compiled for: 4 keeps it within 128
// VGPRs, so 16 one-wave envs (the LDS limit at TeamBattle's size) share a CU
constexpr int GW_STEP_WAVES_PER_EU = 4;
// a pending horizon reset counts as this many agent-steps of remaining work
// (192 -> 384 in round 5: the driver's command median 0.2298 -> 0.2253 ms over
// 8 alternating runs, 100-step fragments unchanged; profiles/r05/ab_prio_reset_w*.jsonl)
constexpr int GW_PRIO_RESET_W = 384;
// lane_step_kernel: steps of actions in flight ahead of the step (gw_lane.inc)
constexpr int GW_LANE_PD = 4;
// SPEC 1: the TeamBattle program without blocking entities and with one
// view range (BASELINE's headline config): the other programs' passes and
// the masked / mixed-range observation fold away at compile time (the
// generic kernel holds every program, and its register pressure spills)
template <int S, int SPEC = 0>
__global__ __launch_bounds__(WAVE, GW_STEP_WAVES_PER_EU) void step_kernel(Params p)
{
    constexpr bool PLAIN = SPEC == 1;
    const int sim_kind = PLAIN ? (int)GW_SIM_TEAM_BATTLE : p.sim_kind;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    if ((int)blockIdx.x >= p.E) return;
    const int e = blockIdx.x;
    const int l = lane_id();
    const int A = p.A;
    const bool valid = l < A;
    const int SS = S ? S * S : p.obs_side * p.obs_side;
    STAMP(0);
    STAMP_WAVE(60, true);
    Smem sm = carve(smem_raw, p);
    // every global load of the prologue is issued before any is used (one
    // memory round trip): the epilogue counters, the previous __all__ (read
    // unconditionally: a branch on it would wait for it), lanes, actions
    const int32_t steps_raw = p.steps[e];
    const uint32_t ad_raw = p.ad_in ? p.ad_in[e] : 0u;
    Lane L;
    load_lane<!PLAIN>(p, e, L, valid);
    // actions (lane = agent); attack == -1 marks "not in action_dict"
    const size_t EA = (size_t)p.E * A;
    const size_t act_row = ((size_t)e * A + (valid ? l : 0)) * p.act_dim;
    int mr, mc, ak;
    {
        const int32_t* ap = p.actions + act_row;
        const int a0 = ap[0], a1 = ap[1], a2 = ap[2];
        mr = valid ? a0 : 0; mc = valid ? a1 : 0; ak = valid ? a2 : -1;
    }
    const uint64_t acting_raw = p.acting ? p.acting[e] : 0ull;
    // the MT key with the prologue's loads (one round trip) when the launch
    // runs several steps: nearly every env of a fragment draws beyond its
    // cached block (crowded cells, placements), and a load on demand puts a
    // memory round trip on that env's chain
    // (also for single-step launches: measured 0.5-1 % slower, the envs that
    // draw nothing pay the load; profiles/r04/ab_closed_loop.jsonl)
    const bool kpre = p.nsteps > 1;
    uint4 kq0 = {}, kq1 = {}, kq2 = {};
    if (kpre) {
        const uint4* ks = (const uint4*)(p.mt + (size_t)e * GW_MT_STRIDE);
        constexpr int N4 = GW_MT_N / 4;
        kq0 = ks[l];
        kq1 = ks[l + WAVE];
        kq2 = ks[l + 2 * WAVE < N4 ? l + 2 * WAVE : l];
    }
    Rng rng;
    uint32_t ctr;
    load_env(p, e, sm, rng, ctr, true);
    if (kpre) {
        uint4* k4 = (uint4*)sm.key;
        k4[l] = kq0;
        k4[l + WAVE] = kq1;
        if (l + 2 * WAVE < GW_MT_N / 4) k4[l + 2 * WAVE] = kq2;
        wave_sync();
        rng.loaded = true;
    }
    int32_t steps = uni(steps_raw);
    uint64_t acting_sum = 0;
    bool prev_all = uni(ad_raw) != 0u;
    // the LDS table holds the template (load_env); lanes are added before
    // the first step that needs them (a reset adds its own)
    bool lanes_in = false, need_tmpl = false;
    for (int t = 0; t < p.nsteps; t++) {
        const Params& p = kernel_params();
        // issue priority (gw_rollout): the four envs of a SIMD start together,
        // and VALU issue goes by priority, then age, so a heavy young wave
        // would trail the others and end the launch alone.  Remaining-work
        // priority: the wave's remaining agent-steps in this fragment (live
        // agents x steps left, a pending horizon reset counted as
        // GW_PRIO_RESET_W agent-steps) against a typical env's (~24 live
        // agents): the SIMD issues the heaviest env first (measured +2.8 %
        // on the driver's command, profiles/r03/ab_prio_remaining_work.jsonl)
        int prio = 0;
        if (p.nsteps > 1) {
            const int left = p.nsteps - t;
            const int nlive = __popcll(__ballot(valid && L.live));
            const bool rpend = p.horizon > 0 && steps + left >= p.horizon;
            const int rem = left * nlive + (rpend ? GW_PRIO_RESET_W : 0);
            const int typ = left * 24;
            prio = rem * 4 >= typ * 6 ? 3 : (rem * 8 >= typ * 9 ? 2 : (rem * 4 >= typ * 3 ? 1 : 0));
        }
        set_prio(prio);
        STAMP(50);
        const int32_t* act_t = p.actions + (size_t)t * EA * p.act_dim;
        int32_t* obs_t = p.obs + (size_t)t * EA * SS;
        double* rew_t = p.reward + (size_t)t * EA;
        uint8_t* done_t = p.done + (size_t)t * EA;
        uint8_t* ad_t = p.all_done + (size_t)t * p.E;
        // this step's actions (step 0's came with the prologue); loading the
        // next step's ahead and parking them in LDS measured 2 % slower per
        // 100-step fragment (profiles/r03/ab_head_prefetch.jsonl)
        // (a step ahead in registers, round 5: neutral on the driver's command
        // and 100-step fragments, profiles/r05/ab_act_ahead_dropped_*.jsonl)
        if (t > 0) {
            const int32_t* ap = act_t + act_row;
            const int a0 = ap[0], a1 = ap[1], a2 = ap[2];
            mr = valid ? a0 : 0; mc = valid ? a1 : 0; ak = valid ? a2 : -1;
        }
        if (need_tmpl) { table_template(p, sm); lanes_in = false; need_tmpl = false; }
        // NEXT_STEP auto-reset: the episode ended in the previous step, so this
        // step is AllStepManager.reset for the env (actions ignored): obs =
        // first observation, reward 0, done = not an Agent, no __all__
        const bool next_reset = p.autoreset == 2 && (prev_all || (p.horizon > 0 && steps >= p.horizon));
        bool reset_now = next_reset;
        if (!next_reset) {
            if (ctr >= SEQ_RENORM) renorm_seq(p, L, ctr);
            const bool acting = valid && L.live && ak >= 0;
            const uint64_t act_mask = __ballot(acting);
            STAMP(10);
            if (!lanes_in) { build_tables(p, sm, L, false); lanes_in = true; }
            STAMP(1);
            L.reward = 0.0;
            // the step raised (GW_ERR_* bits): ReachTheTarget's double remove
            // (KeyError), BinaryAttackActor's numpy array (ValueError)
            uint32_t raised = 0u;

            // AllStepManager(randomize_action_input=True): the shuffled action
            // dict's order (the generic kernel only; TeamBattle, ReachTheTarget,
            // TrafficCorridor programs)
            const int32_t* aord = (!PLAIN && p.act_order) ? p.act_order + (size_t)e * A : nullptr;
            // body(a, k) for the lanes of m in dict order; k = the lane's rank
            // in it (its in-cell insertion offset when it moves)
            auto in_dict_order = [&](uint64_t m, auto&& body) {
                if (aord) {
                    for (int k = 0; k < A; k++) {
                        const int a = uni(aord[k]);
                        if ((m >> a) & 1ull) body(a, k);
                    }
                } else {
                    for (uint64_t it = m; it; it &= it - 1) {
                        const int a = first_lane(it);
                        body(a, a);
                    }
                }
            };
            if (sim_kind == GW_SIM_TEAM_BATTLE) {
                const int my_rank = (!PLAIN && p.act_order) ? p.act_rank[(size_t)e * A + (valid ? l : 0)] : l;
                // ---- attack pass (team_battle_example.py:35-47)
                const bool att = acting && (L.kind & GW_K_ATTACKING) && ak > 0;
                const bool maybe = att && L.active && attack_precheck(p, sm, L);
                const uint64_t maybe_mask = __ballot(maybe);
                // the launch lasts as long as its slowest env: an env with a long
                // serial attack chain gets issue priority over the SIMD's other waves
                {
                    const int nser = __popcll(maybe_mask);
                    if (nser >= 16 && prio < 2) set_prio(2);
                    else if (nser >= 8 && prio < 1) set_prio(1);
        #ifdef GW_STAMPS
                    const int natt = __popcll(__ballot(att));
                    if (l == 0 && p.stamps) {
                        p.stamps[(size_t)e * GW_STAMP_STRIDE + 28] = nser;
                        p.stamps[(size_t)e * GW_STAMP_STRIDE + 29] = natt;
                    }
        #endif
                }
                STAMP(7);
                // Only attackers with a possible target run serially.  The others get
                // (True, []) -> -0.1 if still active at their turn: applied lane-parallel
                // just before the next serial attacker after them (so each lane's
                // reward terms keep their reference order), or after the loop.
                uint64_t pend = __ballot(att) & ~maybe_mask;
        #ifdef GW_STAMPS
                uint64_t att_acc[7] = {0, 0, 0, 0, 0, 0, 0};     // slots 42-47, calls (48)
        #else
                uint64_t* att_acc = nullptr;
        #endif
                // one serial attacker; `before`: the pending lanes whose turn
                // came before a's
                auto serial_attack = [&](int a, uint64_t before) {
                    if (before) {
                        if (((before >> l) & 1ull) && L.active) L.reward -= 0.1;
                        pend &= ~before;
                    }
                    if (!rlb(L.active, a)) return;                  // killed earlier this pass
        #ifdef GW_STAMPS
                    att_acc[6] += 1;
        #endif
                    int nlist, list;
                    bool nd;
                    attack_one<PLAIN>(p, sm, rng, L, a, rl(ak, a), nlist, list, &nd, att_acc);
                    ACC_STAMP_T0(t1);
                    // `not attacked_agents` (team_battle_example.py:41) on a numpy
                    // array of 2 or more agents raises ValueError: the step stops
                    // here, this attack applied
                    if (nd && nlist >= 2 && !p.arr_as_list) { raised = GW_ERR_VALUE_ERROR; return; }
                    if (nlist == 0) { if (l == a) L.reward -= 0.1; }
                    else {
                        for (int t = 0; t < nlist; t++) {
                            const int b = rl(list, t);
                            if (!rlb(L.active, b)) {
                                if (l == b) L.reward -= 1.0;
                                if (l == a) L.reward += 1.0;
                            }
                        }
                    }
                    ACC_STAMP(47, t1);                          // rewards
                };
                if (aord) {
                    // randomize_action_input: the action dict's order
                    for (int k = 0; k < A && !raised; k++) {
                        const int a = uni(aord[k]);
                        if ((maybe_mask >> a) & 1ull) serial_attack(a, pend & __ballot(valid && my_rank < k));
                    }
                } else {
                    for (uint64_t it = maybe_mask; it && !raised; it &= it - 1) {
                        const int a = first_lane(it);
                        serial_attack(a, pend & ((1ull << a) - 1ull));
                    }
                }
                if (((pend >> l) & 1ull) && L.active) L.reward -= 0.1;
        #ifdef GW_STAMPS
                if (l == 0 && p.stamps)
                    for (int q = 0; q < 7; q++) p.stamps[(size_t)e * GW_STAMP_STRIDE + 42 + q] = att_acc[q];
        #endif
                STAMP(2);
                if (!raised) {
                    // ---- move pass (:50-55)
                    const bool mover = acting && L.active;
                    const bool can_move = mover && (L.kind & GW_K_MOVING);
                    const int nr = L.r + mr, nc = L.c + mc;
                    const bool inb = 0 <= nr && nr < p.H && 0 <= nc && nc < p.W;
                    const bool stay = nr == L.r && nc == L.c;
                    const bool real = can_move && inb && !stay;
                    // isolation: no other mover targets my source or target, none leaves my target
                    const int HW = p.H * p.W;
                    const int nw = (HW + 3) / 4;
                    {
                        // 16-byte stores (both arrays start on 16 bytes, padded)
                        const int nw4 = (nw + 3) >> 2;
                        const uint4 z = make_uint4(0u, 0u, 0u, 0u);
                        for (int i = l; i < nw4; i += WAVE) { ((uint4*)sm.tcnt)[i] = z; ((uint4*)sm.scnt)[i] = z; }
                    }
                    wave_sync();
                    const int src = L.r * p.W + L.c, tgt = nr * p.W + nc;
                    if (real) {
                        atomicAdd(&sm.tcnt[cnt_word(p, tgt)], 1u << (8 * (tgt & 3)));
                        atomicAdd(&sm.scnt[cnt_word(p, src)], 1u << (8 * (src & 3)));
                    }
                    wave_sync();
                    bool iso = false, iso_ok = false;
                    if (real && cnt_get(sm.tcnt, tgt) == 1 && cnt_get(sm.scnt, tgt) == 0 &&
                        cnt_get(sm.tcnt, src) == 0) {
                        const uint32_t b = sm.tbl[tbl_idx(p, nr, nc)];
                        if (b != CELL_CROWD) { iso = true; iso_ok = (b == 0) || ((L.ov >> b) & 1u); }
                    }
                    const int pr = L.r, pc = L.c;
                    bool moved = false;
                    if (iso && iso_ok) { L.r = nr; L.c = nc; L.seq = ctr + (uint32_t)my_rank; moved = true; }
                    bool fail = (mover && !can_move) || (can_move && !inb) || (iso && !iso_ok);
            #ifdef GW_STAMPS
                    {
                        const int nser = __popcll(__ballot(real && !iso)), nreal = __popcll(__ballot(real));
                        if (l == 0 && p.stamps) { p.stamps[(size_t)e * GW_STAMP_STRIDE + 30] = nser; p.stamps[(size_t)e * GW_STAMP_STRIDE + 31] = nreal; }
                    }
            #endif
                    STAMP(11);
                    const uint64_t ser = __ballot(real && !iso);
                    if (aord) {
                        // randomize_action_input: movers in the action dict's
                        // order, appended to their cells in that order
                        for (int k = 0; k < A; k++) {
                            const int a = uni(aord[k]);
                            if (!((ser >> a) & 1ull)) continue;
                            const bool ok = move_one(p, L, a, rl(mr, a), rl(mc, a), ctr + (uint32_t)k);
                            if (l == a) { fail = !ok; moved = ok; }
                        }
                    } else {
                        for (uint64_t it = ser; it; it &= it - 1) {
                            const int a = first_lane(it);
                            const bool ok = move_one(p, L, a, rl(mr, a), rl(mc, a), ctr + (uint32_t)a);
                            if (l == a) { fail = !ok; moved = ok; }
                        }
                    }
                    if (fail) L.reward -= 0.1;
                    ctr += (uint32_t)WAVE;
                    // ---- entropy (:58-59)
                    if (acting) L.reward -= 0.01;
                    // cell table after the moves
                    wave_sync();
                    if (moved) {
                        const int oc = pr * p.W + pc, ncl = L.r * p.W + L.c;
                        atomicSub(&sm.cnt[cnt_word(p, oc)], 1u << (8 * (oc & 3)));
                        atomicAdd(&sm.cnt[cnt_word(p, ncl)], 1u << (8 * (ncl & 3)));
                        sm.tbl[tbl_idx(p, pr, pc)] = 0;
                    }
                    wave_sync();
                    if (L.in_grid) sm.tbl[tbl_idx(p, L.r, L.c)] = cell_byte(cnt_get(sm.cnt, L.r * p.W + L.c), L.enc);
                    wave_sync();
                }
            } else if (sim_kind == GW_SIM_REACH_TARGET) {
                // ---- attack pass (reach_the_target.py:96-108): every acting agent,
                // dict order; only AttackingAgents attack (others return False, [])
                const int32_t* act_e = act_t + (size_t)e * A * p.act_dim;
                in_dict_order(__ballot(acting && (L.kind & GW_K_ATTACKING)), [&](int a, int) {
                    if (raised || !rlb(L.active, a)) return;
                    int nlist, list;
                    bool nd = false;
                    const bool status = p.attack_kind == GW_ATTACK_SELECTIVE
                        ? attack_selective(p, sm, rng, L, a, act_e + (size_t)a * p.act_dim + 2, nlist, list)
                        : attack_one<PLAIN>(p, sm, rng, L, a, rl(ak, a), nlist, list, &nd);
                    if (!status) return;
                    // `not attacked_agents` (reach_the_target.py:127) on a numpy array
                    if (nd && nlist >= 2 && !p.arr_as_list) { raised = GW_ERR_VALUE_ERROR; return; }
                    if (nlist == 0) { if (l == a) L.reward -= 0.1; }
                    else {
                        for (int t = 0; t < nlist; t++) {
                            const int b = rl(list, t);
                            if (!rlb(L.active, b)) {
                                if (l == b) L.reward -= 1.0;
                                if (l == a) L.reward += 1.0;
                            }
                        }
                    }
                });
                STAMP(2);
                // ---- move pass (:110-121): MovingAgents in dict order; active ones
                // move (-0.1 on failure); then any of them on the target's cell is
                // rewarded, removed from the grid and deactivated.  Removing one the
                // target already killed there is the reference's KeyError.
                const int t = p.target;
                const int tr = rl(L.r, t), tc = rl(L.c, t);         // the target never moves
                in_dict_order(__ballot(acting && (L.kind & GW_K_MOVING)), [&](int a, int k) {
                    if (raised) return;
                    if (rlb(L.active, a)) {
                        const bool ok = move_one(p, L, a, rl(mr, a), rl(mc, a), ctr + (uint32_t)k);
                        if (!ok && l == a) L.reward -= 0.1;
                    }
                    if (rl(L.r, a) == tr && rl(L.c, a) == tc) {
                        if (!rlb(L.in_grid, a)) {
                            // Grid.remove raises KeyError: the step stops here (no
                            // further moves, no observation draws); the env needs a
                            // reset, which the auto-reset modes do as for an ended
                            // episode (all_done set; SAME_STEP resets it right away)
                            raised = GW_ERR_DOUBLE_REMOVE;
                            return;
                        }
                        if (l == a) {
                            L.reward += 1.0;
                            L.in_grid = false;
                            L.active = false;
                        }
                    }
                });
                ctr += (uint32_t)WAVE;
                if (!raised) {
                    // ---- entropy for the runners (:123-126)
                    if (acting && (L.kind & GW_K_PROGRAM)) L.reward -= 0.01;
                    // the LDS table after the passes (observation)
                    build_tables(p, sm, L, true);
                }
            } else if (sim_kind == GW_SIM_TRAFFIC) {
                // ---- traffic_corridor.py:41-49: the action dict in dict order;
                // a failed move (None for non-MovingAgents) -0.1, then +1 when
                // get_done(agent) holds right after the agent's own move
                in_dict_order(act_mask, [&](int a, int k) {
                    const bool ok = move_one(p, L, a, rl(mr, a), rl(mc, a), ctr + (uint32_t)k);
                    if (!ok && l == a) L.reward -= 0.1;
                    if (lane_done_uniform(p, L, a) && l == a) L.reward += 1.0;
                });
                ctr += (uint32_t)WAVE;
                build_tables(p, sm, L, true);       // the LDS table after the moves
            } else if (sim_kind == GW_SIM_MAZE_NAV) {
                const int n = p.nav, t = p.target;
                if ((act_mask >> n) & 1) {
                    const int pr = rl(L.r, n), pc = rl(L.c, n);
                    const bool ok = move_one(p, L, n, rl(mr, n), rl(mc, n), ctr + (uint32_t)n);
                    if (!ok && l == n) L.reward -= 0.1;
                    const bool at = rl(L.r, n) == rl(L.r, t) && rl(L.c, n) == rl(L.c, t);
                    if (at && l == n) L.reward += 1.0;
                    if (l == n) L.reward -= 0.01;
                    ctr += (uint32_t)WAVE;
                    const int qr = rl(L.r, n), qc = rl(L.c, n);
                    if (ok && (qr != pr || qc != pc)) {
                        table_remove(p, sm, L, n, pr, pc);
                        const int ncl = qr * p.W + qc;
                        if (l == n) atomicAdd(&sm.cnt[cnt_word(p, ncl)], 1u << (8 * (ncl & 3)));
                        wave_sync();
                        if (L.in_grid && L.r == qr && L.c == qc)
                            sm.tbl[tbl_idx(p, qr, qc)] = cell_byte(cnt_get(sm.cnt, ncl), L.enc);
                        wave_sync();
                    }
                }
            }
            STAMP(3);
            if (raised) {
                // the step raised (Grid.remove's KeyError, the attack's
                // ValueError): it stops there (no further attacks or moves, no
                // observation draws, its outputs are not written); the env needs
                // a reset, which the auto-reset modes do as for an ended episode
                // (all_done set; SAME_STEP resets it right away)
                if (l == 0 && p.err) p.err[e] |= raised;
                steps += 1;
                acting_sum += (uint64_t)__popcll(act_mask);
                if (p.autoreset && l == 0) ad_t[e] = 1;
                prev_all = true;
                // the table is not the post-move grid: from the template
                if (p.autoreset == 1) { table_template(p, sm); reset_now = true; }
                else need_tmpl = true;
            } else {

                // ---- observations of the live agents (all_step_manager.py:68-71)
                STAMP(4);
                observe_all<S, PLAIN>(p, e, sm, rng, L, obs_t);
                STAMP(5);

                // ---- rewards, dones (:72-79, smart.py:101-111)
                bool dn;
                bool only_left = false;                 // OnlyAgentLeftDone (reach_the_target.py:41-55)
                if (sim_kind == GW_SIM_MAZE_NAV) {
                    const int n = p.nav, t = p.target;
                    dn = rl(L.r, n) == rl(L.r, t) && rl(L.c, n) == rl(L.c, t);
                } else if (sim_kind == GW_SIM_REACH_TARGET) {
                    const int t = p.target;
                    const bool is_agent = (L.kind & GW_K_OBSERVING) && (L.kind & GW_K_ACTING);
                    only_left = __popcll(__ballot(valid && is_agent && L.active)) <= 1;
                    const bool at_target = L.r == rl(L.r, t) && L.c == rl(L.c, t);
                    // runners: ActiveDone or TargetDone; the target: OnlyAgentLeftDone (:144-150)
                    dn = (L.kind & GW_K_PROGRAM) ? (!L.active || at_target) : only_left;
                } else {
                    dn = lane_done(p, L);
                }
                if (valid) {
                    size_t k = (size_t)e * A + l;
                    rew_t[k] = L.live ? L.reward : 0.0;
                    done_t[k] = L.live ? (uint8_t)dn : (uint8_t)1;
                }
                const bool live_after = valid && L.live && !dn;
                // get_all_done (done.py:49-56,147-153) or maze target reached
                bool all;
                if (sim_kind == GW_SIM_MAZE_NAV) {
                    all = dn;
                } else if (sim_kind == GW_SIM_REACH_TARGET) {
                    all = only_left;
                } else {
                    all = true;
                    // static entities are agents too, always active (done.py:49-56,147-153)
                    if (p.done_kind & GW_DONE_ACTIVE) all = all && p.static_encs == 0 && (__ballot(valid && L.active) == 0);
                    if (p.done_kind & GW_DONE_ONE_TEAM) {
                        uint32_t bits = wave_or((valid && L.active) ? (1u << L.enc) : 0u) | p.static_encs;
                        all = all && (__popc(bits) <= 1);
                    }
                    if (p.done_kind & (GW_DONE_TARGET_AGENT | GW_DONE_TARGET_DESTROYED))
                        all = all && targets_all_done(p, L);
                }
                const bool any_left = __ballot(live_after) != 0;
                L.live = live_after;
                const bool all_done = all || !any_left;
                steps += 1;
                acting_sum += (uint64_t)__popcll(act_mask);
                if (l == 0) ad_t[e] = (uint8_t)all_done;
                prev_all = all_done;
                // SAME_STEP auto-reset: the next episode's first observation replaces obs
                reset_now = p.autoreset == 1 && (all_done || (p.horizon > 0 && steps >= p.horizon));
            }
        }
        if (reset_now) {
            // the reset is the launch's critical path: issue it ahead of the
            // SIMD's stepping waves
            __builtin_amdgcn_s_setprio(3);
            wave_sync();
            STAMP(12);
            reset_env<S, PLAIN>(p, e, sm, rng, L, ctr, true, obs_t);
            STAMP(14);
            steps = 0;
            lanes_in = true;
            if (next_reset) {
                if (valid) {
                    const size_t k = (size_t)e * A + l;
                    rew_t[k] = 0.0;
                    done_t[k] = L.live ? (uint8_t)0 : (uint8_t)1;
                }
                if (l == 0) ad_t[e] = 0;
                prev_all = false;
            }
            set_prio(prio);
        }
    }
    if (l == 0) {
        p.steps[e] = steps;
        if (p.acting) p.acting[e] = acting_raw + acting_sum;
        if (p.ad_out) p.ad_out[e] = (uint8_t)prev_all;
    }
    store_lane<!PLAIN>(p, e, L, valid);
    store_rng(p, e, sm, rng, ctr);
    STAMP(6);
    STAMP_WAVE(61, false);
}

// CrossMoveActor.grid_action (actor.py:142-159): 0 stay, 1 left, 2 down, 3 right, 4 up
__device__ __forceinline__ int cross_row(int d) { return d == 2 ? 1 : (d == 4 ? -1 : 0); }
__device__ __forceinline__ int cross_col(int d) { return d == 1 ? -1 : (d == 3 ? 1 : 0); }

// AbsoluteEncodingObserver.get_obs (observer.py:95-150) for lane a (uniform)
// into out[H][W]: -2 outside the view range and behind blockers (every
// active blocking entity, create_grid_and_mask evaluated per cell with
// shadow_hides, so any view range), -1 the observer's own cell (no draw), 0
// empty, a lone occupant's encoding, and for a crowded cell
// np.random.choice over its occupants' encodings in insertion (seq) order,
// the draws in the window's row-major order (the reference's loop).
__device__ __forceinline__ void observe_absolute(const Params& p, const Smem& sm, Rng& rng, const Lane& L,
                                                 int a, int v, int32_t* out)
{
    const int l = lane_id(), A = p.A;
    const int ra = rl(L.r, a), ca = rl(L.c, a);
    const bool a_in = rlb(L.in_grid, a);
    const int self = a_in ? ra * p.W + ca : -1;
    const int r0 = ra - v > 0 ? ra - v : 0, r1 = ra + v < p.H - 1 ? ra + v : p.H - 1;
    const int c0 = ca - v > 0 ? ca - v : 0, c1 = ca + v < p.W - 1 ? ca + v : p.W - 1;
    const uint64_t blk = __ballot(l < A && L.active && (L.kind & GW_K_BLOCKING));
    auto hidden = [&](int gr, int gc) -> bool {
        bool h = false;
        for (uint64_t it = blk; it; it &= it - 1) {
            const int b = first_lane(it);
            const int dr = rl(L.r, b) - ra, dc = rl(L.c, b) - ca;
            if (dr >= -v && dr <= v && dc >= -v && dc <= v && shadow_hides(dr, dc, gr - ra, gc - ca))
                h = true;
        }
        for (int q = 0; q < p.n_sblk; q++) {          // static blockers: always active
            const int32_t sc = p.sblk[q];
            const int dr = (sc >> 16) - ra, dc = (sc & 0xffff) - ca;
            if (dr >= -v && dr <= v && dc >= -v && dc <= v && shadow_hides(dr, dc, gr - ra, gc - ca))
                h = true;
        }
        return h;
    };
    // crowded cells (>= 2 occupants, so a lane is there) ranked by cell index
    const int my = L.r * p.W + L.c;
    const bool crowded = l < A && L.in_grid && cnt_get(sm.cnt, my) >= 2;
    bool rep = crowded;
    for (uint64_t it = __ballot(crowded); it; it &= it - 1) {
        const int i = first_lane(it);
        if (crowded && i < l && rl(my, i) == my) rep = false;
    }
    const uint64_t reps = __ballot(rep);
    int rank = 0;
    for (uint64_t it = reps; it; it &= it - 1) {
        const int i = first_lane(it);
        if (rep && rl(my, i) < my) rank++;
    }
    const int ncl = __popcll(reps);
    int ccell = -1, cval = 0;                 // lane j: the j-th crowded cell and its value
    for (int j = 0; j < ncl; j++) {
        const int cell = rl(my, first_lane(__ballot(rep && rank == j)));
        const int gr = cell / p.W, gc = cell - gr * p.W;
        int val = -2;
        if (gr >= r0 && gr <= r1 && gc >= c0 && gc <= c1 && cell != self && !hidden(gr, gc)) {
            const uint32_t kk = rng.interval(cnt_get(sm.cnt, cell) - 1u);
            const bool in = l < A && L.in_grid && my == cell;
            uint32_t below = 0;
            for (uint64_t it = __ballot(in); it; it &= it - 1) {
                const int i = first_lane(it);
                if (in && rl(L.seq, i) < L.seq) below++;
            }
            val = rl(L.enc, first_lane(__ballot(in && below == kk)));
        }
        if (l == j) { ccell = cell; cval = val; }
    }
    const int HW = p.H * p.W;
    for (int i = l; i < HW; i += WAVE) {
        const int gr = i / p.W, gc = i - gr * p.W;
        int val;
        if (gr < r0 || gr > r1 || gc < c0 || gc > c1 || hidden(gr, gc)) {
            val = -2;
        } else if (i == self) {
            val = -1;
        } else {
            const uint32_t b = sm.tbl[tbl_idx(p, gr, gc)];
            val = (int)b;
            if (b == CELL_CROWD)
                for (int j = 0; j < ncl; j++)
                    if (rl(ccell, j) == i) val = rl(cval, j);
        }
        out[i] = val;
    }
}

// The component plugin API (state.py / actor.py / observer.py), one
// component call for ONE entity (lane p.obs_only) in every env: the wave
// loads the env, runs the component's body as the fused programs do, and
// stores the env back.  result[e] = {status, n, attacked lanes...}.
template <int S>
__global__ __launch_bounds__(WAVE) void comp_kernel(Params p)
{
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    if ((int)blockIdx.x >= p.E) return;
    const int e = blockIdx.x;
    const int l = lane_id();
    const int A = p.A;
    const bool valid = l < A;
    Smem sm = carve(smem_raw, p);
    Lane L;
    load_lane(p, e, L, valid);
    Rng rng;
    uint32_t ctr;
    load_env(p, e, sm, rng, ctr, true);
    const int op = p.mode, a = p.obs_lane;
    int32_t* res = p.comp_out ? p.comp_out + (size_t)e * (2 + A) : nullptr;
    int status = 0, nlist = 0, list = -1;
    int res2 = -1;                            // DRIFT_MOVE: result[2], the orientation
    uint32_t err = 0;
    // the component's own parameters come with the call (gw_engine.h)
    const int32_t* arg = p.actions ? p.actions + (size_t)e * p.act_dim : nullptr;
    Params q = p;
    if (op == GW_OP_POSITION_RESET || op == GW_OP_HEALTH_RESET) {
        if (arg) q.no_overlap_at_reset = uni(arg[0]);
        uint32_t c2 = ctr;
        const bool ok = do_reset(q, sm, rng, L, c2, err, op == GW_OP_POSITION_RESET ? 1 : 2);
        ctr = c2;
        status = ok ? 1 : 0;
    } else {
        if (ctr >= SEQ_RENORM) renorm_seq(p, L, ctr);
        build_tables(p, sm, L, false);
        if (op == GW_OP_MOVE) {
            // MoveActor.process_action (actor.py:82-114); None for non-MovingAgents
            if (!(rl(L.kind, a) & GW_K_MOVING)) {
                status = -1;
            } else {
                const int mr = uni(arg[0]), mc = uni(arg[1]);
                const int ar = rl(L.r, a), ac = rl(L.c, a);
                const bool in = rlb(L.in_grid, a);
                const bool ok = move_one(p, L, a, mr, mc, ctr + (uint32_t)a);
                // a move off a cell the agent is not in: Grid.remove raises KeyError
                if (ok && !in && (rl(L.r, a) != ar || rl(L.c, a) != ac)) {
                    err |= GW_ERR_NOT_IN_GRID;
                    if (l == a) { L.r = ar; L.c = ac; }
                }
                if (ok && l == a && (L.r != ar || L.c != ac)) L.in_grid = true;
                status = ok ? 1 : 0;
                ctr += (uint32_t)WAVE;
            }
        } else if (op == GW_OP_ATTACK) {
            // AttackActorBaseComponent.process_action (actor.py:306-361)
            if (rl(L.kind, a) & GW_K_ATTACKING) {
                const int f = uni(arg[0]);
                q.stacked = f & 1;
                const uint32_t amap = (uint32_t)uni(arg[1]);
                const uint32_t keep = L.amap;
                if (l == a) L.amap = amap;                  // attack_mapping[attacker's encoding]
                bool nd = false;
                const bool st = (f & 2)
                    ? attack_selective(q, sm, rng, L, a, arg + 2, nlist, list)
                    : attack_one(q, sm, rng, L, a, uni(arg[2]), nlist, list, &nd);
                if (l == a) L.amap = keep;
                status = st ? (nd ? 3 : 1) : 0;             // bit 1: a numpy array (actor.py:412-414)
            }
        } else if (op == GW_OP_CROSS_MOVE || op == GW_OP_DRIFT_MOVE) {
            // CrossMoveActor / DriftMoveActor.process_action (actor.py:161-234):
            // arg[0] the cross action, arg[1] (drift) the agent's orientation
            // (0 = None); status -1 None for an agent of another type, -2 a
            // drift with no orientation (the reference's AssertionError);
            // result[1] = 1 when the drift ran (action_dict['move'] was
            // replaced by the orientation), result[2] = the new orientation
            const uint32_t ak = (uint32_t)rl((int32_t)L.kind, a);
            const int cross = uni(arg[0]);
            const bool drift = op == GW_OP_DRIFT_MOVE;
            int orient = drift ? uni(arg[1]) : 0;
            const bool in = rlb(L.in_grid, a);
            const int ar = rl(L.r, a), ac = rl(L.c, a);
            auto cross_move = [&](int d) -> bool {
                const bool ok = move_one(p, L, a, cross_row(d), cross_col(d), ctr + (uint32_t)a);
                // a move off a cell the agent is not in: Grid.remove raises KeyError
                if (ok && !in && (rl(L.r, a) != ar || rl(L.c, a) != ac)) {
                    err |= GW_ERR_NOT_IN_GRID;
                    if (l == a) { L.r = ar; L.c = ac; }
                }
                if (ok && l == a && (L.r != ar || L.c != ac)) L.in_grid = true;
                return ok;
            };
            if (!(ak & GW_K_MOVING) || (drift && !(ak & GW_K_ORIENTATION))) {
                status = -1;
            } else if (!drift) {
                status = cross_move(cross) ? 1 : 0;
            } else if (cross != 0 && cross_move(cross)) {
                orient = cross;
                status = 1;
            } else if (orient < 1 || orient > 4) {
                status = -2;
            } else {
                nlist = 1;
                status = cross_move(orient) ? 1 : 0;
            }
            if (drift) res2 = orient;
            ctr += (uint32_t)WAVE;
        } else if (op == GW_OP_ORIENT_RESET) {
            // OrientationState.reset (state.py:666-675): initial_orientation or
            // np.random.randint(1, 5), OrientationAgents in agent order;
            // result[2 + lane] = the lane's orientation (0 for other lanes)
            int o = 0;
            for (uint64_t it = __ballot(valid && (L.kind & GW_K_ORIENTATION)); it; it &= it - 1) {
                const int b = first_lane(it);
                int ob = p.spec[b].init_orient;
                if (ob == 0) ob = 1 + (int)rng.interval(3u);
                if (l == b) o = ob;
            }
            status = 1;
            nlist = A;
            list = o;
        } else if (op == GW_OP_OBSERVE_ABS) {
            // arg[0]: the observer's view range (any range; the spec's is capped)
            observe_absolute(p, sm, rng, L, a, arg ? uni(arg[0]) : rl(L.view, a),
                             p.obs + ((size_t)e * A + a) * p.H * p.W);
        } else if (op == GW_OP_OBSERVE) {
            if (arg) q.observe_self = uni(arg[0]);
            q.obs_only = a;
            q.skip_done_obs = 1;
            q.persistent_obs = 0;
            observe_all<S>(q, e, sm, rng, L, p.obs);
        }
    }
    if (res) {
        if (l == 0) { res[0] = status; res[1] = nlist; }
        if (l < nlist && l < A) res[2 + l] = list;
        if (res2 >= 0 && l == 0) res[2] = res2;
    }
    if (l == 0 && p.err && err) p.err[e] |= err;
    store_lane(p, e, L, valid);
    store_rng(p, e, sm, rng, ctr);
}

template <int S>
__global__ __launch_bounds__(WAVE) void reset_kernel(Params p)
{
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    if ((int)blockIdx.x >= p.E) return;
    const int e = blockIdx.x;
    // reset everything when no selector is given; otherwise the union of the
    // explicit mask, the previous step's __all__ and the horizon
    bool go;
    if (p.mask == nullptr && p.prev_all_done == nullptr && p.horizon <= 0) go = true;
    else go = (p.mask && p.mask[e]) || (p.prev_all_done && p.prev_all_done[e]) ||
              (p.horizon > 0 && p.steps[e] >= p.horizon);
    if (!go) return;
    const int l = lane_id();
    const bool valid = l < p.A;
    Smem sm = carve(smem_raw, p);
    Lane L;
    load_lane(p, e, L, valid);
    Rng rng;
    uint32_t ctr;
    load_env(p, e, sm, rng, ctr, false);
    ctr = 0;
    if (l == 0 && p.err) p.err[e] = 0u;     // an explicit reset starts the env's flags afresh
    reset_env<S>(p, e, sm, rng, L, ctr, false, p.obs);
    if (l == 0) p.steps[e] = 0;
    store_lane(p, e, L, valid);
    store_rng(p, e, sm, rng, ctr);
}

// a key written by the host invalidates the cached tempered block
__global__ void invalidate_cache_kernel(uint32_t* mt, int E)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < E) mt[(size_t)e * GW_MT_STRIDE + MT_CBASE_SLOT] = 0xFFFFFFFFu;
}

// F_OBS_M2 is a fact about the engine's own obs buffer, not entity state:
// a snapshot never carries it and a restore clears it, so the next step
// rewrites every row (the restored obs buffer need not hold -2 there)
__global__ void clear_obs_m2_kernel(uint8_t* flags, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flags[i] &= (uint8_t)~F_OBS_M2;
}

__global__ void seed_kernel(uint32_t* mt, const uint32_t* seeds, int E)
{
    // np.random.seed(int) == init_genrand; one thread per env (once per run)
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    uint32_t* k = mt + (size_t)e * GW_MT_STRIDE;
    uint32_t s = seeds[e];
    for (int i = 0; i < GW_MT_N; i++) {
        k[i] = s;
        s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
    }
    k[MT_POS_SLOT] = GW_MT_N;
    k[MT_CTR_SLOT] = 0;
    k[MT_CBASE_SLOT] = 0xFFFFFFFFu;
}

// Philox-4x32-10
__device__ __forceinline__ uint4 philox(uint4 ctr, uint2 key)
{
    for (int i = 0; i < 10; i++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * ctr.x;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr.z;
        ctr = make_uint4((uint32_t)(p1 >> 32) ^ ctr.y ^ key.x, (uint32_t)p1,
                         (uint32_t)(p0 >> 32) ^ ctr.w ^ key.y, (uint32_t)p0);
        key.x += 0x9E3779B9u;
        key.y += 0xBB67AE85u;
    }
    return ctr;
}

// the policy's per-agent constants, packed into the kernel arguments (no
// dependent global load before the first store): kind | move_range << 8 |
// attack_range << 16 | simultaneous << 20
struct PolicySpec { uint32_t w[GW_MAX_LANES]; };
constexpr int RA_CROSS = 100;   // random_actions_kernel: cross moves (Pacman program)

__global__ void random_actions_kernel(PolicySpec ps, int E, int A, uint64_t key,
                                      uint32_t step, uint32_t env_offset, int32_t* actions,
                                      int act_dim, int attack_kind)
{
    // A <= 64: one wave per env, one lane per agent (no index division), 16
    // envs per workgroup; wider envs: one thread per (env, agent)
    int e, a;
    if (A <= WAVE) {
        e = blockIdx.x * 16 + (int)(threadIdx.x >> 6); a = threadIdx.x & 63;
    } else {
        const int i = blockIdx.x * blockDim.x + threadIdx.x;
        e = i / A; a = i - e * A;
    }
    if (e >= E || a >= A) return;
    const size_t i = (size_t)e * A + a;
    const uint32_t pw = ps.w[a];
    struct { uint32_t kind; int move_range, attack_range, simul; } s =
        {pw & 0xffu, (int)((pw >> 8) & 0xffu), (int)((pw >> 16) & 0xfu), (int)(pw >> 20)};
    const uint2 k2 = make_uint2((uint32_t)key, (uint32_t)(key >> 32));
    uint4 r = philox(make_uint4((uint32_t)e + env_offset, step, (uint32_t)a, 0x5EED), k2);
    const int m = s.move_range;
    const uint32_t span = (uint32_t)(2 * m + 1);
    int32_t* o = actions + (size_t)i * act_dim;
    if (attack_kind == RA_CROSS) {
        // CrossMoveActor / DriftMoveActor: Discrete(5); slot 2 >= 0 = in the dict
        o[0] = (s.kind & GW_K_MOVING) ? (int32_t)__umulhi(r.x, 5u) : 0;
        o[1] = 0;
        o[2] = 0;
        return;
    }
    // uniform on [0, n) by multiply-high (no integer division)
    o[0] = (s.kind & GW_K_MOVING) ? (int32_t)__umulhi(r.x, span) - m : 0;
    o[1] = (s.kind & GW_K_MOVING) ? (int32_t)__umulhi(r.y, span) - m : 0;
    const uint32_t na = (uint32_t)(s.simul + 1);
    if (attack_kind != GW_ATTACK_SELECTIVE) {
        o[2] = (s.kind & GW_K_ATTACKING) ? (int32_t)__umulhi(r.z, na) : 0;
        return;
    }
    // SelectiveAttackActor: Box(0, simultaneous, (2r+1, 2r+1)) per cell
    const int d = 2 * s.attack_range + 1;
    const int nc = (s.kind & GW_K_ATTACKING) ? d * d : 0;
    for (int q = 0; q < act_dim - 2; q++) {
        if ((q & 3) == 0 && q > 0)
            r = philox(make_uint4((uint32_t)e + env_offset, step, (uint32_t)a, 0x5EED + (uint32_t)(q >> 2)), k2);
        const uint32_t w = (q & 3) == 0 ? r.z : (q & 3) == 1 ? r.w : (q & 3) == 2 ? r.x : r.y;
        o[2 + q] = q < nc ? (int32_t)__umulhi(w, na) : 0;
    }
}

#ifndef GW_PART_S
#include "gw_pacman.inc"
#include "gw_maze.inc"
#endif
#include "gw_rtt.inc"
#include "gw_lane.inc"

}  // namespace

// ====================================================== per-window-size parts
// The templated kernels are instantiated once per observation window side S
// in their own translation unit (-DGW_PART_S=<S>; _native.build compiles the
// parts in parallel and links them with the host part).  Each part exports a
// launcher and an attribute setter; the host part dispatches on S to them.
enum PartKernel { PK_STEP = 0, PK_RESET = 1, PK_WG_STEP = 2, PK_WG_RESET = 3, PK_COMP = 4, PK_STEP_TB = 5, PK_STEP_LANE = 6,
                  PK_WG_COMP = 7, PK_STEP_LANE_NS = 8 };
// lane_step_kernel's instantiation for the rollout protocol (next-step
// auto-reset, skip_done_obs, no persistent obs buffer): its flags at compile time
#define LANE_FL_NS (2 | (1 << 3))
typedef hipError_t (*part_launch_fn)(int kind, unsigned grid, unsigned block, size_t smem,
                                     hipStream_t st, const void* params, hipEvent_t ev0, hipEvent_t ev1);
typedef hipError_t (*part_attr_fn)(int kind, size_t bytes);
typedef hipError_t (*part_occ_fn)(int kind, unsigned block, size_t smem, int* nblk);
#define GW_PART_CAT2(a, b) a##b
#define GW_PART_CAT(a, b) GW_PART_CAT2(a, b)
#define GW_PART_DECL(S_)                                                                      \
    hipError_t GW_PART_CAT(gw_part_launch_, S_)(int, unsigned, unsigned, size_t, hipStream_t, \
                                                const void*, hipEvent_t, hipEvent_t);         \
    hipError_t GW_PART_CAT(gw_part_attr_, S_)(int, size_t);                                  \
    hipError_t GW_PART_CAT(gw_part_occ_, S_)(int, unsigned, size_t, int*);
GW_PART_DECL(1) GW_PART_DECL(3) GW_PART_DECL(5) GW_PART_DECL(7)
GW_PART_DECL(9) GW_PART_DECL(11) GW_PART_DECL(13) GW_PART_DECL(15)
GW_PART_DECL(0)   // the generic window path: S at run time (> 2 * GW_FIXED_RANGE + 1)

#ifdef GW_PART_S
// ev0 / ev1 (gw_set_launch_events): the kernel's own start / end timestamps
// (hipExtLaunchKernel), no separate event records around the launch
#define GW_LAUNCH(K)                                                                          \
    do {                                                                                      \
        if (ev0) hipExtLaunchKernelGGL(K, dim3(grid), dim3(block), (uint32_t)smem, st, ev0, ev1, 0, p); \
        else hipLaunchKernelGGL(K, dim3(grid), dim3(block), smem, st, p);                     \
    } while (0)
hipError_t GW_PART_CAT(gw_part_launch_, GW_PART_S)(int kind, unsigned grid, unsigned block, size_t smem,
                                                   hipStream_t st, const void* params, hipEvent_t ev0,
                                                   hipEvent_t ev1)
{
    const Params& p = *static_cast<const Params*>(params);
#if GW_PART_S == 0
    // the generic window path: the one-wave step / reset / component kernels
    switch (kind) {
    case PK_STEP: GW_LAUNCH((step_kernel<0, 0>)); break;
    case PK_RESET: GW_LAUNCH((reset_kernel<0>)); break;
    case PK_COMP: GW_LAUNCH((comp_kernel<0>)); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
#else
    constexpr int S = GW_PART_S;
    switch (kind) {
    case PK_STEP: GW_LAUNCH((step_kernel<S, 0>)); break;
    case PK_STEP_TB: GW_LAUNCH((step_kernel<S, 1>)); break;
    case PK_RESET: GW_LAUNCH((reset_kernel<S>)); break;
    case PK_WG_STEP: GW_LAUNCH((wg_step_kernel<S>)); break;
    case PK_WG_RESET: GW_LAUNCH((wg_reset_kernel<S>)); break;
    case PK_COMP: GW_LAUNCH((comp_kernel<S>)); break;
    case PK_STEP_LANE: GW_LAUNCH((lane_step_kernel<S>)); break;
    case PK_STEP_LANE_NS: GW_LAUNCH((lane_step_kernel<S, LANE_FL_NS>)); break;
    case PK_WG_COMP: GW_LAUNCH((wg_comp_kernel<S>)); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
#endif
}

// the part's kernel for a PartKernel kind (nullptr: not in this part)
static const void* part_kernel(int kind)
{
#if GW_PART_S == 0
    return kind == PK_STEP ? (const void*)step_kernel<0, 0>
         : kind == PK_RESET ? (const void*)reset_kernel<0>
         : kind == PK_COMP ? (const void*)comp_kernel<0> : nullptr;
#else
    constexpr int S = GW_PART_S;
    switch (kind) {
    case PK_STEP: return (const void*)step_kernel<S, 0>;
    case PK_STEP_TB: return (const void*)step_kernel<S, 1>;
    case PK_RESET: return (const void*)reset_kernel<S>;
    case PK_WG_STEP: return (const void*)wg_step_kernel<S>;
    case PK_WG_RESET: return (const void*)wg_reset_kernel<S>;
    case PK_COMP: return (const void*)comp_kernel<S>;
    case PK_STEP_LANE: return (const void*)lane_step_kernel<S>;
    case PK_STEP_LANE_NS: return (const void*)lane_step_kernel<S, LANE_FL_NS>;
    case PK_WG_COMP: return (const void*)wg_comp_kernel<S>;
    default: return nullptr;
    }
#endif
}

hipError_t GW_PART_CAT(gw_part_attr_, GW_PART_S)(int kind, size_t bytes)
{
    const void* k = part_kernel(kind);
    if (!k) return hipErrorInvalidValue;
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// resident workgroups per CU of a kind's launch (gw_step_occupancy)
hipError_t GW_PART_CAT(gw_part_occ_, GW_PART_S)(int kind, unsigned block, size_t smem, int* nblk)
{
    const void* k = part_kernel(kind);
    if (!k) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(nblk, k, (int)block, smem);
}
#else   // ------------------------------------------------------- host part

// ====================================================================== C-ABI
struct gw_engine {
    // gw_set_launch_events: start / end events of the next step launch
    mutable hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int device;
    int E, A, H, W, S, max_enc;
    Params base;
    DevAgent* d_spec;
    uint4* d_tmpl;
    uint16_t* d_free;          // free_cell | cell_free
    uint32_t* d_static_bits;
    uint32_t* d_shadow;
    uint32_t* d_smask;
    uint32_t* d_hshadow;       // slot-geometry LUTs (observers with different ranges)
    uint32_t* d_hsmask;
    int32_t* d_sblk;           // static blockers (observe_big)
    int32_t lane_ent[GW_MAX_LANES];
    bool wg;                   // ReachTheTarget on a workgroup per env (gw_rtt.inc)
    bool step_tb;              // step_kernel<S, 1>: TeamBattle, no blockers, one view range
    bool lane_envs;            // lane_step_kernel<S>: MazeNavigation, one lane per env (gw_lane.inc)
    bool lane_envs_config;     // what gw_create chose (a placement order turns lane_envs off)
    int32_t* d_place_order;    // gw_set_placement_order: [E][A]
    int32_t* d_act_order;      // gw_set_action_order: order [E][A] | rank [E][A]
    size_t smem_lane;          // its dynamic LDS: the per-config tables
    PolicySpec policy;
    size_t smem_step, smem_reset;
    // Pacman program
    bool pacman;
    int16_t* d_passive;        // passive_cell [n_passive] | cell_passive [HW]
    int8_t* d_passive_enc;
    int32_t n_ent;             // gw_config.n_agents (lanes + static entities)
};

// gw_set_launch_events arms the NEXT kernel launch of the handle's step /
// reset kernels (part_launch / launch_pac consume and clear them).  Every
// other entry point, and every early return, clears them on exit, so a
// later unrelated launch never records them.
struct EvClear {
    gw_engine* g;
    ~EvClear() { if (g) g->ev0 = g->ev1 = nullptr; }
};

// create_grid_and_mask (utils.py:46-115): the window cells of range R that a
// blocker at offset (rd, cd) hides, as bits k = (r+R)(2R+1) + (c+R)
// (shadow_hides, the reference's arithmetic in double).
static void host_shadow(int R, int rd, int cd, uint32_t* bits)
{
    const int D = 2 * R + 1;
    for (int w = 0; w < mask_words(R); w++) bits[w] = 0u;
    for (int r = -R; r <= R; r++) {
        for (int c = -R; c <= R; c++) {
            if (shadow_hides(rd, cd, r, c)) {
                const int k = (r + R) * D + (c + R);
                bits[k >> 5] |= 1u << (k & 31);
            }
        }
    }
}

static thread_local char g_err[512];

static void set_err(const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

#define HIPCHK(x)                                                                 \
    do {                                                                          \
        hipError_t _e = (x);                                                      \
        if (_e != hipSuccess) {                                                   \
            set_err("%s: %s", #x, hipGetErrorString(_e));                        \
            return GW_E_HIP;                                                      \
        }                                                                         \
    } while (0)

// the parts, indexed by S / 2 (S = 1, 3, ..., 15), then the generic one (S > 15)
static const part_launch_fn k_part_launch[9] = {
    gw_part_launch_1, gw_part_launch_3, gw_part_launch_5, gw_part_launch_7,
    gw_part_launch_9, gw_part_launch_11, gw_part_launch_13, gw_part_launch_15, gw_part_launch_0};
static const part_attr_fn k_part_attr[9] = {
    gw_part_attr_1, gw_part_attr_3, gw_part_attr_5, gw_part_attr_7,
    gw_part_attr_9, gw_part_attr_11, gw_part_attr_13, gw_part_attr_15, gw_part_attr_0};
static const part_occ_fn k_part_occ[9] = {
    gw_part_occ_1, gw_part_occ_3, gw_part_occ_5, gw_part_occ_7,
    gw_part_occ_9, gw_part_occ_11, gw_part_occ_13, gw_part_occ_15, gw_part_occ_0};
constexpr int FIXED_S = 2 * GW_FIXED_RANGE + 1;

static int part_index(int S)
{
    if (S < 1 || !(S & 1) || S > 2 * GW_MAX_RANGE + 1) return -1;
    return S > FIXED_S ? 8 : S >> 1;
}

static hipError_t part_launch(const gw_engine* g, int kind, size_t smem, const Params& p, hipStream_t st)
{
    const int pi = part_index(g->S);
    if (pi < 0) return hipErrorInvalidValue;
    const unsigned block = (kind == PK_WG_STEP || kind == PK_WG_RESET || kind == PK_WG_COMP) ? WAVE * p.nwv : WAVE;
    const int epw = g->S <= FIXED_S ? WAVE / lane_group(g->S) : 1;   // lane_step_kernel: envs per wave
    const unsigned grid = (kind == PK_STEP_LANE || kind == PK_STEP_LANE_NS) ? (unsigned)((g->E + epw - 1) / epw)
                                                                           : (unsigned)g->E;
    // the events of gw_set_launch_events go to the next launch only
    const hipEvent_t ev0 = g->ev0, ev1 = g->ev1;
    g->ev0 = g->ev1 = nullptr;
    return k_part_launch[pi](kind, grid, block, smem, st, &p, ev0, ev1);
}

static hipError_t set_part_attrs(int S, int k0, int k1, size_t a, size_t b)
{
    const int pi = part_index(S);
    if (pi < 0) return hipErrorInvalidValue;
    hipError_t e = k_part_attr[pi](k0, a);
    return e != hipSuccess ? e : k_part_attr[pi](k1, b);
}

static hipError_t launch_pac(const gw_engine* g, const Params& p, hipStream_t st)
{
    // the step protocols' own instantiations (the other modes' code and its
    // registers out of the step loop); resets and the dict API: the generic one
    const hipEvent_t ev0 = g->ev0, ev1 = g->ev1;          // gw_set_launch_events: this launch only
    g->ev0 = g->ev1 = nullptr;
    auto go = [&](auto kernel) {
        if (ev0) hipExtLaunchKernelGGL(kernel, dim3(g->E), dim3(WAVE), (uint32_t)g->smem_step, st, ev0, ev1, 0, p);
        else hipLaunchKernelGGL(kernel, dim3(g->E), dim3(WAVE), g->smem_step, st, p);
    };
    if (p.mode == PAC_STEP_TURN) go(pac_kernel<PAC_STEP_TURN>);
    else if (p.mode == PAC_STEP_ALL) go(pac_kernel<PAC_STEP_ALL>);
    else go(pac_kernel<-1>);
    return hipGetLastError();
}

static hipError_t do_step(const gw_engine* g, Params& p, hipStream_t st)
{
    if (g->pacman) { p.mode = PAC_STEP_ALL; return launch_pac(g, p, st); }
    if (g->lane_envs) {
        const bool ns = p.autoreset == 2 && p.skip_done_obs && !p.persistent_obs;
        return part_launch(g, ns ? PK_STEP_LANE_NS : PK_STEP_LANE, g->smem_lane, p, st);
    }
    // an action order other than the agents dict's runs on the generic kernel
    const bool tb = g->step_tb && !p.act_order;
    return part_launch(g, g->wg ? PK_WG_STEP : (tb ? PK_STEP_TB : PK_STEP), g->smem_step, p, st);
}

static hipError_t do_reset(const gw_engine* g, Params& p, hipStream_t st)
{
    if (g->pacman) { p.mode = PAC_RESET_ALL; return launch_pac(g, p, st); }
    return part_launch(g, g->wg ? PK_WG_RESET : PK_RESET, g->smem_reset, p, st);
}

extern "C" {

int32_t gw_abi_version(void) { return 7; }
const char* gw_last_error(void) { return g_err; }

gw_status gw_create(const gw_config* cfg, int32_t n_envs, int32_t device, gw_handle* out)
{
    if (!cfg || !out || n_envs <= 0) { set_err("invalid argument"); return GW_E_INVALID; }
    const int NE = cfg->n_agents, HW = cfg->rows * cfg->cols;
    if (NE <= 0 || NE > GW_MAX_ENTITIES) {
        set_err("n_agents=%d outside 1..%d", NE, GW_MAX_ENTITIES);
        return GW_E_UNSUPPORTED;
    }
    if (cfg->rows <= 0 || cfg->cols <= 0 || HW > GW_MAX_CELLS) {
        set_err("grid %dx%d outside the engine's %d cells", cfg->rows, cfg->cols, GW_MAX_CELLS);
        return GW_E_UNSUPPORTED;
    }
    if (cfg->obs_range < 0 || cfg->obs_range > GW_MAX_RANGE) {
        set_err("obs_range %d > %d", cfg->obs_range, GW_MAX_RANGE);
        return GW_E_UNSUPPORTED;
    }
    if (cfg->sim_kind != GW_SIM_TEAM_BATTLE && cfg->sim_kind != GW_SIM_MAZE_NAV &&
        cfg->sim_kind != GW_SIM_REACH_TARGET && cfg->sim_kind != GW_SIM_PACMAN &&
        cfg->sim_kind != GW_SIM_TRAFFIC) {
        set_err("unknown sim_kind %d", cfg->sim_kind);
        return GW_E_INVALID;
    }
    int max_enc = 0;
    for (int a = 0; a < NE; a++) {
        const gw_agent_spec& s = cfg->agents[a];
        if (s.encoding < 1 || s.encoding > GW_MAX_ENC) { set_err("agent %d encoding %d", a, s.encoding); return GW_E_UNSUPPORTED; }
        if ((s.kind & GW_K_GRID_OBSERVER) && cfg->obs_kind != GW_OBS_ABSOLUTE &&
            (s.view_range < 0 || s.view_range > cfg->obs_range)) {
            set_err("agent %d view_range %d outside 0..obs_range %d", a, s.view_range, cfg->obs_range);
            return GW_E_UNSUPPORTED;
        }
        if ((s.kind & GW_K_ATTACKING) && (s.attack_range < 0 || s.attack_range > GW_MAX_ATTACK_RANGE)) {
            set_err("agent %d attack_range %d", a, s.attack_range);
            return GW_E_UNSUPPORTED;
        }
        if (s.init_row >= cfg->rows || s.init_col >= cfg->cols) { set_err("agent %d initial position outside the grid", a); return GW_E_INVALID; }
        // the agent classes' own assertions (agent.py:122-288)
        if ((s.kind & GW_K_MOVING) && s.move_range < 0) { set_err("agent %d move_range %d", a, s.move_range); return GW_E_INVALID; }
        if ((s.kind & GW_K_ATTACKING) &&
            (s.simultaneous_attacks < 0 || !(s.attack_strength >= 0.0 && s.attack_strength <= 1.0) ||
             !(s.attack_accuracy >= 0.0 && s.attack_accuracy <= 1.0))) {
            set_err("agent %d attack parameters (simultaneous %d, strength %g, accuracy %g)", a,
                    s.simultaneous_attacks, s.attack_strength, s.attack_accuracy);
            return GW_E_INVALID;
        }
        if ((s.kind & GW_K_HEALTH) && s.initial_health == s.initial_health && s.initial_health >= 0.0 &&
            !(s.initial_health > 0.0 && s.initial_health <= 1.0)) {
            set_err("agent %d initial_health %g outside (0, 1]", a, s.initial_health);
            return GW_E_INVALID;
        }
        if (s.encoding > max_enc) max_enc = s.encoding;
    }
    const bool maze = cfg->sim_kind == GW_SIM_MAZE_NAV;
    const bool rtt = cfg->sim_kind == GW_SIM_REACH_TARGET;
    const bool pac = cfg->sim_kind == GW_SIM_PACMAN;
    if ((cfg->obs_kind == GW_OBS_ABSOLUTE) != pac) {
        set_err("the AbsoluteEncodingObserver runs with the Pacman program (and only it)");
        return GW_E_UNSUPPORTED;
    }
    if (pac) {
        // the program places every entity at its initial position (no two in
        // one cell), keeps the food passive and has no blocking (gw_pacman.inc)
        if (cfg->pacman_agent < 0 || cfg->pacman_agent >= NE) { set_err("pacman needs pacman_agent"); return GW_E_INVALID; }
        std::vector<uint8_t> used(HW, 0);
        for (int a = 0; a < NE; a++) {
            const gw_agent_spec& s = cfg->agents[a];
            if (s.init_row < 0 || s.init_col < 0) { set_err("pacman program: entity %d has no initial position", a); return GW_E_UNSUPPORTED; }
            const int cell = s.init_row * cfg->cols + s.init_col;
            if (used[cell]) { set_err("pacman program: entities share initial cell %d", cell); return GW_E_UNSUPPORTED; }
            used[cell] = 1;
            if (s.kind & GW_K_BLOCKING) { set_err("pacman program: blocking entity %d", a); return GW_E_UNSUPPORTED; }
            if ((s.kind & GW_K_FOOD) && ((s.kind & ~(GW_K_FOOD | GW_K_HEALTH)) || s.initial_health < 0)) {
                set_err("pacman program: food %d must be a HealthAgent with an initial health only", a);
                return GW_E_UNSUPPORTED;
            }
        }
        if (cfg->agents[cfg->pacman_agent].kind & GW_K_FOOD) { set_err("pacman is food"); return GW_E_INVALID; }
    }
    if (maze && (cfg->nav_agent < 0 || cfg->nav_agent >= NE || cfg->target_agent < 0 || cfg->target_agent >= NE)) {
        set_err("maze navigation needs nav_agent/target_agent");
        return GW_E_INVALID;
    }
    if (rtt && (cfg->target_agent < 0 || cfg->target_agent >= NE)) {
        set_err("reach-the-target needs target_agent");
        return GW_E_INVALID;
    }
    if (cfg->attack_kind != GW_ATTACK_BINARY && cfg->attack_kind != GW_ATTACK_SELECTIVE) {
        set_err("unknown attack_kind %d", cfg->attack_kind);
        return GW_E_INVALID;
    }
    if (cfg->attack_kind == GW_ATTACK_SELECTIVE) {
        for (int a = 0; a < NE; a++) {
            const gw_agent_spec& s = cfg->agents[a];
            const int d = 2 * s.attack_range + 1;
            if ((s.kind & GW_K_ATTACKING) && d * d * (s.simultaneous_attacks > 0 ? s.simultaneous_attacks : 1) > WAVE) {
                set_err("agent %d: (2r+1)^2 * simultaneous_attacks > %d attacked slots", a, WAVE);
                return GW_E_UNSUPPORTED;
            }
        }
    }
    // ---- entities -> static entities | lanes (gw_engine.h "Entities and lanes")
    uint32_t attacked = 0, overlapped = 0;
    for (int e = 0; e <= GW_MAX_ENC; e++) { attacked |= cfg->attack_mapping[e]; overlapped |= cfg->overlap[e]; }
    const uint32_t dynamic_kinds = GW_K_OBSERVING | GW_K_ACTING | GW_K_GRID_OBSERVER | GW_K_MOVING |
                                   GW_K_ATTACKING | GW_K_HEALTH;
    std::vector<int> lanes, statics, passive;
    for (int a = 0; a < NE; a++) {
        const gw_agent_spec& s = cfg->agents[a];
        if (pac && (s.kind & GW_K_FOOD)) { passive.push_back(a); continue; }
        const bool st = !cfg->all_lanes && !(s.kind & (dynamic_kinds | GW_K_LANE)) && s.init_row >= 0 && s.init_col >= 0 &&
                        cfg->overlap[s.encoding] == 0 && !((overlapped >> s.encoding) & 1u) &&
                        !((attacked >> s.encoding) & 1u) &&
                        !((maze || rtt) && (a == cfg->nav_agent || a == cfg->target_agent));
        (st ? statics : lanes).push_back(a);
    }
    const int A = (int)lanes.size();
    // ReachTheTarget runs on a workgroup per env when it has more lanes than a
    // wave (or when the config forces it: the parity tests run the small
    // reference fixtures through it)
    // ReachTheTarget (SelectiveAttackActor) and TeamBattle (BinaryAttackActor)
    // run on a workgroup per env when they have more lanes than a wave (or
    // when the config forces it: the parity tests run small reference
    // fixtures through it)
    const bool tb = cfg->sim_kind == GW_SIM_TEAM_BATTLE;
    // (a component-API handle runs only gw_component operations: either
    // attack kind)
    const bool wg_able = (rtt && cfg->attack_kind == GW_ATTACK_SELECTIVE) ||
                         (tb && cfg->attack_kind == GW_ATTACK_BINARY) ||
                         (cfg->component_api && (rtt || tb));
    if (cfg->force_workgroup < 0 || cfg->force_workgroup > GW_MAX_LANES / WAVE) {
        set_err("force_workgroup %d: 0 (automatic), 1 (workgroup kernel) or 2..%d waves per env",
                cfg->force_workgroup, GW_MAX_LANES / WAVE);
        return GW_E_INVALID;
    }
    if (cfg->force_workgroup && !wg_able) {
        set_err("force_workgroup: the workgroup-per-env kernel runs ReachTheTarget with SelectiveAttackActor "
                "and TeamBattle with BinaryAttackActor");
        return GW_E_UNSUPPORTED;
    }
    const bool wg = wg_able && (A > GW_MAX_AGENTS || cfg->force_workgroup);
    // windows wider than the compiled parts: the generic window path of the
    // one-wave kernels (observe_big)
    const bool big = !pac && 2 * cfg->obs_range + 1 > FIXED_S;
    if (big && wg) {
        set_err("view ranges above %d run on the one-wave kernel (at most %d entities)", GW_FIXED_RANGE,
                GW_MAX_AGENTS);
        return GW_E_UNSUPPORTED;
    }
    const int max_lanes = wg_able ? GW_MAX_LANES : GW_MAX_AGENTS;
    if (A == 0 || A > max_lanes) {
        set_err("%d dynamic entities outside 1..%d (%s)", A, max_lanes,
                wg_able ? "one workgroup thread each" : "one wavefront lane each");
        return GW_E_UNSUPPORTED;
    }
    if (wg && tb) {
        for (int l = 0; l < A; l++) {
            const gw_agent_spec& s = cfg->agents[lanes[l]];
            if ((s.kind & GW_K_ATTACKING) && s.simultaneous_attacks > WG_LIST) {
                set_err("agent %d: simultaneous_attacks %d > %d on the workgroup kernel", lanes[l],
                        s.simultaneous_attacks, WG_LIST);
                return GW_E_UNSUPPORTED;
            }
        }
    }
    if ((int)passive.size() > 32 * PAC_MAX_PWORDS) {
        set_err("%d food entities > %d", (int)passive.size(), 32 * PAC_MAX_PWORDS);
        return GW_E_UNSUPPORTED;
    }
    {
        // the cell -> food map holds one food per cell (food_at, pac_tables)
        std::vector<uint8_t> has_food(HW, 0);
        for (int a : passive) {
            if (cfg->agents[a].encoding < 0 || cfg->agents[a].encoding > 127) {   // packed with its index
                set_err("food entity %d: encoding %d outside [0, 127]", a, cfg->agents[a].encoding);
                return GW_E_UNSUPPORTED;
            }
            const int cell = cfg->agents[a].init_row * cfg->cols + cfg->agents[a].init_col;
            if (cell < 0 || cell >= HW || has_food[cell]++) {
                set_err("food entity %d: its cell is off the grid or holds another food", a);
                return GW_E_UNSUPPORTED;
            }
        }
    }
    std::vector<uint8_t> is_static(HW, 0);
    for (int a : statics) {
        const int cell = cfg->agents[a].init_row * cfg->cols + cfg->agents[a].init_col;
        if (is_static[cell]) {   // Grid.place of the second one fails at every reset
            set_err("static entities %d share cell %d (the reference raises at every reset)", a, cell);
            return GW_E_INVALID;
        }
        is_static[cell] = 1;
    }
    for (int a : lanes) {
        const gw_agent_spec& s = cfg->agents[a];
        if (s.init_row >= 0 && is_static[s.init_row * cfg->cols + s.init_col]) {
            set_err("agent %d's initial position holds a static entity (the reference raises at every reset)", a);
            return GW_E_INVALID;
        }
    }
    bool any_block = false, lane_block = false;
    for (int a = 0; a < NE; a++) any_block |= (cfg->agents[a].kind & GW_K_BLOCKING) != 0;
    for (int a : lanes) lane_block |= (cfg->agents[a].kind & GW_K_BLOCKING) != 0;
    if (hipSetDevice(device) != hipSuccess) { set_err("hipSetDevice(%d) failed", device); return GW_E_HIP; }

    gw_engine* g = new gw_engine();
    memset(&g->base, 0, sizeof(Params));
    g->device = device; g->E = n_envs; g->A = A; g->H = cfg->rows; g->W = cfg->cols;
    g->S = pac ? 1 : 2 * cfg->obs_range + 1; g->max_enc = max_enc;
    g->pacman = pac;
    g->wg = wg;
    g->n_ent = NE;
    for (int i = 0; i < A; i++) g->lane_ent[i] = lanes[i];
    const size_t EA = (size_t)n_envs * A;
    Params& p = g->base;
    HIPCHK(hipMalloc(&p.pos, EA * sizeof(int2)));
    HIPCHK(hipMalloc(&p.health, EA * sizeof(double)));
    HIPCHK(hipMalloc(&p.flags, EA));
    HIPCHK(hipMalloc(&p.seq, EA * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&p.mt, (size_t)n_envs * GW_MT_STRIDE * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&p.steps, (size_t)n_envs * sizeof(int32_t)));
    HIPCHK(hipMemset(p.pos, 0, EA * sizeof(int2)));
    HIPCHK(hipMemset(p.health, 0, EA * sizeof(double)));
    HIPCHK(hipMemset(p.flags, 0, EA));
    HIPCHK(hipMemset(p.seq, 0, EA * sizeof(uint32_t)));
    HIPCHK(hipMemset(p.mt, 0, (size_t)n_envs * GW_MT_STRIDE * sizeof(uint32_t)));
    HIPCHK(hipMemset(p.steps, 0, (size_t)n_envs * sizeof(int32_t)));
    HIPCHK(hipMalloc(&p.ammo, EA * sizeof(int32_t)));
    HIPCHK(hipMemset(p.ammo, 0, EA * sizeof(int32_t)));
    DevAgent hs[GW_MAX_LANES];
    for (int l = 0; l < A; l++) {
        const gw_agent_spec& s = cfg->agents[lanes[l]];
        hs[l].enc = s.encoding; hs[l].kind = s.kind; hs[l].init_r = s.init_row; hs[l].init_c = s.init_col;
        hs[l].ov = cfg->overlap[s.encoding]; hs[l].amap = cfg->attack_mapping[s.encoding];
        hs[l].view_range = s.view_range; hs[l].move_range = s.move_range;
        hs[l].attack_range = s.attack_range; hs[l].simul = s.simultaneous_attacks;
        hs[l].strength = s.attack_strength; hs[l].accuracy = s.attack_accuracy;
        hs[l].init_health = s.initial_health;
        hs[l].init_orient = s.initial_orientation;
        hs[l].tgt_lane = -1; hs[l].tgt_pos = 0; hs[l].dtgt_lane = -1;
        // AmmoState.reset assigns initial_ammo through the ammo setter, which
        // clamps to 0 (agent.py:308-311, state.py:651-656)
        hs[l].init_ammo = (s.kind & GW_K_AMMO) ? (s.initial_ammo < 0 ? 0 : s.initial_ammo) : 0;
    }
    for (int l = 0; l < GW_MAX_LANES; l++) {
        g->policy.w[l] = l < A ? ((hs[l].kind & 0xffu) | ((uint32_t)(hs[l].move_range & 0xff) << 8) |
                                  ((uint32_t)(hs[l].attack_range & 0xf) << 16) |
                                  ((uint32_t)(hs[l].simul & 0xfff) << 20)) : 0u;
    }
    // done components' targets (TargetAgentDone / TargetDestroyedDone)
    {
        const uint32_t tbits = GW_DONE_TARGET_AGENT | GW_DONE_TARGET_DESTROYED;
        if ((cfg->done_kind & tbits) && cfg->sim_kind != GW_SIM_TEAM_BATTLE && cfg->sim_kind != GW_SIM_TRAFFIC) {
            set_err("TargetAgentDone / TargetDestroyedDone run with the TeamBattle and traffic programs");
            return GW_E_UNSUPPORTED;
        }
        std::vector<int> lane_of(NE, -1);
        for (int l = 0; l < A; l++) lane_of[lanes[l]] = l;
        for (int a = 0; a < NE; a++) {
            const gw_agent_spec& s = cfg->agents[a];
            if (s.done_target < -1 || s.done_target >= NE || s.destroy_target < -1 || s.destroy_target >= NE) {
                set_err("agent %d: target index outside the entities", a);
                return GW_E_INVALID;
            }
            if (lane_of[a] < 0 && (s.done_target >= 0 || s.destroy_target >= 0)) {
                set_err("static entity %d as a target_mapping key", a);
                return GW_E_UNSUPPORTED;
            }
        }
        for (int l = 0; l < A; l++) {
            const gw_agent_spec& s = cfg->agents[lanes[l]];
            if (s.done_target >= 0) {
                const int t = s.done_target;
                hs[l].tgt_lane = lane_of[t] >= 0 ? lane_of[t] : -2;
                hs[l].tgt_pos = (cfg->agents[t].init_row << 16) | cfg->agents[t].init_col;
            }
            if (s.destroy_target >= 0) hs[l].dtgt_lane = lane_of[s.destroy_target] >= 0 ? lane_of[s.destroy_target] : -2;
        }
    }
    HIPCHK(hipMalloc(&g->d_spec, sizeof(DevAgent) * A));
    HIPCHK(hipMemcpy(g->d_spec, hs, sizeof(DevAgent) * A, hipMemcpyHostToDevice));
    p.spec = g->d_spec;
    p.E = n_envs; p.A = A; p.H = cfg->rows; p.W = cfg->cols; p.max_enc = max_enc;
    p.sim_kind = cfg->sim_kind; p.nav = -1; p.target = -1;
    for (int l = 0; l < A; l++) {
        if (maze && lanes[l] == cfg->nav_agent) p.nav = l;
        if ((maze || rtt) && lanes[l] == cfg->target_agent) p.target = l;
    }
    p.act_dim = gw_config_act_dim(cfg);
    p.attack_kind = cfg->attack_kind;
    p.persistent_obs = cfg->persistent_obs != 0;
    p.obs_only = -1;
    p.comp_amap = -1;
    p.observe_self = cfg->observe_self; p.stacked = cfg->stacked_attacks;
    p.arr_as_list = cfg->attack_array_as_list;
    p.no_overlap_at_reset = cfg->no_overlap_at_reset; p.state_order = cfg->state_order;
    p.done_kind = cfg->done_kind;
    for (int i = 0; i <= GW_MAX_ENC; i++) { p.overlap[i] = cfg->overlap[i]; p.amap[i] = cfg->attack_mapping[i]; }
    // padded cell table: border = max(view range, attack ranges); rows are
    // read as dwords, so the pitch is a multiple of 4 with slack for the
    // over-read, plus one slack row at the end.  Static entities are part of
    // the template.
    // (the generic window path bounds-checks its windows: attack ranges only)
    int pad = big ? 0 : cfg->obs_range;
    for (int l = 0; l < A; l++)
        if ((hs[l].kind & GW_K_ATTACKING) && hs[l].attack_range > pad) pad = hs[l].attack_range;
    const int Sst = big ? 1 : g->S;             // the observation stage's window side
    p.pad = pad;
    p.obs_side = g->S;
    p.pitch = ((cfg->cols + 2 * pad + 3) / 4) * 4 + 4 * ((Sst + 3) / 4 + 1);
    p.tbl_rows = cfg->rows + 2 * pad + 1;
    {
        const size_t tb = align16((size_t)p.tbl_rows * p.pitch);
        std::vector<uint8_t> ht(tb);
        for (size_t i = 0; i < tb; i++) {
            const int row = (int)(i / p.pitch) - pad, col = (int)(i % p.pitch) - pad;
            ht[i] = (row < 0 || row >= cfg->rows || col < 0 || col >= cfg->cols) ? CELL_OFF : 0;
        }
        for (int a : statics) {
            const gw_agent_spec& s = cfg->agents[a];
            ht[(size_t)(s.init_row + pad) * p.pitch + (s.init_col + pad)] = (uint8_t)s.encoding;
        }
        for (int a : passive) {                 // present unless eaten (gw_pacman.inc)
            const gw_agent_spec& s = cfg->agents[a];
            ht[(size_t)(s.init_row + pad) * p.pitch + (s.init_col + pad)] = (uint8_t)s.encoding;
        }
        // + the unpadded copy (pac_kernel keeps one beside the table)
        ht.resize(tb + align16((size_t)HW), 0);
        for (int r = 0; r < cfg->rows; r++)
            for (int c = 0; c < cfg->cols; c++)
                ht[tb + (size_t)r * cfg->cols + c] = ht[(size_t)(r + pad) * p.pitch + (c + pad)];
        HIPCHK(hipMalloc(&g->d_tmpl, ht.size()));
        HIPCHK(hipMemcpy(g->d_tmpl, ht.data(), ht.size(), hipMemcpyHostToDevice));
        p.tbl_tmpl = g->d_tmpl;
        p.ob_tmpl = (const uint4*)((const uint8_t*)g->d_tmpl + tb);
    }
    // free cells (PositionState lists never hold a static cell: every list
    // loses it when the static entity is placed, before any draw)
    p.n_free = HW - (int)statics.size();
    if (!statics.empty()) {
        std::vector<uint16_t> fc(p.n_free + HW);
        std::vector<uint32_t> sb((HW + 31) / 32, 0u);
        int k = 0;
        for (int c = 0; c < HW; c++) {
            fc[p.n_free + c] = (uint16_t)k;
            if (is_static[c]) sb[c >> 5] |= 1u << (c & 31);
            else fc[k++] = (uint16_t)c;
        }
        HIPCHK(hipMalloc(&g->d_free, fc.size() * 2));
        HIPCHK(hipMemcpy(g->d_free, fc.data(), fc.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMalloc(&g->d_static_bits, sb.size() * 4));
        HIPCHK(hipMemcpy(g->d_static_bits, sb.data(), sb.size() * 4, hipMemcpyHostToDevice));
        p.free_cell = g->d_free;
        p.cell_free = g->d_free + p.n_free;
        p.static_bits = g->d_static_bits;
    }
    for (int a : statics) p.static_encs |= 1u << cfg->agents[a].encoding;
    // blocking: shadow LUT for every range, static masks for the ranges in use
    p.blockers = any_block;
    p.lane_blockers = lane_block;
    for (int r = 0; r <= GW_FIXED_RANGE; r++) p.smask_off[r] = -1;
    if (any_block) {
        std::vector<uint32_t> lut;
        for (int r = 0; r <= GW_FIXED_RANGE; r++) {
            p.shadow_off[r] = (int)lut.size();
            const int D = 2 * r + 1, mw = mask_words(r);
            lut.resize(lut.size() + (size_t)D * D * mw);
            for (int dr = -r; dr <= r; dr++)
                for (int dc = -r; dc <= r; dc++)
                    host_shadow(r, dr, dc, lut.data() + p.shadow_off[r] + ((dr + r) * D + (dc + r)) * mw);
        }
        HIPCHK(hipMalloc(&g->d_shadow, lut.size() * 4));
        HIPCHK(hipMemcpy(g->d_shadow, lut.data(), lut.size() * 4, hipMemcpyHostToDevice));
        p.shadow = g->d_shadow;
        bool used[GW_FIXED_RANGE + 1] = {};
        for (int l = 0; l < A; l++) {
            if ((hs[l].kind & GW_K_GRID_OBSERVER) && !big) used[cfg->obs_range] = true;
            if (hs[l].kind & GW_K_ATTACKING) used[hs[l].attack_range] = true;
        }
        std::vector<int> sblock;
        for (int a : statics) if (cfg->agents[a].kind & GW_K_BLOCKING) sblock.push_back(a);
        if (!sblock.empty()) {                  // observe_big / observe_absolute: the static blockers' cells
            std::vector<int32_t> sl;
            for (int a : sblock) sl.push_back((cfg->agents[a].init_row << 16) | cfg->agents[a].init_col);
            HIPCHK(hipMalloc(&g->d_sblk, sl.size() * 4));
            HIPCHK(hipMemcpy(g->d_sblk, sl.data(), sl.size() * 4, hipMemcpyHostToDevice));
            p.sblk = g->d_sblk;
            p.n_sblk = (int)sl.size();
        }
        std::vector<uint32_t> sm;
        for (int r = 0; r <= GW_FIXED_RANGE && !sblock.empty(); r++) {
            if (!used[r]) continue;
            p.smask_off[r] = (int)sm.size();
            const int D = 2 * r + 1, mw = mask_words(r);
            sm.resize(sm.size() + (size_t)HW * mw, 0u);
            for (int cell = 0; cell < HW; cell++) {
                const int cr = cell / cfg->cols, cc = cell % cfg->cols;
                uint32_t* dst = sm.data() + p.smask_off[r] + (size_t)cell * mw;
                for (int a : sblock) {
                    const int dr = cfg->agents[a].init_row - cr, dc = cfg->agents[a].init_col - cc;
                    if (dr < -r || dr > r || dc < -r || dc > r || (dr == 0 && dc == 0)) continue;
                    const uint32_t* src = lut.data() + p.shadow_off[r] + ((dr + r) * D + (dc + r)) * mw;
                    for (int w = 0; w < mw; w++) dst[w] |= src[w];
                }
            }
        }
        if (!sm.empty()) {
            HIPCHK(hipMalloc(&g->d_smask, sm.size() * 4));
            HIPCHK(hipMemcpy(g->d_smask, sm.data(), sm.size() * 4, hipMemcpyHostToDevice));
            p.smask = g->d_smask;
        }
    }
    // observers with different view ranges: their windows sit top-left in an
    // S x S slot; the blocking LUTs are re-laid out in slot geometry per range
    for (int l = 0; l < A; l++)
        if ((hs[l].kind & GW_K_GRID_OBSERVER) && !pac && hs[l].view_range != cfg->obs_range) p.hetero_view = 1;
    for (int r = 0; r <= GW_FIXED_RANGE; r++) { p.hshadow_off[r] = -1; p.hsmask_off[r] = -1; }
    if (p.hetero_view && wg) {
        set_err("observers with different view ranges run on the one-wave kernel only");
        return GW_E_UNSUPPORTED;
    }
    if (p.hetero_view && any_block && !big) {
        const int S = g->S, MWS = mask_words(cfg->obs_range), R = cfg->obs_range;
        bool used[GW_FIXED_RANGE + 1] = {};
        for (int l = 0; l < A; l++) if (hs[l].kind & GW_K_GRID_OBSERVER) used[hs[l].view_range] = true;
        // slot bits of the cells a blocker at (dr, dc) hides from a range-v window
        auto slot_shadow = [&](int v, int dr, int dc, uint32_t* out) {
            uint32_t b[16];
            host_shadow(v, dr, dc, b);
            const int D = 2 * v + 1;
            for (int k = 0; k < D * D; k++)
                if ((b[k >> 5] >> (k & 31)) & 1u) {
                    const int q = (k / D) * S + (k % D);
                    out[q >> 5] |= 1u << (q & 31);
                }
        };
        std::vector<uint32_t> hl, hm;
        std::vector<int> sblock;
        for (int a : statics) if (cfg->agents[a].kind & GW_K_BLOCKING) sblock.push_back(a);
        for (int v = 0; v <= R; v++) {
            if (!used[v]) continue;
            const int D = 2 * v + 1;
            p.hshadow_off[v] = (int)hl.size();
            hl.resize(hl.size() + (size_t)D * D * MWS, 0u);
            for (int dr = -v; dr <= v; dr++)
                for (int dc = -v; dc <= v; dc++)
                    slot_shadow(v, dr, dc, hl.data() + p.hshadow_off[v] + ((dr + v) * D + (dc + v)) * MWS);
            if (sblock.empty()) continue;
            p.hsmask_off[v] = (int)hm.size();
            hm.resize(hm.size() + (size_t)HW * MWS, 0u);
            for (int cell = 0; cell < HW; cell++) {
                const int cr = cell / cfg->cols, cc = cell % cfg->cols;
                for (int a : sblock) {
                    const int dr = cfg->agents[a].init_row - cr, dc = cfg->agents[a].init_col - cc;
                    if (dr < -v || dr > v || dc < -v || dc > v || (dr == 0 && dc == 0)) continue;
                    slot_shadow(v, dr, dc, hm.data() + p.hsmask_off[v] + (size_t)cell * MWS);
                }
            }
        }
        HIPCHK(hipMalloc(&g->d_hshadow, hl.size() * 4));
        HIPCHK(hipMemcpy(g->d_hshadow, hl.data(), hl.size() * 4, hipMemcpyHostToDevice));
        p.hshadow = g->d_hshadow;
        if (!hm.empty()) {
            HIPCHK(hipMalloc(&g->d_hsmask, hm.size() * 4));
            HIPCHK(hipMemcpy(g->d_hsmask, hm.data(), hm.size() * 4, hipMemcpyHostToDevice));
            p.hsmask = g->d_hsmask;
        }
    }
    p.pair_cap = (int)((work_bytes(HW, A, Sst, max_enc) - (size_t)A * Sst * ((Sst + 3) & ~3)) / 2);
    g->smem_step = smem_bytes(HW, A, Sst, max_enc, p.tbl_rows * p.pitch);
    if (pac) {
        // pac_carve: pb | clist | cp | pcell | ob
        const size_t pw = align16(4 * PAC_MAX_PWORDS) + 4 * WAVE +
                          align16(2 * (size_t)HW) + 64 * PAC_MAX_PWORDS +
                          align16((size_t)HW);
        // the Pacman program never places by draws (every entity starts at its
        // initial position): no placement scratch in its work area, so more
        // envs share a CU (8.2 KB -> 5.4 KB per env at pacman.txt's 21x21)
        g->smem_step = align16(GW_MT_N * 4) + align16((size_t)p.tbl_rows * p.pitch) +
                       align16((size_t)((HW + 3) / 4) * 4) + pw;
    }
    g->smem_reset = g->smem_step;
    if (wg) {
        // force_workgroup >= 2 asks for that many waves (the extra threads
        // share the table, observation store and crowded-draw work)
        p.nwv = (A + WAVE - 1) / WAVE;
        if (cfg->force_workgroup > p.nwv) p.nwv = cfg->force_workgroup;
        g->smem_step = g->smem_reset = wg_smem_bytes(HW, A, g->S, max_enc, p.tbl_rows * p.pitch, p.nwv);
        // the lanes that can ever observe (skip_done_obs stores only their rows:
        // config 4's 128 barriers are the first half of its lanes)
        p.obs_lo = A; p.obs_hi = 0;
        for (int l = 0; l < A; l++)
            if (hs[l].kind & GW_K_GRID_OBSERVER) { if (l < p.obs_lo) p.obs_lo = l; p.obs_hi = l + 1; }
        if (p.obs_hi == 0) p.obs_lo = 0;
        // moves run in parallel when every moving lane's encoding may share a
        // cell with every lane encoding (static cells are refused separately)
        uint32_t lane_encs = 0;
        for (int l = 0; l < A; l++) lane_encs |= 1u << hs[l].enc;
        p.par_moves = 1;
        for (int l = 0; l < A; l++)
            if ((hs[l].kind & GW_K_MOVING) && (p.overlap[hs[l].enc] & lane_encs) != lane_encs) p.par_moves = 0;
        // parallel placement needs every list length to follow from the
        // placement order: no two lanes that can share a cell at reset may
        // both remove it from one list (a removal would then not shorten it)
        const uint32_t all_encs = ((2u << max_enc) - 1u) & ~1u;
        auto rmv = [&](int enc) { return cfg->no_overlap_at_reset ? all_encs : (all_encs & ~p.overlap[enc]); };
        // (the sequential wave-0 form for every reset measured 4.22 vs 3.99 ms per
        // 100-step config-4 launch, profiles/r04/ab_wg_place_par.txt)
        p.place_par = 1;
        for (int a = 1; a <= max_enc; a++) {
            if (!((lane_encs >> a) & 1u)) continue;
            for (int b = 1; b <= max_enc; b++) {
                if (!((lane_encs >> b) & 1u)) continue;
                // b placed after a can land on a's cell iff b's list kept it
                if (!((rmv(a) >> b) & 1u) && (rmv(a) & rmv(b))) p.place_par = 0;
            }
        }
        for (int a = 0; a < A; a++)
            for (int b = a + 1; b < A; b++)
                if (hs[a].init_r >= 0 && hs[a].init_r == hs[b].init_r && hs[a].init_c == hs[b].init_c)
                    p.place_par = 0;                         // initial positions shared: sequential

    }
    if (g->smem_step > 160 * 1024) { set_err("LDS need %zu B > 160 KiB", g->smem_step); return GW_E_UNSUPPORTED; }
    if (pac) {
        p.obs_kind = cfg->obs_kind;
        for (int l = 0; l < A; l++) if (lanes[l] == cfg->pacman_agent) p.pacman = l;
        for (int i = 0; i < 4; i++) p.tunnel[i] = cfg->tunnel[i];
        for (int i = 0; i < 5; i++) p.prw[i] = cfg->pac_rewards[i];
        p.agent_lanes = 0;
        for (int l = 0; l < A; l++)
            if ((hs[l].kind & GW_K_OBSERVING) && (hs[l].kind & GW_K_ACTING)) p.agent_lanes |= 1ull << l;
        p.n_passive = (int)passive.size();
        p.pwords = (p.n_passive + 31) / 32;
        // the program's constant tables, each starting on 16 bytes and padded
        // to 16 (the kernel copies them to LDS with one 16-byte load per lane):
        // passive cells [n] i16 | cell -> passive [HW] i16 | per-cell counts
        // [ceil(HW/4)] u32; passive encodings [n] i8 (own allocation)
        const size_t n8 = ((size_t)p.n_passive + 7) & ~(size_t)7;        // i16s, 16 B
        const size_t hw8 = ((size_t)HW + 7) & ~(size_t)7;
        const size_t cw = (((size_t)HW + 3) / 4 + 3) & ~(size_t)3;       // u32s, 16 B
        std::vector<int16_t> pc(n8 + hw8 + 2 * cw, (int16_t)-1);
        std::vector<uint32_t> cnt(cw, 0u);
        std::vector<int8_t> pe((p.n_passive + 15) & ~15, 0);
        if (pe.empty()) pe.resize(16, 0);
        for (int k = 0; k < p.n_passive; k++) {
            const gw_agent_spec& s = cfg->agents[passive[k]];
            const int cell = s.init_row * cfg->cols + s.init_col;
            pc[k] = (int16_t)cell;
            pc[n8 + cell] = (int16_t)(k | (s.encoding << 8));   // food_at: index and encoding
            cnt[cell >> 2] += 1u << (8 * (cell & 3));
            pe[k] = (int8_t)s.encoding;
        }
        memcpy(pc.data() + n8 + hw8, cnt.data(), cw * 4);
        HIPCHK(hipMalloc(&g->d_passive, pc.size() * 2));
        HIPCHK(hipMemcpy(g->d_passive, pc.data(), pc.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMalloc(&g->d_passive_enc, pe.size()));
        HIPCHK(hipMemcpy(g->d_passive_enc, pe.data(), pe.size(), hipMemcpyHostToDevice));
        p.passive_cell = g->d_passive;
        p.cell_passive = g->d_passive + n8;
        p.passive_cnt = (const uint32_t*)(g->d_passive + n8 + hw8);
        p.passive_enc = g->d_passive_enc;
        const size_t pwn = (size_t)n_envs * (p.pwords > 0 ? p.pwords : 1);
        HIPCHK(hipMalloc(&p.pbits, pwn * 4));
        HIPCHK(hipMemset(p.pbits, 0, pwn * 4));
        HIPCHK(hipMalloc(&p.cyc, (size_t)n_envs * 4));
        HIPCHK(hipMemset(p.cyc, 0xff, (size_t)n_envs * 4));      // -1: no turn yet
        HIPCHK(hipFuncSetAttribute((const void*)pac_kernel<-1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)g->smem_step));
        HIPCHK(hipFuncSetAttribute((const void*)pac_kernel<PAC_STEP_TURN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)g->smem_step));
        HIPCHK(hipFuncSetAttribute((const void*)pac_kernel<PAC_STEP_ALL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)g->smem_step));
    }
    HIPCHK(hipMalloc(&p.racc, EA * sizeof(double)));
    HIPCHK(hipMemset(p.racc, 0, EA * sizeof(double)));
    if (wg) {
        HIPCHK(set_part_attrs(g->S, PK_WG_STEP, PK_WG_RESET, g->smem_step, g->smem_step));
        HIPCHK(set_part_attrs(g->S, PK_WG_COMP, PK_WG_COMP, g->smem_step, g->smem_step));
    }
    else if (!pac) HIPCHK(set_part_attrs(g->S, PK_STEP, PK_RESET, g->smem_step, g->smem_reset));
    if (!wg && !pac) HIPCHK(set_part_attrs(g->S, PK_COMP, PK_COMP, g->smem_step, g->smem_step));
    bool any_ammo = false;
    for (int l = 0; l < A; l++) any_ammo |= (hs[l].kind & GW_K_AMMO) != 0;
    g->step_tb = !wg && !pac && !big && p.sim_kind == GW_SIM_TEAM_BATTLE && !p.blockers && !p.lane_blockers &&
                 !p.hetero_view && !any_ammo;
    if (g->step_tb) HIPCHK(set_part_attrs(g->S, PK_STEP_TB, PK_STEP_TB, g->smem_step, g->smem_step));
    // MazeNavigation with the navigator and the target as its only lanes
    // (walls static), both at initial positions that never fail to place, no
    // health, no blocking lane, the target a plain entity: one lane per env
    // (gw_lane.inc)
    {
        // (no AmmoAgent: the lane kernel keeps no ammo, whose reset the one-wave
        // kernel does as AmmoState.reset)
        bool able = maze && A == 2 && !pac && !wg && !big && !p.lane_blockers && !p.hetero_view && p.nav >= 0 &&
                    p.target >= 0 && p.nav != p.target && !any_ammo;
        for (int l = 0; able && l < A; l++) {
            if (hs[l].init_r < 0 || hs[l].init_c < 0 || (hs[l].kind & GW_K_HEALTH)) able = false;
            if (l == p.target && (hs[l].kind & dynamic_kinds)) able = false;
        }
        if (able && hs[0].init_r == hs[1].init_r && hs[0].init_c == hs[1].init_c &&
            !((hs[1].ov >> hs[0].enc) & 1u))
            able = false;                                   // the reset's Grid.place would fail
        // its LDS: padded template + static-blocker masks at the view range +
        // static-cell bits (lane_step_kernel's carve-up)
        const int S = g->S, R = S / 2, MWS = (S * S + 31) / 32;
        const size_t nsm = (p.blockers && R <= GW_FIXED_RANGE && p.smask_off[R] >= 0) ? (size_t)HW * MWS : 0;
        g->smem_lane = 16 * (size_t)((p.tbl_rows * p.pitch + 15) / 16) + 4 * ((nsm + 3) & ~(size_t)3) +
                       (p.static_bits ? 4 * (size_t)((HW + 31) / 32) : 0);
        const size_t static_lds = 4 * GW_MT_N;
        if (g->smem_lane + static_lds > 64 * 1024) able = false;
        // its per-step slabs are addressed by 32-bit buffer offsets
        if ((size_t)n_envs * A * S * S * 4 >= ((size_t)1 << 31)) able = false;
        if (cfg->env_per_lane > 0 && !able) {
            set_err("env_per_lane: the one-lane-per-env kernel runs MazeNavigation with the navigator and "
                    "the target at initial positions as its only dynamic entities");
            return GW_E_UNSUPPORTED;
        }
        g->lane_envs = able && cfg->env_per_lane >= 0;
        g->lane_envs_config = g->lane_envs;
        if (g->lane_envs) HIPCHK(set_part_attrs(g->S, PK_STEP_LANE, PK_STEP_LANE_NS, g->smem_lane, g->smem_lane));
    }
    *out = g;
    return GW_OK;
}

gw_status gw_destroy(gw_handle g)
{
    if (!g) return GW_E_INVALID;
    (void)hipFree(g->base.pos); (void)hipFree(g->base.health); (void)hipFree(g->base.flags);
    (void)hipFree(g->base.seq); (void)hipFree(g->base.mt); (void)hipFree(g->base.steps);
    (void)hipFree(g->base.ammo);
    (void)hipFree(g->d_spec); (void)hipFree(g->d_tmpl); (void)hipFree(g->d_free);
    (void)hipFree(g->d_static_bits); (void)hipFree(g->d_shadow); (void)hipFree(g->d_smask);
    (void)hipFree(g->base.racc); (void)hipFree(g->base.pbits); (void)hipFree(g->base.cyc);
    (void)hipFree(g->d_passive); (void)hipFree(g->d_passive_enc);
    (void)hipFree(g->d_hshadow); (void)hipFree(g->d_hsmask); (void)hipFree(g->d_sblk);
    (void)hipFree(g->d_place_order); (void)hipFree(g->d_act_order);
    delete g;
    return GW_OK;
}

int32_t gw_num_envs(gw_handle g) { return g ? g->E : 0; }
int32_t gw_obs_side(gw_handle g) { return g ? g->S : 0; }
int32_t gw_num_lanes(gw_handle g) { return g ? g->A : 0; }
int32_t gw_env_kernel(gw_handle g)
{
    return !g ? -1 : g->pacman ? GW_KERNEL_PACMAN : g->wg ? GW_KERNEL_WORKGROUP
                   : g->lane_envs ? GW_KERNEL_LANE : GW_KERNEL_WAVE;
}
int32_t gw_act_dim(gw_handle g) { return g ? g->base.act_dim : 0; }

gw_status gw_step_occupancy(gw_handle g, int32_t* blocks_per_cu, int32_t* block_threads, int64_t* lds_bytes)
{
    EvClear ec{g};
    if (!g || !blocks_per_cu) return GW_E_INVALID;
    int nblk = 0;
    unsigned block = WAVE;
    size_t smem = g->smem_step;
    if (g->pacman) {
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nblk, (const void*)pac_kernel<PAC_STEP_ALL>,
                                                            (int)block, smem));
    } else {
        const int pi = part_index(g->S);
        if (pi < 0) return GW_E_INVALID;
        int kind = g->wg ? PK_WG_STEP : (g->step_tb ? PK_STEP_TB : PK_STEP);
        if (g->lane_envs) { kind = PK_STEP_LANE_NS; smem = g->smem_lane; }
        if (g->wg) block = WAVE * g->base.nwv;
        HIPCHK(k_part_occ[pi](kind, block, smem, &nblk));
    }
    *blocks_per_cu = nblk;
    if (block_threads) *block_threads = (int32_t)block;
    if (lds_bytes) *lds_bytes = (int64_t)smem;
    return GW_OK;
}

gw_status gw_set_action_order(gw_handle g, const int32_t* lane_order, int32_t n)
{
    EvClear ec{g};
    if (!g) return GW_E_INVALID;
    if (n == 0 || !lane_order) { g->base.act_order = nullptr; g->base.act_rank = nullptr; return GW_OK; }
    if (n != g->E * g->A) { set_err("action order: %d entries, expected E*A = %d", n, g->E * g->A); return GW_E_INVALID; }
    const int sk = g->base.sim_kind;
    if (g->lane_envs || (g->wg && sk != GW_SIM_REACH_TARGET) ||
        (sk != GW_SIM_TEAM_BATTLE && sk != GW_SIM_REACH_TARGET && sk != GW_SIM_TRAFFIC &&
         sk != GW_SIM_PACMAN)) {
        set_err("randomize_action_input runs with the TeamBattle, ReachTheTarget, TrafficCorridor "
                "and Pacman programs (the workgroup-per-env kernel: ReachTheTarget only)");
        return GW_E_UNSUPPORTED;
    }
    std::vector<int32_t> both((size_t)2 * g->E * g->A);
    for (int e = 0; e < g->E; e++) {
        std::vector<uint8_t> seen(g->A, 0);
        for (int k = 0; k < g->A; k++) {
            const int32_t a = lane_order[(size_t)e * g->A + k];
            if (a < 0 || a >= g->A || seen[a]) { set_err("action order of env %d is not a permutation", e); return GW_E_INVALID; }
            seen[a] = 1;
            both[(size_t)e * g->A + k] = a;
            both[(size_t)g->E * g->A + (size_t)e * g->A + a] = k;
        }
    }
    if (!g->d_act_order) HIPCHK(hipMalloc(&g->d_act_order, both.size() * sizeof(int32_t)));
    // launches already queued on any stream may still read the old order
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(g->d_act_order, both.data(), both.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    g->base.act_order = g->d_act_order;
    g->base.act_rank = g->d_act_order + (size_t)g->E * g->A;
    return GW_OK;
}

gw_status gw_set_placement_order(gw_handle g, const int32_t* lane_order, int32_t n)
{
    EvClear ec{g};
    if (!g) return GW_E_INVALID;
    if (n == 0 || !lane_order) {
        g->base.place_order = nullptr;
        g->lane_envs = g->lane_envs_config;      // agents-dict order again
        return GW_OK;
    }
    if (n != g->E * g->A) { set_err("placement order: %d entries, expected E*A = %d", n, g->E * g->A); return GW_E_INVALID; }
    if (g->wg || g->pacman) {
        set_err("randomize_placement_order runs on the one-wave kernel only");
        return GW_E_UNSUPPORTED;
    }
    for (int e = 0; e < g->E; e++) {                 // a permutation of the lanes per env
        std::vector<uint8_t> seen(g->A, 0);
        for (int k = 0; k < g->A; k++) {
            const int32_t a = lane_order[(size_t)e * g->A + k];
            if (a < 0 || a >= g->A || seen[a]) { set_err("placement order of env %d is not a permutation", e); return GW_E_INVALID; }
            seen[a] = 1;
        }
    }
    if (!g->d_place_order) HIPCHK(hipMalloc(&g->d_place_order, (size_t)g->E * g->A * sizeof(int32_t)));
    // launches already queued on any stream may still read the old order
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(g->d_place_order, lane_order, (size_t)g->E * g->A * sizeof(int32_t), hipMemcpyHostToDevice));
    g->base.place_order = g->d_place_order;
    // the one-lane-per-env maze kernel places in lane order: use the one-wave kernel
    g->lane_envs = false;
    return GW_OK;
}

gw_status gw_lane_entities(gw_handle g, int32_t* out)
{
    if (!g || !out) return GW_E_INVALID;
    for (int i = 0; i < g->A; i++) out[i] = g->lane_ent[i];
    return GW_OK;
}

gw_status gw_seed(gw_handle g, const uint32_t* seeds, void* stream)
{
    EvClear ec{g};
    if (!g || !seeds) return GW_E_INVALID;
    hipLaunchKernelGGL(seed_kernel, dim3((g->E + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       g->base.mt, seeds, g->E);
    HIPCHK(hipGetLastError());
    return GW_OK;
}

gw_status gw_reset(gw_handle g, const uint8_t* mask, const uint8_t* all_done, int32_t horizon,
                   int32_t* obs, uint32_t* err_flags, void* stream)
{
    EvClear ec{g};
    if (!g || !obs) return GW_E_INVALID;
    Params p = g->base;
    p.mask = mask; p.prev_all_done = all_done; p.horizon = horizon; p.obs = obs; p.err = err_flags;
    HIPCHK(do_reset(g, p, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_step(gw_handle g, const int32_t* actions, int32_t* obs, double* reward,
                  uint8_t* done, uint8_t* all_done, uint64_t* acting, uint32_t* err_flags, void* stream)
{
    EvClear ec{g};
    if (!g || !actions || !obs || !reward || !done || !all_done) return GW_E_INVALID;
    Params p = g->base;
    p.actions = actions; p.obs = obs; p.reward = reward; p.done = done; p.all_done = all_done;
    p.acting = acting;
    p.err = err_flags;
    p.autoreset = 0;
    p.nsteps = 1; p.ad_in = all_done;
    HIPCHK(do_step(g, p, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_step_autoreset(gw_handle g, const int32_t* actions, int32_t* obs, double* reward,
                            uint8_t* done, uint8_t* all_done, uint64_t* acting, int32_t horizon,
                            uint32_t* err_flags, void* stream)
{
    EvClear ec{g};
    if (!g || !actions || !obs || !reward || !done || !all_done) return GW_E_INVALID;
    Params p = g->base;
    p.actions = actions; p.obs = obs; p.reward = reward; p.done = done; p.all_done = all_done;
    p.acting = acting;
    p.autoreset = 1;
    p.horizon = horizon;
    p.err = err_flags;
    p.nsteps = 1; p.ad_in = all_done;
    HIPCHK(do_step(g, p, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_step_autoreset_next(gw_handle g, const int32_t* actions, int32_t* obs, double* reward,
                                 uint8_t* done, uint8_t* all_done, uint64_t* acting, int32_t horizon,
                                 uint32_t* err_flags, void* stream)
{
    EvClear ec{g};
    if (!g || !actions || !obs || !reward || !done || !all_done) return GW_E_INVALID;
    Params p = g->base;
    p.actions = actions; p.obs = obs; p.reward = reward; p.done = done; p.all_done = all_done;
    p.acting = acting;
    p.autoreset = 2;
    p.horizon = horizon;
    p.err = err_flags;
    p.nsteps = 1; p.ad_in = all_done;
    HIPCHK(do_step(g, p, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_get_state(gw_handle g, int32_t* pos, double* health, uint8_t* flags, uint32_t* seq,
                       uint32_t* mt, int32_t* steps, void* stream)
{
    EvClear ec{g};
    if (!g) return GW_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    const size_t EA = (size_t)g->E * g->A;
    if (pos) HIPCHK(hipMemcpyAsync(pos, g->base.pos, EA * sizeof(int2), hipMemcpyDeviceToDevice, st));
    if (health) HIPCHK(hipMemcpyAsync(health, g->base.health, EA * 8, hipMemcpyDeviceToDevice, st));
    if (flags) {
        HIPCHK(hipMemcpyAsync(flags, g->base.flags, EA, hipMemcpyDeviceToDevice, st));
        hipLaunchKernelGGL(clear_obs_m2_kernel, dim3((unsigned)((EA + 255) / 256)), dim3(256), 0, st, flags, EA);
        HIPCHK(hipGetLastError());
    }
    if (seq) HIPCHK(hipMemcpyAsync(seq, g->base.seq, EA * 4, hipMemcpyDeviceToDevice, st));
    if (mt) HIPCHK(hipMemcpyAsync(mt, g->base.mt, (size_t)g->E * GW_MT_STRIDE * 4, hipMemcpyDeviceToDevice, st));
    if (steps) HIPCHK(hipMemcpyAsync(steps, g->base.steps, (size_t)g->E * 4, hipMemcpyDeviceToDevice, st));
    return GW_OK;
}

gw_status gw_set_state(gw_handle g, const int32_t* pos, const double* health, const uint8_t* flags,
                       const uint32_t* seq, const uint32_t* mt, const int32_t* steps, void* stream)
{
    EvClear ec{g};
    if (!g) return GW_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    const size_t EA = (size_t)g->E * g->A;
    if (pos) HIPCHK(hipMemcpyAsync(g->base.pos, pos, EA * sizeof(int2), hipMemcpyDeviceToDevice, st));
    if (health) HIPCHK(hipMemcpyAsync(g->base.health, health, EA * 8, hipMemcpyDeviceToDevice, st));
    if (flags) {
        HIPCHK(hipMemcpyAsync(g->base.flags, flags, EA, hipMemcpyDeviceToDevice, st));
        hipLaunchKernelGGL(clear_obs_m2_kernel, dim3((unsigned)((EA + 255) / 256)), dim3(256), 0, st,
                           g->base.flags, EA);
        HIPCHK(hipGetLastError());
    }
    if (seq) HIPCHK(hipMemcpyAsync(g->base.seq, seq, EA * 4, hipMemcpyDeviceToDevice, st));
    if (mt) {
        HIPCHK(hipMemcpyAsync(g->base.mt, mt, (size_t)g->E * GW_MT_STRIDE * 4, hipMemcpyDeviceToDevice, st));
        hipLaunchKernelGGL(invalidate_cache_kernel, dim3((g->E + 255) / 256), dim3(256), 0, st, g->base.mt, g->E);
        HIPCHK(hipGetLastError());
    }
    if (steps) HIPCHK(hipMemcpyAsync(g->base.steps, steps, (size_t)g->E * 4, hipMemcpyDeviceToDevice, st));
    return GW_OK;
}

gw_status gw_get_ammo(gw_handle g, int32_t* ammo, void* stream)
{
    EvClear ec{g};
    if (!g || !ammo) return GW_E_INVALID;
    HIPCHK(hipMemcpyAsync(ammo, g->base.ammo, (size_t)g->E * g->A * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_set_ammo(gw_handle g, const int32_t* ammo, void* stream)
{
    EvClear ec{g};
    if (!g || !ammo) return GW_E_INVALID;
    HIPCHK(hipMemcpyAsync(g->base.ammo, ammo, (size_t)g->E * g->A * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_obs_shape(gw_handle g, int32_t* rows, int32_t* cols)
{
    if (!g || !rows || !cols) return GW_E_INVALID;
    if (g->base.obs_kind == GW_OBS_ABSOLUTE) { *rows = g->H; *cols = g->W; }
    else { *rows = g->S; *cols = g->S; }
    return GW_OK;
}

int32_t gw_num_passive(gw_handle g) { return g ? g->base.n_passive : 0; }

gw_status gw_turn_reset(gw_handle g, const uint8_t* mask, int32_t* obs, uint8_t* returned,
                        int32_t* turn, uint32_t* err_flags, void* stream)
{
    EvClear ec{g};
    if (!g || !obs || !returned || !turn) return GW_E_INVALID;
    if (!g->pacman) { set_err("turn-based protocol: Pacman program only"); return GW_E_UNSUPPORTED; }
    Params p = g->base;
    p.mask = mask; p.obs = obs; p.returned = returned; p.turn = turn; p.err = err_flags;
    p.mode = PAC_RESET_TURN;
    if (!mask) {                     // every env: a mask-less reset of all
        p.prev_all_done = nullptr; p.horizon = 0;
    }
    HIPCHK(launch_pac(g, p, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_turn_step(gw_handle g, const int32_t* actions, int32_t* obs, double* reward,
                       uint8_t* done, uint8_t* all_done, uint8_t* returned, int32_t* turn,
                       uint64_t* acting, int32_t horizon, uint32_t* err_flags, void* stream)
{
    EvClear ec{g};
    if (!g || !actions || !obs || !reward || !done || !all_done || !returned || !turn) return GW_E_INVALID;
    if (!g->pacman) { set_err("turn-based protocol: Pacman program only"); return GW_E_UNSUPPORTED; }
    Params p = g->base;
    p.actions = actions; p.obs = obs; p.reward = reward; p.done = done; p.all_done = all_done;
    p.returned = returned; p.turn = turn; p.acting = acting; p.horizon = horizon; p.err = err_flags;
    p.mode = PAC_STEP_TURN;
    p.nsteps = 1; p.ad_in = all_done;       // all_done is in/out
    HIPCHK(launch_pac(g, p, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_turn_rollout(gw_handle g, int32_t n_steps, const int32_t* actions, int32_t* obs, double* reward,
                          uint8_t* done, uint8_t* all_done, uint8_t* all_done_in, uint8_t* returned,
                          int32_t* turn, uint64_t* acting, int32_t horizon, uint32_t* err_flags, void* stream)
{
    EvClear ec{g};
    if (!g || n_steps <= 0 || !actions || !obs || !reward || !done || !all_done || !returned || !turn)
        return GW_E_INVALID;
    if (!g->pacman) { set_err("turn-based protocol: Pacman program only"); return GW_E_UNSUPPORTED; }
    Params p = g->base;
    p.actions = actions; p.obs = obs; p.reward = reward; p.done = done; p.all_done = all_done;
    p.returned = returned; p.turn = turn; p.acting = acting; p.horizon = horizon; p.err = err_flags;
    p.mode = PAC_STEP_TURN;
    p.nsteps = n_steps; p.ad_in = all_done_in; p.ad_out = all_done_in;
    HIPCHK(launch_pac(g, p, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_sim_reset(gw_handle g, const uint8_t* mask, uint32_t* err_flags, void* stream)
{
    EvClear ec{g};
    if (!g) return GW_E_INVALID;
    if (!g->pacman) { set_err("simulation-only protocol: Pacman program only"); return GW_E_UNSUPPORTED; }
    Params p = g->base;
    p.mask = mask; p.err = err_flags; p.mode = PAC_RESET_SIM;
    HIPCHK(launch_pac(g, p, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_sim_step(gw_handle g, const int32_t* actions, double* reward, uint8_t* done,
                      uint8_t* all_done, uint32_t* err_flags, void* stream)
{
    EvClear ec{g};
    if (!g || !actions || !reward || !done || !all_done) return GW_E_INVALID;
    if (!g->pacman) { set_err("simulation-only protocol: Pacman program only"); return GW_E_UNSUPPORTED; }
    Params p = g->base;
    p.actions = actions; p.reward = reward; p.done = done; p.all_done = all_done; p.err = err_flags;
    p.mode = PAC_STEP_SIM;
    HIPCHK(launch_pac(g, p, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_observe(gw_handle g, int32_t lane, int32_t* obs, void* stream)
{
    EvClear ec{g};
    if (!g || !obs || lane < 0 || lane >= g->A) return GW_E_INVALID;
    if (!g->pacman) { set_err("on-demand observation: Pacman program only"); return GW_E_UNSUPPORTED; }
    Params p = g->base;
    p.obs = obs; p.obs_lane = lane; p.mode = PAC_OBSERVE;
    HIPCHK(launch_pac(g, p, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_get_aux_state(gw_handle g, double* racc, uint32_t* passive_bits, int32_t* turn_pos,
                           void* stream)
{
    EvClear ec{g};
    if (!g) return GW_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    const size_t EA = (size_t)g->E * g->A;
    if (racc) HIPCHK(hipMemcpyAsync(racc, g->base.racc, EA * 8, hipMemcpyDeviceToDevice, st));
    if (passive_bits && g->base.pwords)
        HIPCHK(hipMemcpyAsync(passive_bits, g->base.pbits, (size_t)g->E * g->base.pwords * 4, hipMemcpyDeviceToDevice, st));
    if (turn_pos && g->base.cyc) HIPCHK(hipMemcpyAsync(turn_pos, g->base.cyc, (size_t)g->E * 4, hipMemcpyDeviceToDevice, st));
    return GW_OK;
}

gw_status gw_set_aux_state(gw_handle g, const double* racc, const uint32_t* passive_bits,
                           const int32_t* turn_pos, void* stream)
{
    EvClear ec{g};
    if (!g) return GW_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    const size_t EA = (size_t)g->E * g->A;
    if (racc) HIPCHK(hipMemcpyAsync(g->base.racc, racc, EA * 8, hipMemcpyDeviceToDevice, st));
    if (passive_bits && g->base.pwords)
        HIPCHK(hipMemcpyAsync(g->base.pbits, passive_bits, (size_t)g->E * g->base.pwords * 4, hipMemcpyDeviceToDevice, st));
    if (turn_pos && g->base.cyc) HIPCHK(hipMemcpyAsync(g->base.cyc, turn_pos, (size_t)g->E * 4, hipMemcpyDeviceToDevice, st));
    return GW_OK;
}

// diagnostic hook (not in the public header): violation record for -DGW_CHECKS builds
gw_status gw_debug_set_checks(gw_handle g, uint32_t* dbg)
{
    if (!g) return GW_E_INVALID;
    g->base.dbg = dbg;
    return GW_OK;
}

// diagnostic hook (not in the public header): stamps buffer for -DGW_STAMPS builds
gw_status gw_debug_set_stamps(gw_handle g, uint64_t* stamps)
{
    if (!g) return GW_E_INVALID;
    g->base.stamps = stamps;
    return GW_OK;
}

gw_status gw_random_actions(gw_handle g, uint64_t key, uint32_t step, uint32_t env_offset,
                            int32_t* actions, void* stream)
{
    EvClear ec{g};
    if (!g || !actions) return GW_E_INVALID;
    const dim3 grid = g->A <= WAVE ? dim3((g->E + 15) / 16) : dim3((unsigned)(((size_t)g->E * g->A + 255) / 256));
    hipLaunchKernelGGL(random_actions_kernel, grid, dim3(g->A <= WAVE ? 16 * WAVE : 256), 0,
                       (hipStream_t)stream, g->policy, g->E, g->A, key, step, env_offset, actions,
                       g->base.act_dim, g->pacman ? RA_CROSS : g->base.attack_kind);
    HIPCHK(hipGetLastError());
    return GW_OK;
}

gw_status gw_rollout_step(gw_handle g, uint64_t key, uint32_t step, uint32_t env_offset,
                          int32_t* actions, int32_t* obs, double* reward, uint8_t* done,
                          uint8_t* all_done, uint64_t* acting, int32_t horizon, int32_t autoreset,
                          uint32_t* err_flags, void* stream)
{
    EvClear ec{g};
    if (!g || !actions || !obs || !reward || !done || !all_done || autoreset < 0 || autoreset > 2)
        return GW_E_INVALID;
    // the armed launch events belong to the step, not to the action kernel
    const hipEvent_t ev0 = g->ev0, ev1 = g->ev1;
    const gw_status s = gw_random_actions(g, key, step, env_offset, actions, stream);
    if (s != GW_OK) return s;
    g->ev0 = ev0; g->ev1 = ev1;
    Params p = g->base;
    p.actions = actions; p.obs = obs; p.reward = reward; p.done = done; p.all_done = all_done;
    p.acting = acting; p.autoreset = autoreset; p.horizon = horizon; p.err = err_flags;
    p.nsteps = 1; p.ad_in = all_done;
    HIPCHK(do_step(g, p, (hipStream_t)stream));
    return GW_OK;
}

static gw_status maze_launch(gw_engine* g, int mode, const int32_t* args, const int32_t* start, int8_t* maze,
                             int32_t* result, uint32_t* err_flags, hipStream_t st)
{
    if (g->H * g->W > GW_MAX_CELLS || g->H < 1 || g->W < 1) return GW_E_INVALID;
    MazeCall m;
    m.mode = mode; m.start = start; m.maze_out = maze;
    m.T = maze_table_slots(g->H, g->W);
    const size_t smem = maze_smem_bytes(g->H, g->W, m.T);
    if (smem > 160 * 1024) { set_err("maze: %zu B of LDS per env", smem); return GW_E_UNSUPPORTED; }
    // per call: the attribute belongs to the current device
    if (smem > 64 * 1024)
        HIPCHK(hipFuncSetAttribute((const void*)maze_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)smem));
    Params p = g->base;
    p.actions = args; p.comp_out = result; p.err = err_flags;
    hipLaunchKernelGGL(maze_kernel, dim3(g->E), dim3(WAVE), smem, st, p, m);
    HIPCHK(hipGetLastError());
    return GW_OK;
}

gw_status gw_generate_maze(gw_handle g, const int32_t* start, int8_t* maze, void* stream)
{
    EvClear ec{g};
    if (!g || !maze) return GW_E_INVALID;
    if (g->pacman) { set_err("generate_maze: not on a Pacman handle"); return GW_E_UNSUPPORTED; }
    return maze_launch(g, 0, nullptr, start, maze, nullptr, nullptr, (hipStream_t)stream);
}

gw_status gw_component(gw_handle g, int32_t op, int32_t lane, const int32_t* args, int32_t* result,
                       int32_t* obs, uint32_t* err_flags, void* stream)
{
    EvClear ec{g};
    if (!g || op < GW_OP_POSITION_RESET || op > GW_OP_OBSERVE_ABS) return GW_E_INVALID;
    if (g->pacman) {
        set_err("component operations run on the one-wave and workgroup engines (not the Pacman kernel)");
        return GW_E_UNSUPPORTED;
    }
    if (op == GW_OP_MAZE_RESET) {
        if (g->wg) { set_err("MazePlacementState runs on the one-wave engine (at most 64 entities)"); return GW_E_UNSUPPORTED; }
        if (!args || g->base.act_dim < 3) return GW_E_INVALID;
        if (g->n_ent != g->A) {
            set_err("MazePlacementState places every entity: the handle must hold no static entities (all_lanes)");
            return GW_E_UNSUPPORTED;
        }
        return maze_launch(g, 1, args, nullptr, nullptr, result, err_flags, (hipStream_t)stream);
    }
    const bool moves = op == GW_OP_MOVE || op == GW_OP_CROSS_MOVE || op == GW_OP_DRIFT_MOVE;
    const bool needs_lane = moves || op == GW_OP_ATTACK || op == GW_OP_OBSERVE || op == GW_OP_OBSERVE_ABS;
    if (needs_lane && (lane < 0 || lane >= g->A)) { set_err("lane %d outside 0..%d", lane, g->A - 1); return GW_E_INVALID; }
    if ((moves || op == GW_OP_ATTACK) && !args) return GW_E_INVALID;
    if ((op == GW_OP_ATTACK || op == GW_OP_DRIFT_MOVE) && g->base.act_dim < 3) return GW_E_INVALID;
    if ((op == GW_OP_OBSERVE || op == GW_OP_OBSERVE_ABS) && !obs) return GW_E_INVALID;
    if (op == GW_OP_ORIENT_RESET && !result) return GW_E_INVALID;
    Params p = g->base;
    p.mode = op; p.obs_lane = lane; p.actions = args; p.comp_out = result; p.obs = obs; p.err = err_flags;
    p.nsteps = 1;
    HIPCHK(part_launch(g, g->wg ? PK_WG_COMP : PK_COMP, g->smem_step, p, (hipStream_t)stream));
    return GW_OK;
}

gw_status gw_rollout(gw_handle g, int32_t n_steps, const int32_t* actions, int32_t* obs, double* reward,
                     uint8_t* done, uint8_t* all_done, uint8_t* all_done_in, uint64_t* acting,
                     int32_t horizon, int32_t autoreset, int32_t skip_done_obs, uint32_t* err_flags,
                     void* stream)
{
    EvClear ec{g};
    if (!g || n_steps <= 0 || !actions || !obs || !reward || !done || !all_done ||
        autoreset < 1 || autoreset > 2)
        return GW_E_INVALID;
    hipStream_t st = (hipStream_t)stream;
    Params p = g->base;
    p.acting = acting; p.autoreset = autoreset; p.horizon = horizon; p.err = err_flags;
    p.persistent_obs = 0;                  // every step has its own obs slab
    // one launch: each env runs its n_steps back to back (step_kernel,
    // lane_step_kernel, wg_step_kernel, pac_kernel)
    p.actions = actions; p.obs = obs; p.reward = reward; p.done = done; p.all_done = all_done;
    p.nsteps = n_steps; p.ad_in = all_done_in; p.skip_done_obs = skip_done_obs != 0;
    p.ad_out = all_done_in;                // each env's wave reads it first, writes it last
    HIPCHK(do_step(g, p, st));
    return GW_OK;
}

gw_status gw_set_launch_events(gw_handle g, void* start_event, void* stop_event)
{
    if (!g || (start_event == nullptr) != (stop_event == nullptr)) return GW_E_INVALID;
    g->ev0 = (hipEvent_t)start_event;
    g->ev1 = (hipEvent_t)stop_event;
    return GW_OK;
}

}  // extern "C"
#endif  // GW_PART_S
