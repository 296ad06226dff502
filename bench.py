"""Benchmark: agent-steps/s of random-policy TeamBattle rollouts on MI355X.

Workload (BASELINE.json configs[2], the metric's config): TeamBattle 32x32,
64 BattleAgents in 2 teams, 4096 envs per GPU (weak scaling: N GPUs run
N x 4096 envs, sharded by global env id, no data-path collective), horizon
200 with on-device auto-reset.  One timed "step" = random-policy actions
(Philox kernel) + one fused AllStepManager.step launch for every env.

Auto-reset (--autoreset): 'next_step' (default; gymnasium NEXT_STEP, the
batched form of RLlib calling reset() after __all__: an env whose episode
ended is reset by the next launch, which counts no agent-steps for it) or
'same_step' (the reset observation is returned by the terminal step's
launch).  Both run every reset; the line reports the chosen mode and the
other one under "other_autoreset".

Metric: agent-steps/s = sum over env-steps of the acting (not-done) agents,
the reference's len(action_dict), over all ranks / the max
wall time over ranks.  The engine counts acting agents on device.

Usage: python bench.py [--gpus N --steps K --warmup W]
       N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = json.load(open(os.path.join(ROOT, 'BASELINE.json')))['metric']
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def team_battle_sim(rows=32, cols=32, n_agents=64, n_teams=2):
    from abmarl_amd.examples import BattleAgent, TeamBattleSim
    agents = {f'agent{i}': BattleAgent(id=f'agent{i}', encoding=i % n_teams + 1)
              for i in range(n_agents)}
    return TeamBattleSim.build_sim(
        rows, cols, agents=agents,
        overlapping={t: {t} for t in range(1, n_teams + 1)},
        attack_mapping={t: {u for u in range(1, n_teams + 1) if u != t}
                        for t in range(1, n_teams + 1)},
        states={'PositionState', 'HealthState'},
        observers={'PositionCenteredEncodingObserver'},
        dones={'OneTeamRemainingDone'})


def maze_sim():
    """BASELINE config 2: MazeNavigation 16x16 (generated maze, blocking walls)."""
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    from tests.cases import load_golden, build_maze
    return build_maze(load_golden('maze_16')['case'])


def pacman_sim():
    """BASELINE config 5: pacman.txt with four baddies (TurnBasedManager)."""
    from abmarl_amd.examples.pacman import build_pacman
    return build_pacman()


def rtt_sim():
    """BASELINE config 4: ReachTheTarget 64x64, 128 barriers + 127 runners +
    the target (256 entities, the workgroup-per-env kernel)."""
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    from tests.cases import build_rtt, RTT_CONFIG4
    return build_rtt(dict(RTT_CONFIG4))


def pacman_turn_bytes(E, A, HW, pwords):
    """Algorithmic HBM bytes of one turn-based Pacman launch: actions read
    (move + present, 8 B per lane), ONE lane's absolute observation 4*HW,
    per lane reward 8 + done 1 + returned 1, state read+write 2*(pos 8 +
    seq 4 + health 8 + flags 1 + reward accumulator 8) per lane, food bits
    2*4*pwords, per env all_done 1 + turn 4 + cycle 2*4 + steps 2*4 +
    acting 2*8 + RNG pos/counter 2*8."""
    return E * (A * (8 + 8 + 1 + 1 + 2 * 29) + 4 * HW + 8 * pwords + 1 + 4 + 8 + 8 + 16 + 16)


def step_bytes(E, A, S):
    """Algorithmic HBM bytes of one step launch:
    per entity slot: actions 12 + obs 4*S*S + reward 8 + done 1 +
    state read+write 2*(pos 8 + seq 4 + health 8 + flags 1); per env:
    __all__ 1 + steps 2*4 + acting 2*8 + RNG pos/counter 2*8."""
    per_slot = 12 + 4 * S * S + 8 + 1 + 2 * (8 + 4 + 8 + 1)
    per_env = 1 + 8 + 16 + 16
    return E * (A * per_slot + per_env)


def rtt_step_bytes(E, A, S, act_dim):
    """step_bytes with the SelectiveAttackActor's wider action rows
    (4 * act_dim B per entity slot instead of 12)."""
    return step_bytes(E, A, S) + E * A * (4 * act_dim - 12)


def cpu_baseline(cc, seconds=10.0, envs=512, horizon=200, mode='next_step'):
    """The oracle (C port of the reference step, OpenMP over envs) on this
    host's cores, bounded to ~`seconds` of work on a sample of the workload,
    with the same auto-reset flow as the GPU line."""
    from oracle.oracle import Oracle, lib
    threads = int(os.environ.get('OMP_NUM_THREADS', '0')) or min(16, os.cpu_count() or 1)
    lib().gwo_set_threads(threads)
    o = Oracle(cc, envs)
    from abmarl_amd.engine import env_seeds
    o.seed(env_seeds(envs))
    E, A, S = envs, cc.n_agents, cc.obs_side
    obs = o.new_obs()
    rew = np.zeros((E, A)); done = np.zeros((E, A), np.uint8); ad = np.zeros(E, np.uint8)
    acting = np.zeros(E, np.uint64)
    o.reset(obs)
    rng = np.random.RandomState(7)
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < seconds:
        act = np.zeros((E, A, 3), np.int32)
        act[..., :2] = rng.randint(-1, 2, size=(E, A, 2))
        act[..., 2] = rng.randint(0, 2, size=(E, A))
        if mode == 'next_step':
            rs = (ad != 0) | (o.state()['steps'] >= horizon)
            if rs.any():
                o.reset(obs, mask=rs.astype(np.uint8))
                ad[rs] = 0
            o.step(act, obs, rew, done, ad, acting, mask=(~rs).astype(np.uint8))
        else:
            o.step(act, obs, rew, done, ad, acting)
            o.reset(obs, all_done=ad, horizon=horizon)
        steps += 1
    dt = time.perf_counter() - t0
    return dict(value=float(acting.sum()) / dt, unit='agent-steps/s', cores=threads, kind='port',
                sample=f'{envs} envs x {steps} steps, {mode} auto-reset (incl. action generation '
                       f'in numpy), {dt:.1f} s, oracle/gw_oracle.c with {threads} OpenMP threads')


def quick_config(name, steps=200, warmup=20):
    """A short single-GPU measurement of another BASELINE config (not the
    metric's): agent-steps/s and the step kernel's average launch time."""
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    if name == 'maze':
        cc, E, horizon = maze_sim().compiled(), 1024, 200
    elif name.startswith('rtt'):
        cc, E, horizon = rtt_sim().compiled(), (8192 if name == 'rtt_8192' else 1024), 200
    else:
        cc, E, horizon = pacman_sim().compiled(), 16384, 200
    eng = GridWorldEngine(cc, E, seeds=env_seeds(E))
    if name == 'maze' or name.startswith('rtt'):
        eng.reset()
        eng.all_done.zero_()
        step = lambda: eng.step_autoreset_next(horizon=horizon)
    else:
        eng.turn_reset()
        eng.all_done.zero_()
        step = lambda: eng.turn_step(horizon=horizon)
    key = 0x5eed0001
    for t in range(warmup):
        eng.random_actions(key, t)
        step()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    a0 = int(eng.acting.sum().item())
    t0 = time.perf_counter()
    for t in range(steps):
        eng.random_actions(key, warmup + t)
        evs[t][0].record()
        step()
        evs[t][1].record()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    acting = int(eng.acting.sum().item()) - a0
    if name == 'maze':
        nbytes = step_bytes(E, eng.A, cc.obs_side)
        desc = 'MazeNavigation 16x16 (maze_16 fixture map), 1024 envs, AllStep, next_step auto-reset'
    elif name.startswith('rtt'):
        nbytes = rtt_step_bytes(E, eng.A, cc.obs_side, eng.act_dim)
        desc = (f'ReachTheTarget 64x64, 128 barriers + 127 runners + target (256 entities, '
                f'workgroup-per-env kernel), {E} envs on one GPU '
                f'({"all of config 4" if E == 8192 else "one GPU share of config 4 8192 envs / 8"}), '
                'AllStep, horizon 200, next_step auto-reset')
    else:
        nbytes = pacman_turn_bytes(E, eng.A, cc.rows * cc.cols, (eng.n_passive + 31) // 32)
        desc = ('Pacman pacman.txt, 4 baddies + pacman, 16384 envs, TurnBasedManager protocol '
                '(one agent acts per env per call), next_step auto-reset')
    return {'workload': desc, 'value': round(acting / dt, 1), 'unit': 'agent-steps/s',
            'env_steps_per_s': round(E * steps / dt, 1), 'ms_per_step': round(dt / steps * 1e3, 4),
            'kernel_ms': round(kms, 4), 'bytes_per_launch': nbytes,
            'achieved_GBs': round(nbytes / (kms * 1e-3) / 1e9, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=500)
    ap.add_argument('--warmup', type=int, default=50)
    ap.add_argument('--envs', type=int, default=4096, help='envs per GPU')
    ap.add_argument('--horizon', type=int, default=200)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    ap.add_argument('--autoreset', choices=['next_step', 'same_step'], default='next_step')
    ap.add_argument('--no-other', action='store_true',
                    help='skip the other auto-reset mode and the other configs')
    ap.add_argument('--workload', choices=['team_battle', 'rtt'], default='team_battle',
                    help="'rtt': BASELINE config 4 (ReachTheTarget 64x64, 256 entities; "
                         "--envs 1024 = one GPU's share of 8192) as the timed workload, "
                         "for profiling its kernel (not the headline metric)")
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    from abmarl_amd import _abi
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    from abmarl_amd.parallel import shard_envs, gather_episode_stats
    sim = team_battle_sim() if args.workload == 'team_battle' else rtt_sim()
    cc = sim.compiled()
    if args.workload == 'rtt' and args.envs == 4096:
        args.envs = 1024
    first, E_local = shard_envs(args.envs * world, rank, world)
    key = 0x5eed0000  # policy key shared by all ranks; global env ids make streams distinct

    def run(mode):
        """Fresh engine (same seeds), warmup, then K timed steps."""
        eng = GridWorldEngine(cc, E_local, seeds=env_seeds(E_local, run=0, first_env=first))
        eng.reset()
        eng.all_done.zero_()
        torch.cuda.synchronize()
        eng.check_errors()
        step = eng.step_autoreset_next if mode == 'next_step' else eng.step_autoreset

        def one_step(t, ev=None):
            eng.random_actions(key, t, env_offset=first)
            if ev is not None:
                ev[0].record()
            step(horizon=args.horizon)
            if ev is not None:
                ev[1].record()

        for t in range(args.warmup):
            one_step(t)
        torch.cuda.synchronize()
        # ReachTheTarget: a runner placed on the target's cell and killed there
        # raises the reference's KeyError; the auto-reset modes reset that env
        eng.check_errors(allow=_abi.GW_ERR_DOUBLE_REMOVE if args.workload == 'rtt' else 0)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        acting0 = int(eng.acting.sum().item())
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(args.steps):
            one_step(args.warmup + t, evs[t])
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        dt = time.perf_counter() - t0
        acting = int(eng.acting.sum().item()) - acting0
        step_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        tot = torch.tensor([acting, dt, E_local], dtype=torch.float64, device=eng.device)
        kms = torch.tensor([step_ms], dtype=torch.float64, device=eng.device)
        if dist:
            acts = tot.clone(); dist.all_reduce(acts, op=dist.ReduceOp.SUM)
            tmax = tot.clone(); dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
            dist.all_reduce(kms, op=dist.ReduceOp.MAX)
            tot = torch.stack([acts[0], tmax[1], acts[2]])
        return eng, dict(acting=tot[0].item(), dt=tot[1].item(), envs=tot[2].item(),
                         step_ms=step_ms, step_ms_max=kms[0].item())

    other = 'same_step' if args.autoreset == 'next_step' else 'next_step'
    eng, r = run(args.autoreset)
    A, S = eng.A, cc.obs_side
    stats = gather_episode_stats(eng.acting, eng.get_state()['steps'], dist)
    del eng
    r2 = None if args.no_other else run(other)[1]
    acting_all, dt_all, envs_all, step_ms = r['acting'], r['dt'], r['envs'], r['step_ms']
    step_ms_all = r['step_ms_max']

    if rank == 0:
        value = acting_all / dt_all
        nbytes = step_bytes(E_local, A, S)
        kname = 'step_kernel<7>'
        workload = ('TeamBattle 32x32, 64 agents / 2 teams, 4096 envs per GPU, '
                    f'horizon 200, {args.autoreset} auto-reset')
        if args.workload == 'rtt':
            nbytes = rtt_step_bytes(E_local, A, S, cc.act_dim)
            kname = 'wg_step_kernel<7>'
            workload = (f'ReachTheTarget 64x64 (BASELINE config 4), 256 entities, {E_local} envs per GPU, '
                        f'horizon 200, {args.autoreset} auto-reset (profiling run, not the headline metric)')
        achieved = nbytes / (step_ms * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, 'profiles', 'pmc_step_kernel.json' if args.workload == 'team_battle'
                           else 'pmc_wg_step_kernel.json')
        if os.path.exists(pmc):
            traffic = json.load(open(pmc)).get('hbm_bytes_per_launch')
        out = {
            'metric': METRIC,
            'value': round(value, 1),
            'unit': 'agent-steps/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(dt_all / args.steps * 1e3, 4),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'int32 (positions/obs), f64 (health/reward)',
            'data': 'synthetic: Philox random-policy actions, random-init TeamBattle episodes',
            'config': {'workload': workload,
                       'envs_per_gpu': E_local, 'global_envs': int(envs_all),
                       'parallelism': f'env-sharded x{world} (no data-path collective)'},
            'env_steps_per_s': round(envs_all * args.steps / dt_all, 1),
            'mean_acting_agents_per_env_step': round(acting_all / (envs_all * args.steps), 2),
            'roofline': {'bound': 'hbm', 'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 5),
                         'traffic': traffic, 'kernel': kname,
                         'kernel_ms': round(step_ms_all, 4),
                         'bytes_per_launch': nbytes},
            'episode_stats': stats,
            'autoreset': args.autoreset,
            'other_autoreset': None if r2 is None else {
                'mode': other, 'value': round(r2['acting'] / r2['dt'], 1),
                'ms_per_step': round(r2['dt'] / args.steps * 1e3, 4),
                'kernel_ms': round(r2['step_ms_max'], 4)},
        }
        if world == 1 and not args.no_other and args.workload == 'team_battle':
            # BASELINE configs 2 and 5 (single GPU, short runs; not the metric)
            out['other_configs'] = {'maze_16': quick_config('maze'),
                                    'reach_the_target_64': quick_config('rtt'),
                                    'reach_the_target_64_all_8192': quick_config('rtt_8192'),
                                    'pacman_turn_based': quick_config('pacman')}
        if world == 1 and not args.no_cpu_baseline and args.workload == 'team_battle':
            out['cpu_baseline'] = cpu_baseline(cc, seconds=args.cpu_seconds, horizon=args.horizon,
                                               mode=args.autoreset)
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
