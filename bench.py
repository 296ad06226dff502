"""Benchmark: agent-steps/s of random-policy TeamBattle rollouts on MI355X.

Workload (BASELINE.json configs[2], the metric's config): TeamBattle 32x32,
64 BattleAgents in 2 teams, 4096 envs per GPU (weak scaling: N GPUs run
N x 4096 envs, sharded by global env id, no data-path collective;
--global-envs G: strong scaling, G envs in total), horizon 200 with
on-device auto-reset.  Before the warmup, --preroll steps (default 1000,
five horizons) run untimed so that the timed window is steady state:
episodes at mixed phases, envs resetting inside the window.

Timed protocol, default --mode rollout (the headline line): the K timed
steps' random-policy actions (Philox kernel) are generated into HBM BEFORE
the timed region -- inputs resident in HBM, legitimate for a random policy,
not for a policy that reads observations -- and the timed region holds only
gw_rollout launches of --fragment steps each (K = 20 is ONE launch), with
skip_done_obs: obs rows of entities that get no observation in a step (done
entities, all_step_manager.py:68-71) are not written.  --mode step (and the
line's "closed_loop" block) is the RLlib per-step protocol instead: one
Philox action launch + one fused AllStepManager.step launch per timed step.
--workload maze | rtt | pacman times BASELINE configs 2, 4 and 5 instead
(their own lines).

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
       N > 1 launches N ranks itself (torch.distributed.run, one process per
       GPU, RCCL) unless it already runs under a launcher that set WORLD_SIZE,
       which must then equal N (--gpus omitted: N = WORLD_SIZE):
       python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
       Readiness runs of the multi-rank path on a one-GPU box only:
       --share-gpu --dist-backend gloo (every rank on cuda:0; the collectives
       over gloo on host copies; RCCL refuses two ranks on one GPU).  Such a
       line is not a scaling measurement.
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

from abmarl_amd.examples.workloads import team_battle_sim, maze_sim, rtt_sim, pacman_sim  # noqa: E402

# the reference's own AllStepManager TeamBattle loop, measured in
# the build container during the survey (pure Python, one process per core)
REFERENCE_RATE_PER_CORE = 14.3e3


def host_cpu():
    """CPU model and logical core count of this host (cpu_baseline)."""
    model = 'unknown'
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                model = line.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    return model, os.cpu_count()


def pacman_turn_bytes(E, A, HW, pwords):
    """Algorithmic HBM bytes of one turn-based Pacman launch: actions read
    (move + present, 8 B per lane), ONE lane's absolute observation 4*HW,
    per lane reward 8 + done 1 + returned 1, state read+write 2*(pos 8 +
    seq 4 + health 8 + flags 1 + reward accumulator 8) per lane, food bits
    2*4*pwords, per env all_done 1 + turn 4 + cycle 2*4 + steps 2*4 +
    acting 2*8 + RNG pos/counter 2*8."""
    return E * (A * (8 + 8 + 1 + 1 + 2 * 29) + 4 * HW + 8 * pwords + 1 + 4 + 8 + 8 + 16 + 16)


def pacman_turn_rollout_bytes(E, A, HW, pwords, n_steps, returned):
    """Algorithmic HBM bytes of one gw_turn_rollout launch of n_steps turns:
    per turn and lane actions read 8 (move + present), reward 8 + done 1 +
    returned 1; per turn and env all_done 1 + turn 4; 4*HW per returned obs
    row (`returned` over the launch, approximated by the acting agent-steps:
    one row per turn except at an episode's end); per launch the state
    read+write of pacman_turn_bytes."""
    return (n_steps * E * (A * (8 + 8 + 1 + 1) + 1 + 4) + 4 * HW * returned +
            E * (A * 2 * 29 + 8 * pwords + 8 + 8 + 16 + 16))


def step_bytes(E, A, S):
    """Algorithmic HBM bytes of one step launch:
    per entity slot: actions 12 + obs 4*S*S + reward 8 + done 1 +
    state read+write 2*(pos 8 + seq 4 + health 8 + flags 1); per env:
    __all__ 1 + steps 2*4 + acting 2*8 + RNG pos/counter 2*8."""
    per_slot = 12 + 4 * S * S + 8 + 1 + 2 * (8 + 4 + 8 + 1)
    per_env = 1 + 8 + 16 + 16
    return E * (A * per_slot + per_env)


def rollout_bytes(E, A, S, n_steps, acting, act_dim=3):
    """Algorithmic HBM bytes of one gw_rollout launch of n_steps steps with
    skip_done_obs (SURVEY §8d per agent-step, obs only for the agents that get
    one): per step and entity slot actions 4*act_dim + reward 8 + done 1,
    per step and env __all__ 1, obs 4*S*S per acting agent-step (`acting`
    over the launch: every acting agent observes in these programs), and the
    per-launch state read+write 2*(pos 8 + seq 4 + health 8 + flags 1) per
    slot + 41 B per env (step / acting counters, RNG position)."""
    return (n_steps * E * (A * (4 * act_dim + 8 + 1) + 1) + 4 * S * S * acting +
            E * A * 2 * (8 + 4 + 8 + 1) + E * 41)


def rtt_step_bytes(E, A, S, act_dim):
    """step_bytes with the SelectiveAttackActor's wider action rows
    (4 * act_dim B per entity slot instead of 12)."""
    return step_bytes(E, A, S) + E * A * (4 * act_dim - 12)


def physical_cpus():
    """One logical CPU per physical core among the CPUs this process may run
    on (sched_getaffinity; SMT siblings dropped via sysfs topology)."""
    avail = sorted(os.sched_getaffinity(0))
    seen, out = set(), []
    for c in avail:
        try:
            sib = open(f'/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list').read().strip()
        except OSError:
            sib = str(c)
        if sib not in seen:
            seen.add(sib)
            out.append(c)
    return out, len(avail)


def cpu_baseline(cc, seconds=10.0, envs_per_core=64, horizon=200, mode='next_step'):
    """The C oracle (a port of the reference step) as ONE single-threaded
    process per physical core, each pinned with sched_setaffinity and running
    its own envs, for ~`seconds` of wall time, with the same
    auto-reset flow as the GPU line.  Processes are capped at the job's CPU
    share (OMP_NUM_THREADS, 16 on the GPU box): the pool gives one GPU job
    16 cores, so the whole-socket figure is extrapolated from the per-core
    rate and labelled as such."""
    import subprocess
    cores, n_logical = physical_cpus()
    share = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or len(cores)
    use = cores[:max(1, min(share, len(cores)))]
    procs = []
    for k, cpu in enumerate(use):
        cmd = [sys.executable, '-m', 'oracle.cpu_worker', '--cpu', str(cpu), '--seconds', str(seconds),
               '--envs', str(envs_per_core), '--first-env', str(k * envs_per_core),
               '--horizon', str(horizon), '--mode', mode]
        env = dict(os.environ, OMP_NUM_THREADS='1')
        procs.append(subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, env=env))
    res = []
    for pr in procs:
        out, _ = pr.communicate(timeout=seconds * 6 + 120)
        if pr.returncode != 0:
            raise RuntimeError(f'cpu_worker failed ({pr.returncode})')
        res.append(json.loads(out.decode().strip().splitlines()[-1]))
    per_core = [r['acting'] / r['seconds'] for r in res]
    total = float(sum(per_core))
    model, ncpu = host_cpu()
    # physical cores on the socket(s): distinct (package, core) ids in sysfs
    phys = set()
    for c in range(ncpu or 0):
        try:
            d = f'/sys/devices/system/cpu/cpu{c}/topology/'
            phys.add((open(d + 'physical_package_id').read().strip(), open(d + 'core_id').read().strip()))
        except OSError:
            pass
    n_phys = len(phys) or None
    steps = min(r['steps'] for r in res)
    return dict(value=total, unit='agent-steps/s', cores=len(use), kind='port',
                per_core=round(float(np.mean(per_core)), 1),
                per_core_min=round(float(np.min(per_core)), 1),
                sample=f'{len(use)} pinned single-threaded processes x {envs_per_core} envs, '
                       f'>= {steps} steps each, {mode} auto-reset (numpy action generation included), '
                       f'{seconds:.0f} s each, oracle/gw_oracle.c via oracle/cpu_worker.py',
                host_cpu=model, host_logical_cpus=ncpu, host_physical_cores=n_phys,
                affinity_logical_cpus=n_logical,
                extrapolated_all_physical_cores=(round(float(np.mean(per_core)) * n_phys, 1)
                                                 if n_phys else None),
                note=('a C port of the reference step (oracle/), not the reference itself: the '
                      'reference AllStepManager is pure Python and runs about '
                      f'{REFERENCE_RATE_PER_CORE:.0f} agent-steps/s per core (SURVEY §6, measured in '
                      'the build container); it cannot travel to the GPU box.  cores = the job\'s CPU '
                      'share (one pinned process per physical core in it); '
                      'extrapolated_all_physical_cores = per_core x every physical core of the host'))


def _traffic(roll, pmc, envs=None):
    """The committed PMC evidence of a launch shape (tools/prof_headline.sh
    <tag> rtt|pacman, tools/profile.sh maze) into a quick_config rollout
    block: HBM bytes over the algorithmic bytes of the SAME profiled launch.
    envs: only a profile of that many envs counts (None: any)."""
    if not os.path.exists(pmc):
        return
    prof = json.load(open(pmc))
    if prof.get('algorithmic_bytes_per_launch') and prof.get('hbm_bytes_per_launch') and \
            (envs is None or prof.get('envs') == envs):
        roll['traffic'] = round(prof['hbm_bytes_per_launch'])
        roll['traffic_ratio'] = round(prof['hbm_bytes_per_launch'] / prof['algorithmic_bytes_per_launch'], 4)
        roll['traffic_source'] = f'profiles/{os.path.basename(pmc)} ({prof.get("tag")})'
        if prof.get('traffic_ratio_calibrated'):
            # WRITE_SIZE calibrated on the launch's own store pattern (known bytes)
            roll['traffic_ratio_calibrated'] = round(prof['traffic_ratio_calibrated'], 4)
            roll['write_size_calibration'] = prof['write_size_calibration']['source']


def quick_config(name, steps=200, warmup=400):
    """A short single-GPU measurement of another BASELINE config (not the
    metric's): agent-steps/s and the step kernel's average launch time, after
    an untimed pre-roll of `warmup` steps (two horizons: steady state)."""
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
        step = lambda: eng.step_autoreset_next(horizon=horizon)
    else:
        eng.turn_reset()
        step = lambda: eng.turn_step(horizon=horizon)
    eng.all_done.zero_()
    # episode phases spread over the horizon (as in the headline line)
    eng.set_state(steps=torch.as_tensor((np.arange(E) * horizon // E).astype(np.int32), device=eng.device))
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
    roll = None
    if name == 'pacman':
        # the same engine as gw_turn_rollout fragments of 50 turns on actions
        # resident in HBM
        F = 50
        acts = torch.empty((steps,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
        for t in range(steps):
            eng.random_actions(key, warmup + steps + t, out=acts[t])
        out = eng.turn_rollout_buffers(F)
        eng.turn_rollout(acts[:F], horizon=horizon, out=out)           # untimed first launch
        revs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(F, steps, F)]
        torch.cuda.synchronize()
        r0 = int(eng.acting.sum().item())
        t1 = time.perf_counter()
        for i, ev in zip(range(F, steps, F), revs):
            ev[0].record()
            eng.turn_rollout(acts[i:i + F], horizon=horizon, out=out)
            ev[1].record()
        torch.cuda.synchronize()
        rdt = time.perf_counter() - t1
        ra = int(eng.acting.sum().item()) - r0
        lms = float(np.mean([a.elapsed_time(b) for a, b in revs]))
        rb = pacman_turn_rollout_bytes(E, eng.A, cc.rows * cc.cols, (eng.n_passive + 31) // 32, F,
                                       ra / len(revs))
        roll = {'value': round(ra / rdt, 1), 'ms_per_step': round(rdt / (steps - F) * 1e3, 4),
                'launch_ms': round(lms, 4), 'steps_per_launch': F, 'bytes_per_launch': round(rb),
                'achieved_GBs': round(rb / (lms * 1e-3) / 1e9, 2),
                'protocol': 'gw_turn_rollout fragments (one launch per 50 turns) on actions resident in HBM'}
        _traffic(roll, os.path.join(ROOT, 'profiles', f'pmc_pac_kernel_rollout_f{F}.json'), envs=E)
    else:
        # the same engine as gw_rollout fragments of 100 steps on actions
        # resident in HBM (the headline line's protocol)
        # (an untimed first fragment: the rollout instantiation's first launch
        # in the process, then three timed ones)
        F, NF = 100, 4
        acts = torch.empty((NF * F,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
        for t in range(NF * F):
            eng.random_actions(key, warmup + steps + t, out=acts[t])
        out = eng.rollout_buffers(F)
        eng.rollout(acts[:F], horizon=horizon, autoreset='next_step', skip_done_obs=True, out=out)
        revs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(F, NF * F, F)]
        for a_, b_ in revs:
            a_.record()
            b_.record()
        launches = [eng.rollout_launcher(acts[i:i + F], horizon=horizon, autoreset='next_step',
                                         skip_done_obs=True, out=out, events=ev)
                    for i, ev in zip(range(F, NF * F, F), revs)]
        torch.cuda.synchronize()
        r0 = int(eng.acting.sum().item())
        t1 = time.perf_counter()
        for launch in launches:
            launch()
        torch.cuda.synchronize()
        rdt = time.perf_counter() - t1
        ra = int(eng.acting.sum().item()) - r0
        lms = float(np.mean([a.elapsed_time(b) for a, b in revs]))
        rb = rollout_bytes(E, eng.A, cc.obs_side, F, ra / len(revs), eng.act_dim)
        roll = {'value': round(ra / rdt, 1), 'ms_per_step': round(rdt / ((NF - 1) * F) * 1e3, 4),
                'launch_ms': round(lms, 4), 'steps_per_launch': F, 'bytes_per_launch': round(rb),
                'achieved_GBs': round(rb / (lms * 1e-3) / 1e9, 2),
                'protocol': 'gw_rollout fragments of 100 steps on actions resident in HBM (after an '
                            'untimed first fragment), launch events recorded by the dispatch'}
        kn = {'maze': 'lane_step_kernel', 'rtt': 'wg_step_kernel', 'rtt_8192': 'wg_step_kernel'}[name]
        _traffic(roll, os.path.join(ROOT, 'profiles', f'pmc_{kn}_rollout_f{F}.json'),
                 envs=8192 if name == 'rtt_8192' else None)
    if name == 'maze':
        nbytes = step_bytes(E, eng.A, cc.obs_side)
        desc = ('MazeNavigation 16x16 (workloads.MAZE_16), 1024 envs, AllStep, next_step auto-reset '
                '(lane-group-per-env kernel)')
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
            'protocol': 'one step launch per step (closed loop), Philox action kernel in the timed region',
            'env_steps_per_s': round(E * steps / dt, 1), 'ms_per_step': round(dt / steps * 1e3, 4),
            'kernel_ms': round(kms, 4), 'bytes_per_launch': nbytes,
            'achieved_GBs': round(nbytes / (kms * 1e-3) / 1e9, 2),
            'rollout': roll}


WORKLOADS = {
    # name: (builder, default envs per GPU, step-kernel name, description)
    'team_battle': (team_battle_sim, 4096, 'step_kernel<7, 1>',
                    'TeamBattle 32x32, 64 agents / 2 teams'),
    'maze': (maze_sim, 1024, 'lane_step_kernel<5, 10>',
             'MazeNavigation 16x16 (BASELINE config 2), 1 navigator, blocking walls'),
    'rtt': (rtt_sim, 1024, 'wg_step_kernel<7>',
            'ReachTheTarget 64x64 (BASELINE config 4), 256 entities'),
    'pacman': (pacman_sim, 16384, 'pac_kernel',
               'Pacman pacman.txt (BASELINE config 5), 4 baddies + pacman, TurnBasedManager'),
}


def launch_ranks(n):
    """`bench.py --gpus N` outside a launcher: start the N ranks as
    `torch.distributed.run --nproc-per-node N` children (rendezvous on
    127.0.0.1) and return their exit code.  Called before anything touches
    the GPU (torch.cuda.device_count() does not initialise it)."""
    import socket
    import subprocess
    if torch.cuda.is_initialized():
        raise RuntimeError('launch_ranks: HIP is already initialised in the launching process')
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, cwd=ROOT)


def resolve_gpus(gpus):
    """--gpus as given, or (omitted) the launcher's WORLD_SIZE, else 1."""
    if gpus is not None:
        return gpus
    return int(os.environ.get('WORLD_SIZE', '1'))


def check_world(gpus, share_gpu=False, backend='nccl'):
    """The rank layout --gpus N asks for: None when this process is one of the
    N ranks (or N == 1), 'launch' when it must start them, else an error.
    Reads no GPU state (torch.cuda.device_count() does not initialise HIP on
    this image; tests/test_bench_launch.py checks the launcher leaves it
    uninitialised)."""
    world = os.environ.get('WORLD_SIZE')
    if gpus < 1:
        return f'--gpus {gpus}: at least one GPU'
    if share_gpu and gpus > 1 and backend != 'gloo':
        return '--share-gpu needs --dist-backend gloo (RCCL refuses two ranks on one GPU)'
    if share_gpu and gpus > 16:
        return f'--share-gpu with {gpus} ranks: at most 16 processes may share a GPU'
    if world is not None:
        if int(world) != gpus:
            return f'--gpus {gpus} but WORLD_SIZE={world}: the launcher and --gpus disagree'
        return None
    if gpus == 1:
        return None
    if not share_gpu:
        ndev = torch.cuda.device_count()
        if gpus > ndev:
            return f'--gpus {gpus} but this node has {ndev} visible GPU(s)'
    return 'launch'


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None,
                    help='ranks, one per GPU (default: WORLD_SIZE under a launcher, else 1)')
    ap.add_argument('--dist-backend', choices=['nccl', 'gloo'], default='nccl',
                    help='process group backend for N > 1 (nccl = RCCL over xGMI; gloo only for '
                         'readiness runs with --share-gpu)')
    ap.add_argument('--share-gpu', action='store_true',
                    help='readiness runs of the multi-rank path on a one-GPU box: every rank on '
                         'cuda:0 (needs --dist-backend gloo; not a scaling measurement)')
    ap.add_argument('--steps', type=int, default=500)
    ap.add_argument('--warmup', type=int, default=50)
    ap.add_argument('--preroll', type=int, default=1000,
                    help='untimed steps before the warmup, so the timed window is steady state '
                         '(episodes at mixed phases, auto-resets inside the window)')
    ap.add_argument('--envs', type=int, default=0, help='envs per GPU (weak scaling; default: the workload\'s)')
    ap.add_argument('--global-envs', type=int, default=0,
                    help='strong scaling: this many envs in total, sharded over the ranks')
    ap.add_argument('--horizon', type=int, default=200)
    ap.add_argument('--no-stagger', action='store_true',
                    help='start every episode at step 0 (default: the first episode of global env '
                         'e starts at step e * horizon // envs, so horizon resets are spread over '
                         'the steps instead of all envs resetting together every horizon)')
    ap.add_argument('--mode', choices=['rollout', 'step'], default='rollout',
                    help="rollout (default): the timed steps run as gw_rollout fragments (one launch "
                         "per --fragment steps, each env steps back to back inside it) on actions "
                         "already in HBM; step: one launch per step (closed loop, the RLlib "
                         "per-step protocol), with the Philox action kernel in the timed region")
    ap.add_argument('--fragment', type=int, default=100,
                    help='steps per gw_rollout launch (rollout mode)')
    ap.add_argument('--event-every', type=int, default=4,
                    help='HIP events around the step kernel of every n-th timed step (the others '
                         'go through the one-call gw_rollout_step path)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    ap.add_argument('--autoreset', choices=['next_step', 'same_step'], default='next_step')
    ap.add_argument('--no-other', action='store_true',
                    help='skip the other auto-reset mode and the other configs')
    ap.add_argument('--workload', choices=sorted(WORKLOADS), default='team_battle',
                    help="the timed workload; the metric's is team_battle (BASELINE configs[2]); the "
                         "others are BASELINE configs 2, 4, 5 (their own lines, not the headline metric)")
    ap.add_argument('--workgroup-waves', type=int, default=0,
                    help='team_battle: run on the workgroup-per-env kernel with this many waves per '
                         'env (2-4; the small-batch variant, gw_config.force_workgroup); 0: the '
                         'one-wave kernel')
    args = ap.parse_args()

    # --gpus N: N ranks, launched here if no launcher did (before any GPU call)
    args.gpus = resolve_gpus(args.gpus)
    chk = check_world(args.gpus, args.share_gpu, args.dist_backend)
    if chk == 'launch':
        sys.exit(launch_ranks(args.gpus))
    if chk is not None:
        print(f'bench.py: {chk}', file=sys.stderr)
        sys.exit(2)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = 0 if args.share_gpu else int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group('gloo')
    gloo = dist is not None and args.dist_backend == 'gloo'

    def coll(t):
        """a tensor on the process group's device (gloo: a host copy)"""
        return t.cpu() if gloo else t

    from abmarl_amd import _abi
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    from abmarl_amd.parallel import shard_envs, gather_episode_stats
    builder, default_envs, kname, wdesc = WORKLOADS[args.workload]
    sim = builder()
    cc = sim.compiled()
    if args.workgroup_waves:
        cc.cfg.force_workgroup = args.workgroup_waves
        kname = 'wg_step_kernel<7>'
        wdesc += f' (workgroup kernel, {args.workgroup_waves} waves per env)'
    turn = args.workload == 'pacman'
    strong = args.global_envs > 0
    total_envs = args.global_envs if strong else (args.envs or default_envs) * world
    first, E_local = shard_envs(total_envs, rank, world)
    key = 0x5eed0000  # policy key shared by all ranks; global env ids make streams distinct
    allow = _abi.GW_ERR_DOUBLE_REMOVE if args.workload == 'rtt' else 0
    untimed = args.preroll + args.warmup

    def run(mode, rollout):
        """Fresh engine (same seeds), pre-roll + warmup, then K timed steps."""
        eng = GridWorldEngine(cc, E_local, seeds=env_seeds(E_local, run=0, first_env=first))
        if turn:
            eng.turn_reset()
        else:
            eng.reset()
        eng.all_done.zero_()
        if not args.no_stagger:
            # episode phases spread over the horizon by global env id: the
            # horizon resets (most TeamBattle episodes end there) land on
            # every step instead of all envs together, so any window of the
            # rollout, however short, is steady state
            gid = np.arange(first, first + E_local, dtype=np.int64)
            eng.set_state(steps=torch.as_tensor((gid * args.horizon // total_envs).astype(np.int32),
                                                device=eng.device))
        torch.cuda.synchronize()
        eng.check_errors()
        step = (lambda: eng.turn_step(horizon=args.horizon)) if turn else \
            (eng.step_autoreset_next if mode == 'next_step' else eng.step_autoreset)
        if rollout:
            return eng, run_rollout(eng, mode)
        for t in range(untimed):
            if turn:
                eng.random_actions(key, t, env_offset=first)
                step()
            else:
                eng.rollout_step(key, t, env_offset=first, horizon=args.horizon, autoreset=mode)
        torch.cuda.synchronize()
        # ReachTheTarget: a runner placed on the target's cell and killed there
        # raises the reference's KeyError; the auto-reset modes reset that env
        eng.check_errors(allow=allow)
        every = max(1, args.event_every)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(0, args.steps, every)]
        acting0 = int(eng.acting.sum().item())
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(args.steps):
            if turn or t % every == 0:
                # HIP events on the launch stream around the step kernel
                eng.random_actions(key, untimed + t, env_offset=first)
                ev = evs[t // every] if t % every == 0 else None
                if ev:
                    ev[0].record()
                if turn:
                    step()
                else:
                    step(horizon=args.horizon)
                if ev:
                    ev[1].record()
            else:
                eng.rollout_step(key, untimed + t, env_offset=first, horizon=args.horizon,
                                 autoreset=mode)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        dt = time.perf_counter() - t0
        eng.check_errors(allow=allow)
        acting = int(eng.acting.sum().item()) - acting0
        step_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        tot = coll(torch.tensor([acting, dt, E_local], dtype=torch.float64, device=eng.device))
        kms = coll(torch.tensor([step_ms], dtype=torch.float64, device=eng.device))
        if dist:
            acts = tot.clone(); dist.all_reduce(acts, op=dist.ReduceOp.SUM)
            tmax = tot.clone(); dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
            dist.all_reduce(kms, op=dist.ReduceOp.MAX)
            tot = torch.stack([acts[0], tmax[1], acts[2]])
        return eng, dict(acting=tot[0].item(), dt=tot[1].item(), envs=tot[2].item(),
                         step_ms=step_ms, step_ms_max=kms[0].item(), steps_per_launch=1,
                         acting_local=acting)

    def run_rollout(eng, mode):
        """Pre-roll and warmup as rollout fragments, then the K timed steps as
        gw_rollout fragments of up to --fragment steps on actions generated
        into HBM before the timed region; HIP events around every launch.

        The GPU works until the synchronize that opens the timed region: the
        timed steps' actions and the acting-counter snapshot are produced
        before the last warmup fragment / right after it, on the device, so
        no host round trip leaves the GPU idle between the warmup and t0."""
        F = max(1, min(args.fragment, args.steps))
        nfrag = max(F, min(args.fragment, max(untimed, 1)))
        # warmup actions [0, nfrag), timed actions [nfrag, nfrag + steps)
        acts_all = torch.empty((nfrag + args.steps,) + tuple(eng.actions.shape),
                               dtype=torch.int32, device=eng.device)
        acts = acts_all[:nfrag]
        out = (eng.turn_rollout_buffers if turn else eng.rollout_buffers)(nfrag)
        # untimed pre-roll + warmup as fragments of up to nfrag steps, the
        # last one exactly F steps: it writes the same output slabs and reads
        # actions laid out as the timed fragments'
        sizes, rest = [], untimed
        last = min(F, rest)
        rest -= last
        while rest > 0:
            sizes.append(min(nfrag, rest))
            rest -= sizes[-1]
        if last:
            sizes.append(last)
        all_acts = acts_all[nfrag:nfrag + args.steps]
        frags = [(i, min(F, args.steps - i)) for i in range(0, args.steps, F)]
        if not sizes:
            for s in range(args.steps):
                eng.random_actions(key, untimed + s, env_offset=first, out=all_acts[s])
        t = 0
        for k, f in enumerate(sizes):
            for s in range(f):
                eng.random_actions(key, t + s, env_offset=first, out=acts[s])
            if k == len(sizes) - 1:
                # the timed steps' actions (inputs resident in HBM before timing)
                for s in range(args.steps):
                    eng.random_actions(key, untimed + s, env_offset=first, out=all_acts[s])
            if turn:
                eng.turn_rollout(acts[:f], horizon=args.horizon, out=out)
            else:
                eng.rollout(acts[:f], horizon=args.horizon, autoreset=mode, skip_done_obs=True, out=out)
            t += f
            if k == len(sizes) - 2:
                torch.cuda.synchronize()
                eng.check_errors(allow=allow)
        # prepared launches (validated here, one ctypes call each when timed);
        # their events, created by a first record outside the timed region,
        # are recorded by each launch's own kernel dispatch (its start and
        # end timestamps, gw_set_launch_events): no event record call inside
        # the timed region
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in frags]
        for a_, b_ in evs:
            a_.record()
            b_.record()
        launches = [eng.turn_rollout_launcher(all_acts[i:i + f], horizon=args.horizon, out=out, events=ev)
                    if turn else
                    eng.rollout_launcher(all_acts[i:i + f], horizon=args.horizon, autoreset=mode,
                                         skip_done_obs=True, out=out, events=ev)
                    for (i, f), ev in zip(frags, evs)]
        acting0 = eng.acting.clone()                      # after the last warmup fragment
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for launch in launches:
            launch()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        dt = time.perf_counter() - t0
        eng.check_errors(allow=allow)
        acting = int((eng.acting - acting0).sum().item())
        # launch-weighted mean: ms per launch of the full-size fragments
        full = [a.elapsed_time(b) for (i, f), (a, b) in zip(frags, evs) if f == F]
        launch_ms = float(np.mean(full))
        tot = coll(torch.tensor([acting, dt, E_local], dtype=torch.float64, device=eng.device))
        kms = coll(torch.tensor([launch_ms], dtype=torch.float64, device=eng.device))
        if dist:
            acts_t = tot.clone(); dist.all_reduce(acts_t, op=dist.ReduceOp.SUM)
            tmax = tot.clone(); dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
            dist.all_reduce(kms, op=dist.ReduceOp.MAX)
            tot = torch.stack([acts_t[0], tmax[1], acts_t[2]])
        return dict(acting=tot[0].item(), dt=tot[1].item(), envs=tot[2].item(),
                    step_ms=launch_ms, step_ms_max=kms[0].item(), steps_per_launch=F,
                    acting_local=acting)

    mode = 'next_step' if turn else args.autoreset
    rollout = args.mode == 'rollout'
    other = 'same_step' if mode == 'next_step' else 'next_step'
    eng, r = run(mode, rollout)
    A, n_passive = eng.A, eng.n_passive
    stats = gather_episode_stats(coll(eng.acting), coll(eng.get_state()['steps']), dist)
    del eng
    r2 = None if (args.no_other or turn) else run(other, rollout)[1]
    # the per-step (closed-loop) protocol beside the rollout line
    r3 = run(mode, False)[1] if (rollout and not args.no_other) else None
    acting_all, dt_all, envs_all = r['acting'], r['dt'], r['envs']
    step_ms_all = r['step_ms_max']

    if rank == 0:
        value = acting_all / dt_all
        S = cc.obs_side
        F = r['steps_per_launch']
        if rollout and turn:
            nbytes = pacman_turn_rollout_bytes(E_local, A, cc.rows * cc.cols, (n_passive + 31) // 32, F,
                                               r['acting_local'] * F / args.steps)
        elif rollout:
            # per launch: the local rank's acting agent-steps scaled to one launch
            nbytes = rollout_bytes(E_local, A, S, F, r['acting_local'] * F / args.steps, cc.act_dim)
        elif args.workload == 'team_battle' or args.workload == 'maze':
            nbytes = step_bytes(E_local, A, S)
        elif args.workload == 'rtt':
            nbytes = rtt_step_bytes(E_local, A, S, cc.act_dim)
        else:
            nbytes = pacman_turn_bytes(E_local, A, cc.rows * cc.cols, (n_passive + 31) // 32)
        scaling = 'strong' if strong else 'weak'
        workload = (f'{wdesc}, {E_local} envs per GPU ({int(envs_all)} in total, {scaling} scaling), '
                    f'horizon {args.horizon}, {mode} auto-reset, {args.preroll}-step pre-roll, ' +
                    (f'{"gw_turn_rollout" if turn else "gw_rollout"} fragments of {F} steps on actions '
                     f'resident in HBM (one launch '
                     f'per fragment, obs written for the agents that get one)' if rollout else
                     'one step launch per step + the Philox action kernel'))
        if args.workload != 'team_battle':
            workload += ' (not the headline metric\'s config)'
        achieved = nbytes / (step_ms_all * 1e-3) / 1e9
        traffic, rocprof_ms = None, None
        # the committed rocprofv3 evidence of this exact launch shape (a
        # rollout profile is per fragment length: tools/profile.sh ... <F>)
        pmc = os.path.join(ROOT, 'profiles', f'pmc_{kname.split("<")[0]}{f"_rollout_f{F}" if rollout else ""}.json')
        prof = {}
        if args.workload in ('team_battle', 'maze', 'rtt', 'pacman') and not args.workgroup_waves and os.path.exists(pmc):
            prof = json.load(open(pmc))
            traffic = prof.get('hbm_bytes_per_launch')
            rocprof_ms = prof.get('rocprof_avg_ms')
        roof = {'bound': 'hbm', 'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS,
                'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 5),
                'traffic': traffic, 'kernel': kname, 'kernel_ms': round(step_ms_all, 4),
                'kernel_timing': (f'HIP events recorded by every gw_rollout launch\'s own kernel dispatch '
                                  f'(hipExtLaunchKernel start/stop, {F} steps) on the launch stream, mean; '
                                  f'max over ranks' if rollout else
                                  f'HIP events around the step kernel of every {max(1, args.event_every)}'
                                  f'-th timed step (launch stream), mean; max over ranks'),
                'steps_per_launch': F,
                'bytes_per_launch': nbytes}
        if rocprof_ms:
            # the same ratio with the committed rocprofv3 kernel-trace average
            # (no event / dispatch time in it)
            roof['rocprof_kernel_ms'] = rocprof_ms
            roof['frac_rocprof'] = round(nbytes / (rocprof_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
        if traffic and prof.get('algorithmic_bytes_per_launch'):
            # PMC bytes over the algorithmic bytes of the SAME profiled launch
            # (its own acting count), not of this run's launch
            roof['traffic_ratio'] = round(traffic / prof['algorithmic_bytes_per_launch'], 4)
            roof['traffic_source'] = (f"profiles/{os.path.basename(pmc)} ({prof.get('tag')}: "
                                      f"{prof.get('workload_args', '')})")
        out = {
            'metric': METRIC,
            'value': round(value, 1),
            'unit': 'agent-steps/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'preroll_steps': args.preroll,
            'stagger': None if args.no_stagger else
            'first episode of global env e starts at step e*horizon//envs',
            'ms_per_step': round(dt_all / args.steps * 1e3, 4),
            'higher_is_better': True,
            'scaling': scaling,
            'vs_baseline': None,
            'dtype': 'int32 (positions/obs), f64 (health/reward)',
            'data': 'synthetic: Philox random-policy actions, random-init episodes',
            'config': {'workload': workload,
                       'envs_per_gpu': E_local, 'global_envs': int(envs_all),
                       'lanes': A, 'passive_entities': n_passive, 'cells': cc.rows * cc.cols,
                       'parallelism': f'env-sharded x{world} (no data-path collective)'},
            'dist': None if dist is None else {
                'backend': args.dist_backend, 'ranks_share_one_gpu': bool(args.share_gpu),
                'note': ('readiness run of the multi-rank path: every rank on cuda:0, collectives '
                         'over gloo; NOT a scaling measurement') if args.share_gpu else
                        'one rank per GPU'},
            'env_steps_per_s': round(envs_all * args.steps / dt_all, 1),
            'mean_acting_agents_per_env_step': round(acting_all / (envs_all * args.steps), 2),
            'acting_agent_steps': int(acting_all),
            'roofline': roof,
            'episode_stats': stats,
            'autoreset': mode,
            'other_autoreset': None if r2 is None else {
                'mode': other, 'value': round(r2['acting'] / r2['dt'], 1),
                'ms_per_step': round(r2['dt'] / args.steps * 1e3, 4),
                'kernel_ms': round(r2['step_ms_max'], 4)},
            'closed_loop': None if r3 is None else {
                'protocol': 'one step launch per step (RLlib per-step protocol), Philox action '
                            f'kernel in the timed region, HIP events on every {max(1, args.event_every)}'
                            '-th step kernel',
                'value': round(r3['acting'] / r3['dt'], 1),
                'ms_per_step': round(r3['dt'] / args.steps * 1e3, 4),
                'kernel_ms': round(r3['step_ms_max'], 4)},
        }
        if world == 1 and not args.no_other and args.workload == 'team_battle':
            # BASELINE configs 2, 4 and 5 (single GPU, short runs; not the metric)
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
