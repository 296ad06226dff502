"""TEST INFRASTRUCTURE ONLY — one single-threaded, core-pinned C-oracle
process for bench.py's cpu_baseline leg (one process per core,
pinned with sched_setaffinity, each running independent envs).

    python -m oracle.cpu_worker --cpu C --seconds S --envs N --first-env F
                                [--horizon H] [--mode next_step|same_step]

Prints one JSON line: acting agent-steps, env-steps and the wall time of
this process's loop.  Only bench.py's cpu_baseline starts it; the product
path never does.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cpu', type=int, required=True)
    ap.add_argument('--seconds', type=float, default=10.0)
    ap.add_argument('--envs', type=int, default=64)
    ap.add_argument('--first-env', type=int, default=0)
    ap.add_argument('--horizon', type=int, default=200)
    ap.add_argument('--mode', choices=['next_step', 'same_step'], default='next_step')
    a = ap.parse_args()
    os.sched_setaffinity(0, {a.cpu})
    import numpy as np
    from oracle.oracle import Oracle, lib
    from abmarl_amd.examples.workloads import team_battle_sim
    lib().gwo_set_threads(1)
    cc = team_battle_sim().compiled()
    E, A = a.envs, cc.n_agents
    o = Oracle(cc, E)
    # the GPU line's seeds for global env ids first_env .. first_env + E - 1
    e = np.arange(a.first_env, a.first_env + E, dtype=np.uint64)
    o.seed((e & np.uint64(0xFFFFFFFF)).astype(np.uint32))
    obs = o.new_obs()
    rew = np.zeros((E, A)); done = np.zeros((E, A), np.uint8); ad = np.zeros(E, np.uint8)
    acting = np.zeros(E, np.uint64)
    o.reset(obs)
    rng = np.random.RandomState(7 + a.first_env)
    act = np.zeros((E, A, 3), np.int32)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.seconds:
        act[..., :2] = rng.randint(-1, 2, size=(E, A, 2))
        act[..., 2] = rng.randint(0, 2, size=(E, A))
        if a.mode == 'next_step':
            rs = (ad != 0) | (o.state()['steps'] >= a.horizon)
            if rs.any():
                o.reset(obs, mask=rs.astype(np.uint8))
                ad[rs] = 0
            o.step(act, obs, rew, done, ad, acting, mask=(~rs).astype(np.uint8))
        else:
            o.step(act, obs, rew, done, ad, acting)
            o.reset(obs, all_done=ad, horizon=a.horizon)
        steps += 1
    dt = time.perf_counter() - t0
    print(json.dumps(dict(cpu=a.cpu, acting=int(acting.sum()), env_steps=E * steps, steps=steps,
                          seconds=dt)), flush=True)


if __name__ == '__main__':
    main()
