"""A trajectory of user components registered beside the REFERENCE's
built-in components (tests/user_lanterns.py: lantern keepers sharing oil
with the keepers they can see, blocking wanderers), run in this container on
the reference's PositionState / MoveActor / PositionCenteredEncodingObserver /
create_grid_and_mask under its AllStepManager.

Output: tests/golden/lanterns.json -- per env the seed, and after reset and
every step the actions, observations (grid windows and oil readings),
rewards, dones, positions, oil levels and the numpy RNG position + key CRC.
Floats are stored as float.hex (bit-exact).
Run:  python tests/golden/make_comms.py      (needs /root/reference)
"""
import json
import os
import sys
import types
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get('ABMARL_REFERENCE', '/root/reference')


def fhex(x):
    return float(x).hex()


def enc_obs(o):
    out = {}
    for aid, d in o.items():
        e = {}
        if 'position_centered_encoding' in d:
            e['grid'] = np.asarray(d['position_centered_encoding']).astype(int).tolist()
        if 'oil' in d:
            e['oil'] = [fhex(v) for v in d['oil']]
        out[aid] = e
    return out


def snapshot(sim):
    st = np.random.get_state()
    return dict(pos={a.id: [int(x) for x in a.position] for a in sim.agents.values()},
                oil={a.id: fhex(a.oil) for a in sim.agents.values() if hasattr(a, '_oil')},
                mt_pos=int(st[2]),
                mt_crc=zlib.crc32(np.ascontiguousarray(st[1], dtype=np.uint32).tobytes()))


def reference_namespace():
    from abmarl.sim import ObservingAgent, ActingAgent
    from abmarl.sim.gridworld.agent import GridWorldAgent, MovingAgent, GridObservingAgent
    from abmarl.sim.gridworld.base import GridWorldSimulation
    from abmarl.sim.gridworld.state import StateBaseComponent, PositionState
    from abmarl.sim.gridworld.actor import ActorBaseComponent, MoveActor
    from abmarl.sim.gridworld.observer import ObserverBaseComponent, PositionCenteredEncodingObserver
    from abmarl.sim.gridworld.done import DoneBaseComponent
    from abmarl.sim.gridworld.utils import create_grid_and_mask
    from abmarl.tools import Box
    from gym.spaces import Discrete, Dict
    return types.SimpleNamespace(**{k: v for k, v in locals().items()})


def main():
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import gym_stub
    gym_stub.install()
    sys.path.insert(0, REF)
    import user_lanterns
    from abmarl.managers import AllStepManager
    from abmarl.sim.gridworld.registry import register, registry
    classes = user_lanterns.lantern_classes(reference_namespace())
    for k in user_lanterns.USER_COMPONENTS:
        register(classes[k])
    assert classes['OilGauge'] in registry['observer'].values()
    c = user_lanterns.CASE
    rng = np.random.RandomState(c['action_seed'])
    envs = []
    for seed in c['seeds']:
        sim = user_lanterns.build(classes)
        m = AllStepManager(sim)
        np.random.seed(seed)
        rec = dict(seed=seed, reset=dict(obs=enc_obs(m.reset()), **snapshot(sim)), steps=[])
        for t in range(c['n_steps']):
            acts = user_lanterns.actions(sim, rng, m.done_agents)
            o, r, d, _ = m.step(acts)
            rec['steps'].append(dict(
                actions={k: {kk: (np.asarray(vv).tolist()) for kk, vv in v.items()} for k, v in acts.items()},
                obs=enc_obs(o), reward={k: fhex(v) for k, v in r.items()},
                done={k: bool(v) for k, v in d.items()}, **snapshot(sim)))
            if d['__all__']:
                break
        envs.append(rec)
    path = os.path.join(HERE, 'lanterns.json')
    json.dump(dict(case=c, envs=envs), open(path, 'w'))
    print(f"lanterns: {len(envs)} envs, {[len(e['steps']) for e in envs]} steps -> "
          f"{os.path.getsize(path)} B")


if __name__ == '__main__':
    main()
