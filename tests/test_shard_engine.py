"""The multi-GPU path's sharding, on one GPU: engines that each hold a
contiguous shard of the global env range -- seeded from the global env ids
(env_seeds(first_env=...)), driven by Philox actions keyed by global env id
(random_actions(env_offset=...)), episode phases staggered by global env id
-- reproduce one engine over the whole range bit for bit, through the
headline's launch shape (gw_rollout fragments, next-step auto-reset,
skip_done_obs).  This is what bench.py runs per rank (shard_envs, run());
the per-env episode counters the ranks all-gather summarise to the whole's."""
import numpy as np
import pytest

from tests.cases import team_battle, build_rtt, RTT_CONFIG4

pytestmark = pytest.mark.gpu


def _engine(cc, first, n, total, horizon, run=0):
    import torch
    from abmarl_amd.engine import GridWorldEngine, env_seeds
    eng = GridWorldEngine(cc, n, seeds=env_seeds(n, run=run, first_env=first))
    eng.reset()
    eng.all_done.zero_()
    gid = np.arange(first, first + n, dtype=np.int64)
    eng.set_state(steps=torch.as_tensor((gid * horizon // total).astype(np.int32), device=eng.device))
    return eng


def _fragment(eng, key, t0, K, first):
    import torch
    acts = torch.empty((K,) + tuple(eng.actions.shape), dtype=torch.int32, device=eng.device)
    for t in range(K):
        eng.random_actions(key, t0 + t, env_offset=first, out=acts[t])
    return acts


def _run(eng, acts, horizon, skip):
    """One fragment into fresh slabs pre-filled with the same byte pattern in
    every engine: rows an env leaves unwritten (a step that raised: outputs
    not written) then compare equal."""
    out = eng.rollout_buffers(int(acts.shape[0]))
    for v in out.values():
        v.view(-1).view(__import__('torch').uint8).fill_(0xA5)
    return eng.rollout(acts, horizon=horizon, skip_done_obs=skip, out=out)


def _check_shards(cc, total, shards, horizon, frags, skip, key=0x5eed0000, allow_err=False):
    from abmarl_amd.parallel import shard_envs, gather_episode_stats
    whole = _engine(cc, 0, total, total, horizon)
    parts = []
    for r in range(shards):
        first, n = shard_envs(total, r, shards)
        parts.append((first, n, _engine(cc, first, n, total, horizon)))
    t = 0
    prev = None                # the previous step's done slab (whole engine)
    for K in frags:
        out_w = _run(whole, _fragment(whole, key, t, K, 0), horizon, skip)
        outs = [(first, n, _run(e, _fragment(e, key, t, K, first), horizon, skip)) for first, n, e in parts]
        for s in range(K):
            for first, n, out in outs:
                sl = slice(first, first + n)
                w = {k: v[s].cpu().numpy() for k, v in out_w.items()}
                p = {k: v[s].cpu().numpy() for k, v in out.items()}
                assert (w['reward'][sl].view(np.uint64) == p['reward'].view(np.uint64)).all(), (t + s, first)
                assert (w['done'][sl] == p['done']).all(), (t + s, first)
                assert (w['all_done'][sl] == p['all_done']).all(), (t + s, first)
                if skip:
                    # rows without an observation this step are left unwritten:
                    # an entity is observed when live after the step or before it
                    live = p['done'] == 0
                    if prev is not None:
                        live = live | (prev[sl] == 0)
                    assert (w['obs'][sl][live] == p['obs'][live]).all(), (t + s, first)
                else:
                    assert (w['obs'][sl] == p['obs']).all(), (t + s, first)
            prev = out_w['done'][s].cpu().numpy()
        t += K
    sw = {k: v.cpu().numpy() for k, v in whole.get_state().items()}
    for first, n, e in parts:
        sp = {k: v.cpu().numpy() for k, v in e.get_state().items()}
        sl = slice(first, first + n)
        for k in ('pos', 'health', 'seq', 'steps'):
            assert (sw[k][sl] == sp[k]).all(), k
        assert ((sw['flags'][sl] & 7) == (sp['flags'] & 7)).all(), 'flags'
        assert (sw['mt'][sl, :625] == sp['mt'][:, :625]).all(), 'RNG'
        assert (whole.acting.cpu().numpy()[sl] == e.acting.cpu().numpy()).all(), 'acting'
        assert (whole.err.cpu().numpy()[sl] == e.err.cpu().numpy()).all(), 'err'
    if not allow_err:
        assert not whole.err.any().item()
    # the report-time summary (gather_episode_stats: the ranks' all-gather) of
    # the shards' counters, concatenated in rank order, is the whole's
    import torch
    cat_a = torch.cat([e.acting for _, _, e in parts])
    cat_s = torch.cat([e.get_state()['steps'] for _, _, e in parts])
    st = whole.get_state()['steps']
    assert gather_episode_stats(cat_a, cat_s) == gather_episode_stats(whole.acting, st)


def test_shards_reproduce_the_whole_headline():
    """4096 global envs of the headline config as two shards [0, 2048) and
    [2048, 4096), 20-step fragments over a 200-step horizon (the bench's
    launch shape), against one 4096-env engine."""
    _check_shards(team_battle(), 4096, 2, horizon=200, frags=(20, 20, 20), skip=True)


def test_shards_reproduce_the_whole_uneven():
    """An uneven split (1000 envs over 3 shards: 334 / 333 / 333) with resets
    inside the fragments (horizon 30), every obs row written."""
    _check_shards(team_battle(), 1000, 3, horizon=30, frags=(25, 25), skip=False)


def test_shards_reproduce_the_whole_config4():
    """BASELINE config 4 (the workgroup-per-env kernel): 512 global envs as
    four shards, the double remove allowed."""
    kw = {k: v for k, v in RTT_CONFIG4.items() if k != 'kind'}
    cc = build_rtt(dict(kind='rtt', **kw)).compiled()
    _check_shards(cc, 512, 4, horizon=20, frags=(15, 15), skip=False, allow_err=True)
