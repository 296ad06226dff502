"""bench.py --gpus N: the rank layout it runs or refuses (CPU only: the
refusals happen before anything touches the GPU)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=300)


def test_check_world_layouts(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    assert bench.check_world(1) is None
    monkeypatch.setattr(bench.torch.cuda, 'device_count', lambda: 8)
    assert bench.check_world(8) == 'launch'
    assert 'visible GPU' in bench.check_world(9)
    assert 'at least one' in bench.check_world(0)
    monkeypatch.setenv('WORLD_SIZE', '8')
    assert bench.check_world(8) is None           # a rank under torch.distributed.run
    assert 'disagree' in bench.check_world(4)


@pytest.mark.skipif(__import__('torch').cuda.device_count() >= 2, reason='a multi-GPU host launches')
def test_more_gpus_than_visible_is_refused():
    r = _bench(['--gpus', '2', '--steps', '1', '--warmup', '0'])
    assert r.returncode == 2, (r.returncode, r.stderr[-500:])
    assert 'visible GPU' in r.stderr


def test_world_size_mismatch_is_refused():
    r = _bench(['--gpus', '4', '--steps', '1', '--warmup', '0'], WORLD_SIZE='2', RANK='0', LOCAL_RANK='0')
    assert r.returncode == 2, (r.returncode, r.stderr[-500:])
    assert 'disagree' in r.stderr


def test_gpus_defaults_to_the_launchers_world(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    assert bench.resolve_gpus(None) == 1
    monkeypatch.setenv('WORLD_SIZE', '4')
    assert bench.resolve_gpus(None) == 4              # torchrun --nproc-per-node 4 bench.py
    assert bench.resolve_gpus(2) == 2                 # explicit: check_world flags the mismatch


def test_share_gpu_layouts(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    monkeypatch.setattr(bench.torch.cuda, 'device_count', lambda: 1)
    assert bench.check_world(2, share_gpu=True, backend='gloo') == 'launch'
    assert 'gloo' in bench.check_world(2, share_gpu=True, backend='nccl')
    assert 'at most 16' in bench.check_world(17, share_gpu=True, backend='gloo')
    assert 'visible GPU' in bench.check_world(2)


def test_launcher_leaves_hip_uninitialised(monkeypatch):
    """The launching parent of `bench.py --gpus N` starts the ranks before
    anything initialises HIP (an exec or fork after HIP init is forbidden on
    the GPU pool): main() reaches launch_ranks with torch.cuda uninitialised."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    seen = {}

    def fake_launch(n):
        seen['n'] = n
        seen['init'] = bench.torch.cuda.is_initialized()
        return 0
    monkeypatch.setattr(bench, 'launch_ranks', fake_launch)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '2', '--share-gpu', '--dist-backend', 'gloo',
                                      '--steps', '1', '--warmup', '0'])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 0
    assert seen == {'n': 2, 'init': False}
