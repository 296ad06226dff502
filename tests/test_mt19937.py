"""The oracle's MT19937 restatement vs numpy's legacy RandomState (the
reference's RNG: np.random.seed / uniform / randint / choice / permutation,
SURVEY §8a R15)."""
import numpy as np
import pytest


@pytest.mark.parametrize('seed', [0, 1, 24, 17, 1000003, 2**32 - 1])
def test_raw_words(oracle_mod, seed):
    got = oracle_mod.mt_probe(seed, 0, 0, 2000).astype(np.uint64)
    ref = np.random.RandomState(seed).randint(0, 2**32, size=2000, dtype=np.uint64)
    # legacy randint on the full uint32 range consumes one raw word each
    ref32 = np.random.RandomState(seed).randint(0, 2**32, size=2000, dtype=np.uint32)
    assert (got == ref32.astype(np.uint64)).all()
    assert ref.shape == got.shape


@pytest.mark.parametrize('seed', [3, 24, 99])
def test_uniform(oracle_mod, seed):
    got = oracle_mod.mt_probe(seed, 1, 0, 1500)
    rs = np.random.RandomState(seed)
    ref = np.array([rs.uniform() for _ in range(1500)])
    assert (got.view(np.uint64) == ref.view(np.uint64)).all()


@pytest.mark.parametrize('max_', [0, 1, 2, 5, 63, 64, 1000, 1023, 2**31 + 5])
def test_bounded(oracle_mod, max_):
    got = oracle_mod.mt_probe(7, 2, max_, 700)
    rs = np.random.RandomState(7)
    ref = np.array([rs.randint(0, max_ + 1) for _ in range(700)], dtype=np.float64)
    assert (got == ref).all()
    # choice(list) consumes exactly like randint(0, len)
    rs2 = np.random.RandomState(7)
    if max_ < 5000:
        lst = list(range(max_ + 1))
        ref2 = np.array([rs2.choice(lst) for _ in range(700)], dtype=np.float64)
        assert (got == ref2).all()


def test_permutation_is_fisher_yates_on_bounded_draws(oracle_mod):
    # permutation(n) = for i = n-1..1: j = bounded(i); swap  (legacy shuffle)
    for n in [1, 2, 3, 7, 30]:
        rs = np.random.RandomState(11)
        ref = rs.permutation(n)
        draws = oracle_mod.mt_probe(11, 2, 0, 0)  # noqa: F841 (probe API sanity)
        rs2 = np.random.RandomState(11)
        arr = list(range(n))
        for i in range(n - 1, 0, -1):
            j = rs2.randint(0, i + 1)
            arr[i], arr[j] = arr[j], arr[i]
        assert arr == list(ref)
        # and the stream position afterwards agrees
        assert rs.randint(0, 2**32, dtype=np.uint32) == rs2.randint(0, 2**32, dtype=np.uint32)


def test_choice_without_replacement_is_permutation_prefix():
    for n, k in [(1, 1), (3, 1), (5, 2), (9, 3)]:
        rs = np.random.RandomState(5)
        got = rs.choice(n, size=k, replace=False)
        rs2 = np.random.RandomState(5)
        assert list(got) == list(rs2.permutation(n)[:k])
