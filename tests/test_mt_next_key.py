"""The MT19937 identity the placement kernels use to draw past a twist without
twisting (gw_engine.hip position_reset_jacobi, gw_rtt.inc wg_stream_word):
word j < 227 of the NEXT key is key[j + 397] ^ (y >> 1) ^ (y & 1 ? MATRIX_A : 0)
with y = (key[j] & UPPER) | (key[j + 1] & LOWER), all from the CURRENT key,
because mt19937's twist rewrites key[j] from key[j], key[j + 1] and
key[j + 397], none of them rewritten yet for j < 227.  Checked here against
numpy's legacy RandomState (the reference's generator) drawing raw words
across the twist."""
import numpy as np


def _temper(y):
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9d2c5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xefc60000))
    return y ^ (y >> np.uint32(18))


def _next_key_words(key, n):
    j = np.arange(n)
    y = (key[j] & np.uint32(0x80000000)) | (key[j + 1] & np.uint32(0x7fffffff))
    mag = np.where((y & np.uint32(1)) != 0, np.uint32(0x9908b0df), np.uint32(0))
    return _temper(key[j + 397] ^ (y >> np.uint32(1)) ^ mag)


def test_words_past_the_twist_from_the_untwisted_key():
    for seed in (0, 1, 12345, 2 ** 31 - 1):
        rs = np.random.RandomState(seed)
        rs.random_sample(777)                        # some position inside a key
        name, key, pos = rs.get_state()[:3]
        key = np.asarray(key, dtype=np.uint32)
        # draw the rest of this key, then 226 words of the next one, raw
        # (a full-range uint32 randint is one untouched word per value)
        rest = rs.randint(0, 2 ** 32, size=624 - pos, dtype=np.uint32)
        assert (rest == _temper(key[pos:])).all()
        nxt = rs.randint(0, 2 ** 32, size=226, dtype=np.uint32)
        assert (nxt == _next_key_words(key, 226)).all(), seed
