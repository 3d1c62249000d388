"""CPU check of the K2 tiling algorithm (tests/k2_model.py) vs the oracle."""
import numpy as np
import pytest

from oracle import coracle
from tests import k2_model


def _check(lengths, tid, pos, span, origin=0):
    d, coff, ext = k2_model.model(np.asarray(lengths, np.int64), tid, pos, span, origin)
    ref, ext2, coff2 = coracle.depth(lengths, tid, pos, span)
    assert list(ext) == list(ext2)
    for t in range(len(lengths)):
        assert np.array_equal(d[coff[t]:coff[t] + ext[t]], ref[coff2[t]:coff2[t] + ext2[t]]), t


def _case(lengths, n, lo, hi, seed):
    rng = np.random.default_rng(seed)
    lengths = np.asarray(lengths, np.int64)
    live = np.nonzero(lengths > 0)[0]
    tid = rng.choice(live, size=n).astype(np.int32)
    pos = (rng.random(n) * lengths[tid]).astype(np.int32)
    span = rng.integers(lo, hi + 1, size=n).astype(np.int32)
    o = np.lexsort((pos, tid))
    return lengths, tid[o], pos[o], span[o]


@pytest.mark.parametrize("args", [
    ([300_000], 3000, 1, 200, 1),
    ([65536 * 3 + 17, 4096 * 5], 4000, 1, 9000, 3),
    ([500_000, 200_000, 70_000, 3], 2000, 1, 150_000, 6),
    ([300_000], 3000, 4090, 4100, 8),
    ([0, 1, 2, 63, 64, 65, 4095, 4096, 4097, 65535, 65536, 65537], 500, 1, 30, 2),
])
def test_model_random(args):
    _check(*_case(*args))


def test_model_end_on_chunk_start():
    # long reads whose end lands exactly on a chunk start (8192 with the small
    # genome's 2-tile chunks; 65536 / 32768 on large ones) or a tile start
    lengths = [200_000]
    pos = np.array([100, 5000, 60_000, 61_440, 3000, 1], np.int32)
    span = np.array([65436, 60536, 5536, 69632, 5192, 16383], np.int32)
    o = np.argsort(pos)
    _check(lengths, np.zeros(len(pos), np.int32), pos[o], span[o])


@pytest.mark.parametrize("origin", [(1 << 32) - 5 * 32768, (1 << 33) + 7 * 32768, 3 * 8192])
def test_model_read_words_past_2_32(origin):
    # K2's 18-bit read words as a genome whose global positions run past 2^32
    # (origin: a multiple of the chunk width, 8-tile chunks or the small
    # genome's 2-tile ones); spans above the cap, long reads, gaps wider than
    # the word's range between a chunk's reads and the reads before it
    lengths = [400_000, 900_000]
    tid = np.array([0, 0, 0, 0, 1, 1, 1, 1, 1], np.int32)
    pos = np.array([5, 300, 262_100, 390_000, 1, 2, 300_000, 300_001, 899_000], np.int32)
    span = np.array([150, 20_000, 70_000, 9_000, 4096, 4097, 150, 16_384, 1000], np.int32)
    _check(lengths, tid, pos, span, origin=origin)
    _check(*_case([700_000], 3000, 1, 30_000, 11), origin=origin)
