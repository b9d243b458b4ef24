"""The block-parallel first-true search of the hot-key rate-limit path
(`block_first` in engine.hip: a hot (ip, rule) run's end in `k_long_ends`, its
fixed windows in `k_long_windows`) against brute force, on the host build of
the same narrowing step.

Round 2's step skipped the positions between the last sample taken below `hi`
and `lo + (K-1) * stride` when no sample was true: a hot run ending there was
extended over the next keys' records, and `k_long_fill` overwrote their
outcomes (GPUTEST_r02: a new IP's first event reported InsideInterval +
Exceeded; reference internal/rate_limit.go:37-78 gives FirstTime)."""
import ctypes
import os
import random
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def lib():
    d = tempfile.mkdtemp(prefix="bjx_bs_")
    so = os.path.join(d, "libbs.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", so,
                    os.path.join(HERE, "cpu", "block_search.cpp")], check=True)
    L = ctypes.CDLL(so)
    L.bjx_test_block_first.restype = ctypes.c_uint64
    L.bjx_test_block_first.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
    return L


def _want(lo, hi, x):
    return min(max(x, lo), hi)


def test_round2_counterexample(lib):
    # 460 positions, stride 2: the samples stop at offset 458, the answer is 459
    assert lib.bjx_test_block_first(8, 468, 467, 256) == 467


@pytest.mark.parametrize("K", [256, 64, 7])
def test_against_brute_force(lib, K):
    rng = random.Random(K)
    for _ in range(20000):
        lo = rng.randint(0, 1000)
        n = rng.choice([rng.randint(0, 3 * K), rng.randint(1, 10 ** 6), rng.randint(1, 10 ** 12)])
        hi = lo + n
        x = max(0, rng.choice([rng.randint(lo, hi + 1), hi - 1, hi, lo, lo + 1, hi - rng.randint(0, 3 * K)]))
        assert lib.bjx_test_block_first(lo, hi, x, K) == _want(lo, hi, x), (lo, hi, x, K)


def test_every_tail_position(lib):
    # every answer position in ranges whose length is not a multiple of the stride
    for n in (257, 300, 460, 511, 513, 1000, 65537):
        for x in range(n - 600 if n > 600 else 0, n + 1):
            assert lib.bjx_test_block_first(0, n, x, 256) == min(x, n)
