"""CPU: the drop-in cache's keyed digest (csrc/dropin_digest.hpp) built for the
host with g++ and checked against a Python restatement of its definition
(NH blocks of 64 words, two Horner layers in GF(2^127 - 1)); a one-word change
of the input changes both halves; two freshly drawn keys differ."""
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "digest_check.cpp")
P127 = (1 << 127) - 1
M64 = (1 << 64) - 1


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("digest") / "digest_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-w", "-o", out, SRC], check=True)
    return out


def run(exe, lines):
    out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True).stdout
    return out.split("\n")[:-1]


def splitmix(state):
    state = (state + 0x9E3779B97F4A7C15) & M64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return state, z ^ (z >> 31)


def py_digest(seed, words, chunk):
    s = seed
    nh = []
    for _ in range(66):
        s, w = splitmix(s)
        nh.append(w)
    kb, kc = [], []
    for _ in range(2):
        s, hi = splitmix(s)
        s, lo = splitmix(s)
        kb.append(((hi << 64) | lo) & P127)
        s, hi = splitmix(s)
        s, lo = splitmix(s)
        kc.append(((hi << 64) | lo) & P127)
    parts = []
    for c0 in range(0, len(words), chunk):
        cw = words[c0:c0 + chunk]
        acc = [1, 1]
        for b in range(0, len(cw), 64):
            blk = cw[b:b + 64] + [0] * (64 - len(cw[b:b + 64]))
            for j in range(2):
                h = 0
                for i in range(0, 64, 2):
                    h += ((blk[i] + nh[i + 2 * j]) & M64) * ((blk[i + 1] + nh[i + 1 + 2 * j]) & M64)
                h &= (1 << 128) - 1
                acc[j] = (acc[j] * kb[j] + h) % P127
        parts.append(acc)
    d = [1, 1]
    for p in parts:
        for j in range(2):
            d[j] = (d[j] * kc[j] + p[j]) % P127
    return d


def test_mulmod127(exe):
    rng = random.Random(127)
    pairs = [(0, 0), (1, P127 - 1), (P127 - 1, P127 - 1), ((1 << 126), 2), ((1 << 64) - 1, (1 << 64) + 1)]
    pairs += [(rng.randrange(P127), rng.randrange(P127)) for _ in range(500)]
    rows = run(exe, ["mul %x %x" % ab for ab in pairs])
    for (a, b), row in zip(pairs, rows):
        assert int(row, 16) == a * b % P127, (a, b)


@pytest.mark.parametrize("nwords,chunk", [(8, 64), (64, 64), (200, 64), (1000, 256), (4096 + 8, 1024)])
def test_digest_matches_definition(exe, nwords, chunk):
    seed, wseed = 0xD16E57 + nwords, 0x5EED + chunk
    rows = run(exe, ["digest %d %d %d %d" % (seed, nwords, chunk, wseed)])
    s, words = wseed, []
    for _ in range(nwords):
        s, w = splitmix(s)
        words.append(w)
    d0, d1 = (int(x, 16) for x in rows[0].split())
    assert [d0, d1] == py_digest(seed, words, chunk)


def test_other_words_change_both_halves(exe):
    """Different word seeds (every word different) and the same key: the
    digests differ in both halves; the same inputs give the same digest."""
    rows = run(exe, ["digest 7 4096 1024 1", "digest 7 4096 1024 1", "digest 7 4096 1024 2"])
    assert rows[0] == rows[1]
    a, b = rows[0].split(), rows[2].split()
    assert a[0] != b[0] and a[1] != b[1]


def test_keys_are_random(exe):
    """Each context draws its own key from the OS RNG: two draws differ."""
    a, b = run(exe, ["rand"])[0].split()
    assert a != b
