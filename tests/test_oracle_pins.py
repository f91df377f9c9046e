"""Pin the CPU oracle (oracle/w2v_oracle.cpp) before trusting it.

The reference is unbuildable here (needs Eigen) and ships no tests, so the
oracle is pinned against (a) libstdc++ itself — golden vectors produced by
tests/golden/gen_libstdcxx_golden.cpp, the library the reference delegates
its RNG / shuffle / heap / sort / hash-map behaviour to — and (b) independent
Python restatements (tests/refpy.py) of the reference's float arithmetic and
draw order. CPU only.
"""
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import Oracle, philox
from tests import refpy
from tests.corpus import zipf_sentences
from tests.harness import MODES, oracle_run

G = json.loads((Path(__file__).parent / "golden" / "libstdcxx_golden.json").read_text())


def test_mt19937_restatement_matches_libstdcxx():
    g = refpy.MT19937(1234)
    assert [g() for _ in range(2000)] == G["mt19937_seed1234"]


def test_canonical_float_matches_uniform_real():
    g = refpy.MT19937(77)
    got = [int(refpy.uniform_real(g, 0.0, 1.0).view(np.uint32)) for _ in range(2000)]
    assert got == G["uniform01_seed77_bits"]


def test_init_weights_distribution_bits():
    g = refpy.MT19937(5)
    got = [int(np.float32(refpy.uniform_real(g, -0.5, 0.5) / np.float32(7)).view(np.uint32)) for _ in range(700)]
    assert got == G["init_weights_seed5_dim7_bits"]


def test_lemire_uniform_int_matches_libstdcxx():
    g = refpy.MT19937(99)
    a = [refpy.uniform_int(g, 0, 4) for _ in range(2000)]
    b = [refpy.uniform_int(g, 0, 100_000_000 - 1) for _ in range(2000)]
    assert a == G["window5_seed99"]
    assert b == G["table1e8_after_window_seed99"]


@pytest.mark.parametrize("n", [1, 2, 17, 1000, 70000])
def test_shuffle_matches_libstdcxx(n):
    g = refpy.MT19937(2024)
    assert refpy.shuffle(list(range(n)), g) == G[f"shuffle_n{n}_seed2024"]
    assert g() == G[f"shuffle_n{n}_seed2024_next_draw"][0]


def test_oracle_vocab_order_matches_libstdcxx_pointer_sort():
    toks = G["vocab_tokens_seed3"]
    o = Oracle(min_count=5, word_dim=4, negative=0, train_method="hs", model="cbow")
    o.load_sentences([toks])
    o.build_vocab()
    words, counts = o.vocab()
    want = G["vocab_order_seed3"]
    assert words == [w for w, _ in want]
    assert counts.tolist() == [c for _, c in want]


@pytest.mark.parametrize("key", ["", "_eq33"])
def test_oracle_huffman_matches_pointer_heap(key):
    counts = G["huffman_counts"] if key == "" else [4] * 33
    o = Oracle(min_count=1, word_dim=4, negative=0, train_method="hs", model="cbow")
    o.set_vocab_counts(np.array(counts))
    codes, points, off = o.huffman()
    assert codes.tolist() == G[f"huffman{key}_codes"]
    assert points.tolist() == G[f"huffman{key}_points"]
    assert off.tolist() == G[f"huffman{key}_offsets"]


@pytest.mark.parametrize("seed,vmax,ts", [(1, 300, 20_000), (2, 50, 3_000), (3, 2000, 50_000), (4, 3, 10)])
def test_oracle_table_and_probs_match_float32_restatement(seed, vmax, ts):
    sents = zipf_sentences(30, 300, vmax, seed=seed)
    o = oracle_run(sents, "sg_ns", table_size=ts, min_count=1, train=False, subsample=1e-3)
    _, counts = o.vocab()
    np.testing.assert_array_equal(o.table(), refpy.make_table(counts.tolist(), ts))
    np.testing.assert_array_equal(o.sample_probs().view(np.uint32),
                                  refpy.sample_probs(counts.tolist(), 1e-3).view(np.uint32))


def test_sample_probs_disabled_is_one():
    sents = zipf_sentences(5, 100, 30, seed=2)
    o = oracle_run(sents, "sg_ns", min_count=1, train=False, subsample=0.0, table_size=1000)
    assert (o.sample_probs() == 1.0).all()


@pytest.mark.parametrize("mode", list(MODES))
def test_oracle_records_the_reference_draw_order(mode):
    """The oracle's recorded stream equals an independent restatement of the
    reference's draw order on the same mt19937 (init_weights x2, shuffle, then
    the sentence loop)."""
    sents = zipf_sentences(7, 60, 40, seed=4, ragged=True)
    dim, window, ts, seed = 6, 3, 5000, 99
    o = oracle_run(sents, mode, dim=dim, window=window, iters=1, table_size=ts, min_count=1, seed=seed)
    stream, offs, orders = o.stream(1)
    ids, off = o.samples()
    V = o.V
    g = refpy.MT19937(seed)
    m = MODES[mode]
    n_init = V * dim * (2 if (m["model"] == "cbow" and m["train_method"] == "hs") else 1)
    for _ in range(2 * n_init):  # main.cpp:190 and Word2Vec.cpp:358
        g()
    order = refpy.shuffle(list(range(off.size - 1)), g)
    assert orders.tolist() == order
    draws = refpy.reference_draws(ids, off, o.sample_probs(), order, window, m["negative"], ts, m["model"], g)
    assert [v for _, v in draws] == stream.tolist()


@pytest.mark.parametrize("ctr,key,out", refpy.PHILOX_KAT)
def test_philox_known_answers(ctr, key, out):
    assert refpy.philox4x32_10(ctr, key) == out
    k64 = key[0] | (key[1] << 32)
    assert tuple(philox(np.array(ctr, np.uint32), k64).tolist()) == out


def test_philox_oracle_matches_python_random_counters():
    rng = np.random.default_rng(0)
    for _ in range(50):
        ctr = tuple(int(x) for x in rng.integers(0, 2**32, 4))
        key = tuple(int(x) for x in rng.integers(0, 2**32, 2))
        k64 = key[0] | (key[1] << 32)
        assert tuple(philox(np.array(ctr, np.uint32), k64).tolist()) == refpy.philox4x32_10(ctr, key)


@pytest.mark.parametrize("mode", list(MODES))
def test_oracle_replay_reproduces_reference_mode(mode):
    sents = zipf_sentences(9, 150, 300, seed=6, ragged=True)
    o = oracle_run(sents, mode, dim=24, iters=2)
    s, off, orders = o.stream(2)
    fin = [o.matrix(k) for k in range(3)]
    ini = [o.matrix(k, True) for k in range(3)]
    cw = o.current_words
    for k in range(3):
        if ini[k].size:
            o.set_matrix(k, ini[k])
    o.train_replay(2, orders, s, off, 0)
    assert o.current_words == cw
    for k in range(3):
        np.testing.assert_array_equal(o.matrix(k), fin[k])
    # the model actually moved
    assert any(np.abs(fin[k] - ini[k]).max() > 0 for k in range(3) if fin[k].size)
