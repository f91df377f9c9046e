"""Host products that feed the device (libword2vec_amd.so, include/w2v_host.h)
are bit-exact with the oracle: table boundaries (make_table, Word2Vec.cpp:81-113),
subsampling probabilities (precalc_sampling, :115-130) and Huffman codes/points
(create_huffman_tree, :32-79). CPU only."""
import json
from pathlib import Path

import numpy as np
import pytest

from tests.corpus import zipf_sentences
from tests.harness import oracle_run
from word2vec_amd import host

G = json.loads((Path(__file__).parent / "golden" / "libstdcxx_golden.json").read_text())

CASES = [
    (1, 400, 100_000, 1e-3),
    (2, 3000, 1_000_000, 1e-4),
    (3, 20000, 100_000_000, 1e-4),  # the reference's default table size
    (4, 50, 1000, 1e-5),
    (5, 5000, 3000, 1e-3),  # table smaller than the vocab: trailing words get no entries
    (6, 2, 17, 0.0),
]


@pytest.mark.parametrize("seed,vmax,ts,sub", CASES)
def test_table_bounds_and_probs_bit_exact(seed, vmax, ts, sub):
    sents = zipf_sentences(40 if ts < 10**8 else 60, 1000, vmax, seed=seed)
    o = oracle_run(sents, "sg_ns", train=False, table_size=ts, subsample=sub, min_count=1 if vmax < 10 else 2)
    _, counts = o.vocab()
    b = host.table_bounds(counts, ts)
    np.testing.assert_array_equal(b, o.table_bounds())
    if ts <= 1_000_000:
        np.testing.assert_array_equal(host.table_fill(b, ts), o.table())
    else:  # 1e8: compare a hash of the expanded tables instead of holding both
        t_h, t_o = host.table_fill(b, ts), o.table()
        assert np.array_equal(t_h, t_o)
    np.testing.assert_array_equal(host.sample_probs(counts, sub).view(np.uint32), o.sample_probs().view(np.uint32))


@pytest.mark.parametrize("seed,vmax", [(1, 400), (2, 3000), (7, 40), (8, 5)])
def test_huffman_bit_exact(seed, vmax):
    sents = zipf_sentences(30, 500, vmax, seed=seed)
    o = oracle_run(sents, "cbow_hs", train=False, min_count=1)
    _, counts = o.vocab()
    for a, b in zip(host.huffman(counts), o.huffman()):
        np.testing.assert_array_equal(a, b)


def test_huffman_golden_ties():
    for key, counts in (("", G["huffman_counts"]), ("_eq33", [4] * 33)):
        codes, points, off = host.huffman(np.array(counts))
        assert codes.tolist() == G[f"huffman{key}_codes"]
        assert points.tolist() == G[f"huffman{key}_points"]
        assert off.tolist() == G[f"huffman{key}_offsets"]


def test_huffman_is_optimal_prefix_code():
    import heapq

    counts = np.array(sorted(np.random.default_rng(3).integers(1, 1000, 500).tolist(), reverse=True))
    codes, points, off = host.huffman(counts)
    depth = np.diff(off)
    # Kraft equality (full binary tree) and optimal weighted path length
    assert abs(sum(2.0 ** -d for d in depth) - 1.0) < 1e-12
    h = [int(c) for c in counts]
    heapq.heapify(h)
    cost = 0
    while len(h) > 1:
        a, b = heapq.heappop(h), heapq.heappop(h)
        cost += a + b
        heapq.heappush(h, a + b)
    assert int((depth * counts).sum()) == cost
    # every path starts at the root (point V-2) and points stay in range
    V = counts.size
    assert all(points[off[w]] == V - 2 for w in range(V))
    assert points.min() >= 0 and points.max() <= V - 2


def test_huffman_rejects_single_word():
    with pytest.raises(ValueError):
        host.huffman(np.array([5]))
