"""The evaluator (word2vec_amd/evaluate.py) on hand-made vectors; Spearman vs scipy."""
import numpy as np
import pytest
from scipy.stats import spearmanr

from word2vec_amd.evaluate import (analogy_accuracy, read_analogies, read_similarity, read_word2vec_text,
                                   similarity_score, spearman)


def test_analogy_on_additive_vectors():
    rng = np.random.default_rng(0)
    rows, cols, d = 6, 3, 32
    R, Cc = rng.standard_normal((rows, d)), rng.standard_normal((cols, d))
    words, vecs = [], []
    for i in range(rows):
        for j in range(cols):
            words.append(f"e{i}_{j}")
            vecs.append(R[i] + Cc[j])
    words.append("noise")
    vecs.append(rng.standard_normal(d))
    qs = [(f"e{i}_{l}", f"e{i}_{j}", f"e{k}_{l}", f"e{k}_{j}") for i in range(rows) for k in range(rows) if i != k
          for j in range(cols) for l in range(cols) if j != l]
    qs.append(("e0_0", "e0_1", "missing", "e1_1"))
    r = analogy_accuracy(words, np.array(vecs), qs)
    assert r["accuracy"] == 100.0 and r["skipped"] == 1 and r["answered"] == len(qs) - 1
    # the answer may never be one of the question words
    r2 = analogy_accuracy(["a", "b", "c"], np.eye(3), [("a", "b", "c", "a")])
    assert r2["accuracy"] == 0.0
    r3 = analogy_accuracy(["a", "b", "c", "d"], np.eye(4), [("a", "b", "c", "a")])
    assert r3["accuracy"] == 0.0


def test_spearman_matches_scipy():
    rng = np.random.default_rng(1)
    for _ in range(20):
        a = rng.integers(0, 5, 30).astype(float)
        b = a + rng.standard_normal(30)
        assert abs(spearman(a, b) - spearmanr(a, b).correlation) < 1e-9


def test_similarity_and_file_formats(tmp_path):
    words = ["x", "y", "z"]
    vecs = np.array([[1, 0], [0.9, 0.1], [0, 1]], np.float32)
    pairs = [("x", "y", 9.0), ("x", "z", 1.0), ("y", "z", 2.0), ("x", "q", 5.0)]
    s = similarity_score(words, vecs, pairs)
    assert s["pairs"] == 3 and s["skipped"] == 1 and s["spearman"] == pytest.approx(100.0)
    (tmp_path / "q.txt").write_text(": capital\nA B C D\nE F G H\n")
    assert read_analogies(tmp_path / "q.txt") == [("A", "B", "C", "D"), ("E", "F", "G", "H")]
    (tmp_path / "s.txt").write_text("# comment\nx y 3.5\nbad line\nx z 1\n")
    assert read_similarity(tmp_path / "s.txt") == [("x", "y", 3.5), ("x", "z", 1.0)]
    (tmp_path / "v.txt").write_text("2 3\nfoo 1 2 3\nbar -1 0.5 1e-05\n")
    w, v = read_word2vec_text(tmp_path / "v.txt")
    assert w == ["foo", "bar"] and np.allclose(v, [[1, 2, 3], [-1, 0.5, 1e-5]])
