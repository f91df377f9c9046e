"""Word-vector evaluation: analogy (3CosAdd) and word similarity (Spearman).

The reference has no evaluator; the north star's third
correctness level compares analogy / similarity scores with the reference's.
Formats: analogy questions as in word2vec's questions-words.txt (": section"
headers, then "a b c d" lines: a is to b as c is to d); similarity pairs as
"word1 word2 score" lines (WordSim-353 / SimLex style). Questions with a word
outside the vocabulary are skipped and counted, as word2vec's compute-accuracy
does.
"""
from __future__ import annotations

import numpy as np


def normalize(vecs: np.ndarray) -> np.ndarray:
    v = np.asarray(vecs, dtype=np.float32)
    n = np.linalg.norm(v, axis=1, keepdims=True)
    return v / np.maximum(n, 1e-12)


def read_analogies(path) -> list[tuple[str, str, str, str]]:
    out = []
    for line in open(path, encoding="utf-8", errors="replace"):
        if line.startswith(":") or not line.strip():
            continue
        a, b, c, d = line.split()[:4]
        out.append((a, b, c, d))
    return out


def read_similarity(path) -> list[tuple[str, str, float]]:
    out = []
    for line in open(path, encoding="utf-8", errors="replace"):
        p = line.split()
        if len(p) < 3 or p[0].startswith("#"):
            continue
        try:
            out.append((p[0], p[1], float(p[2])))
        except ValueError:
            continue
    return out


def analogy_accuracy(words: list[str], vecs: np.ndarray, questions, restrict: int | None = None,
                     lowercase: bool = False, batch: int = 1024) -> dict:
    """3CosAdd: argmax_x cos(x, b - a + c) over the vocabulary (the first
    `restrict` words if given), excluding a, b, c. Returns accuracy in percent."""
    idx = {}
    for i, w in enumerate(words):
        idx.setdefault(w.lower() if lowercase else w, i)
    E = normalize(vecs)
    cand = E if restrict is None else E[:restrict]
    q = []
    for a, b, c, d in questions:
        key = [x.lower() if lowercase else x for x in (a, b, c, d)]
        ids = [idx.get(k) for k in key]
        if any(i is None for i in ids) or (restrict is not None and any(i >= restrict for i in ids)):
            continue
        q.append(ids)
    if not q:
        return {"accuracy": 0.0, "correct": 0, "answered": 0, "skipped": len(questions)}
    Q = np.array(q, dtype=np.int64)
    correct = 0
    for s in range(0, len(Q), batch):
        qa, qb, qc, qd = Q[s:s + batch].T
        target = E[qb] - E[qa] + E[qc]
        sims = target @ cand.T
        rows = np.arange(len(qa))
        for excl in (qa, qb, qc):
            ok = excl < cand.shape[0]
            sims[rows[ok], excl[ok]] = -np.inf
        best = sims.argmax(axis=1)
        answerable = np.isfinite(sims[rows, best])  # every candidate excluded -> wrong
        correct += int(((best == qd) & answerable).sum())
    return {"accuracy": 100.0 * correct / len(Q), "correct": correct, "answered": int(len(Q)),
            "skipped": len(questions) - int(len(Q))}


def _rank(x: np.ndarray) -> np.ndarray:
    order = np.argsort(x, kind="mergesort")
    r = np.empty(len(x), dtype=np.float64)
    xs = x[order]
    i = 0
    while i < len(x):  # average ranks for ties
        j = i
        while j + 1 < len(x) and xs[j + 1] == xs[i]:
            j += 1
        r[order[i:j + 1]] = (i + j) / 2.0 + 1
        i = j + 1
    return r


def spearman(a, b) -> float:
    ra, rb = _rank(np.asarray(a, np.float64)), _rank(np.asarray(b, np.float64))
    ra -= ra.mean()
    rb -= rb.mean()
    den = np.sqrt((ra * ra).sum() * (rb * rb).sum())
    return float((ra * rb).sum() / den) if den > 0 else 0.0


def similarity_score(words: list[str], vecs: np.ndarray, pairs, lowercase: bool = False) -> dict:
    """Spearman correlation (x100) between cosine similarity and the gold scores."""
    idx = {}
    for i, w in enumerate(words):
        idx.setdefault(w.lower() if lowercase else w, i)
    E = normalize(vecs)
    got, gold = [], []
    for w1, w2, s in pairs:
        k1, k2 = (w1.lower(), w2.lower()) if lowercase else (w1, w2)
        if k1 in idx and k2 in idx:
            got.append(float(E[idx[k1]] @ E[idx[k2]]))
            gold.append(s)
    if len(got) < 2:
        return {"spearman": 0.0, "pairs": len(got), "skipped": len(pairs) - len(got)}
    return {"spearman": 100.0 * spearman(got, gold), "pairs": len(got), "skipped": len(pairs) - len(got)}


def read_word2vec_text(path) -> tuple[list[str], np.ndarray]:
    """Read the text format save_word2vec writes (Word2Vec.cpp:428-436)."""
    with open(path, encoding="utf-8", errors="replace") as f:
        rows, cols = map(int, f.readline().split())
        words, vecs = [], np.zeros((rows, cols), np.float32)
        for i, line in enumerate(f):
            p = line.rstrip("\n").split(" ")
            words.append(p[0])
            vecs[i] = np.array(p[1:1 + cols], dtype=np.float32)
    return words, vecs
