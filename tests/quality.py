"""A synthetic planted-relation corpus for the end-to-end quality gate.

No real analogy or similarity set (questions-words.txt, WordSim) or text8 is
available offline, so relations are planted: entity e_{i,j} (row i = a
"category", column j = a "role") appears with topic words of row i and role
words of column j, inside Zipf filler. Embeddings that capture the
co-occurrence structure become approximately additive (row + column), which
makes e_{i,j} - e_{i,l} + e_{k,l} ≈ e_{k,j} the analogy to solve, and puts
same-row / same-column entity pairs closer together (the similarity gold).
Noise (filler, cross-talk) keeps accuracy away from 100 % so the gate is
sensitive.
"""
from __future__ import annotations

import numpy as np


def planted_corpus(n_sent=3000, sent_len=200, rows=30, cols=4, topic_per_row=6, role_per_col=6,
                   filler=3000, p_entity=0.08, p_topic=0.22, p_role=0.22, p_cross=0.1, seed=0):
    rng = np.random.default_rng(seed)
    ent = [[f"e{i}_{j}" for j in range(cols)] for i in range(rows)]
    topic = [[f"t{i}_{k}" for k in range(topic_per_row)] for i in range(rows)]
    role = [[f"r{j}_{k}" for k in range(role_per_col)] for j in range(cols)]
    fw = np.array([f"f{k}" for k in range(filler)])
    pz = 1.0 / np.arange(1, filler + 1)
    pz /= pz.sum()
    sents = []
    for _ in range(n_sent):
        i, j = rng.integers(rows), rng.integers(cols)
        u = rng.random(sent_len)
        fill = rng.choice(fw, size=sent_len, p=pz)
        s = []
        for t in range(sent_len):
            x = u[t]
            if x < p_entity:
                # the sentence's entity, sometimes a same-row or same-column neighbour
                if rng.random() < p_cross:
                    s.append(ent[i][rng.integers(cols)] if rng.random() < 0.5 else ent[rng.integers(rows)][j])
                else:
                    s.append(ent[i][j])
            elif x < p_entity + p_topic:
                s.append(topic[i][rng.integers(topic_per_row)])
            elif x < p_entity + p_topic + p_role:
                s.append(role[j][rng.integers(role_per_col)])
            else:
                s.append(str(fill[t]))
        sents.append(s)
    questions = []
    for i in range(rows):
        for k in range(rows):
            if i == k:
                continue
            for j in range(cols):
                for l in range(cols):
                    if j != l:
                        questions.append((ent[i][l], ent[i][j], ent[k][l], ent[k][j]))
    pairs = []
    for a in range(rows):
        for b in range(cols):
            for c in range(rows):
                for d in range(cols):
                    if (a, b) < (c, d) and rng.random() < 0.15:
                        pairs.append((ent[a][b], ent[c][d], float((a == c) + (b == d))))
    return sents, questions, pairs


def planted_zipf_corpus(n_tokens=10_000_000, sent_len=1000, filler=100_000, rows=50, cols=4, topic_per_row=8,
                        role_per_col=8, planted_frac=0.25, seed=0):
    """Text8-like statistics: Zipf(s=1) filler over `filler` word types (the
    function words are the hottest rows), 1000-token sentences, and the planted
    relations of planted_corpus() embedded at mid frequency: in each sentence a
    fraction `planted_frac` of positions carries the sentence's (row, col)
    entity / topic / role words, spread through the filler."""
    rng = np.random.default_rng(seed)
    n_sent = n_tokens // sent_len
    ent = np.array([[f"e{i}_{j}" for j in range(cols)] for i in range(rows)])
    topic = np.array([[f"t{i}_{k}" for k in range(topic_per_row)] for i in range(rows)])
    role = np.array([[f"r{j}_{k}" for k in range(role_per_col)] for j in range(cols)])
    p = 1.0 / np.arange(1, filler + 1)
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    fill_ids = np.searchsorted(cdf, rng.random(n_sent * sent_len), side="right").clip(0, filler - 1)
    sents = []
    for s in range(n_sent):
        toks = [f"f{x}" for x in fill_ids[s * sent_len:(s + 1) * sent_len]]
        i, j = rng.integers(rows), rng.integers(cols)
        pos = np.flatnonzero(rng.random(sent_len) < planted_frac)
        kind = rng.random(pos.size)
        for q, kk in zip(pos, kind):
            if kk < 0.34:
                toks[q] = ent[i, j] if rng.random() > 0.25 else (ent[i, rng.integers(cols)] if rng.random() < 0.5
                                                                  else ent[rng.integers(rows), j])
            elif kk < 0.67:
                toks[q] = topic[i, rng.integers(topic_per_row)]
            else:
                toks[q] = role[j, rng.integers(role_per_col)]
        sents.append(toks)
    questions = [(ent[i, l], ent[i, j], ent[k, l], ent[k, j]) for i in range(rows) for k in range(rows) if i != k
                 for j in range(cols) for l in range(cols) if j != l]
    pairs = []
    for a in range(rows):
        for b in range(cols):
            for c in range(rows):
                for d in range(cols):
                    if (a, b) < (c, d) and rng.random() < 0.05:
                        pairs.append((ent[a, b], ent[c, d], float((a == c) + (b == d))))
    return sents, questions, pairs
