"""Planted-relation Zipf corpora as token ids (vectorised numpy), for the
large-scale quality gates and studies: the text8-like corpus of
tests/quality.py (planted_zipf_corpus: Zipf filler, entity / topic / role words
of a (row, col) grid planted at mid frequency) at sizes where Python strings
would not fit, plus the reference's build_vocab / build_sample on ids
(Word2Vec.cpp:132-169, 212-230: count, drop < min_count, sort by count
descending, drop OOV tokens) and the analogy / similarity scorer.

Test infrastructure: used by tests/golden/gen_headline_planted_golden.py (the
sequential oracle's scores at configs[2]'s scale), tests/test_gpu_quality.py
(the GPU side of that gate) and tools/replica_study.py."""
from __future__ import annotations

import numpy as np


def planted_zipf_ids(n_tokens, sent_len=1000, filler=100_000, rows=50, cols=4, topic=8, role=8, planted_frac=0.10,
                     seed=0, zipf_s=1.0, zipf_q=0.0):
    """Raw ids: filler ids [0, filler) drawn from p(r) ~ (r + q)^-s (r = 1 ..
    filler), then entities, topics, roles. Returns (tok int64, n_sent, names,
    questions, pairs)."""
    rng = np.random.default_rng(seed)
    n_sent = n_tokens // sent_len
    E0 = filler
    T0 = E0 + rows * cols
    R0 = T0 + rows * topic
    n_raw = R0 + cols * role
    if zipf_s == 1.0 and zipf_q == 0.0:
        p = 1.0 / np.arange(1, filler + 1)  # the round-3 probes' corpus, bit for bit
    else:
        p = (np.arange(1, filler + 1) + zipf_q) ** -zipf_s
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    tok = np.empty(n_sent * sent_len, np.int64)
    chunk = 1 << 24
    for s in range(0, tok.size, chunk):  # the same draws as one call, in bounded memory
        e = min(tok.size, s + chunk)
        tok[s:e] = np.searchsorted(cdf, rng.random(e - s), side="right")
    np.clip(tok, 0, filler - 1, out=tok)
    si = rng.integers(rows, size=n_sent)
    sj = rng.integers(cols, size=n_sent)
    pos = np.flatnonzero(rng.random(n_sent * sent_len) < planted_frac)
    s = pos // sent_len
    i, j = si[s], sj[s]
    kind = rng.random(pos.size)
    ent = kind < 0.34
    top = (kind >= 0.34) & (kind < 0.67)
    rol = kind >= 0.67
    # entity: the sentence's (i, j) w.p. 0.75, else a same-row or same-column neighbour
    r1 = rng.random(pos.size)
    r2 = rng.random(pos.size)
    ei, ej = i.copy(), j.copy()
    cross = r1 <= 0.25
    rowx = cross & (r2 < 0.5)
    colx = cross & (r2 >= 0.5)
    ej[rowx] = rng.integers(cols, size=int(rowx.sum()))
    ei[colx] = rng.integers(rows, size=int(colx.sum()))
    out = np.empty(pos.size, np.int64)
    out[ent] = E0 + ei[ent] * cols + ej[ent]
    out[top] = T0 + i[top] * topic + rng.integers(topic, size=int(top.sum()))
    out[rol] = R0 + j[rol] * role + rng.integers(role, size=int(rol.sum()))
    tok[pos] = out
    names = ([f"f{k}" for k in range(filler)] + [f"e{a}_{b}" for a in range(rows) for b in range(cols)]
             + [f"t{a}_{k}" for a in range(rows) for k in range(topic)]
             + [f"r{b}_{k}" for b in range(cols) for k in range(role)])
    assert len(names) == n_raw
    qs = [(f"e{a}_{l}", f"e{a}_{b}", f"e{c}_{l}", f"e{c}_{b}") for a in range(rows) for c in range(rows) if a != c
          for b in range(cols) for l in range(cols) if b != l]
    prs = []
    for a in range(rows):
        for b in range(cols):
            for c in range(rows):
                for d in range(cols):
                    if (a, b) < (c, d) and rng.random() < 0.05:
                        prs.append((f"e{a}_{b}", f"e{c}_{d}", float((a == c) + (b == d))))
    return tok, n_sent, names, qs, prs


def build(tok, n_sent, sent_len, names, min_count=5):
    """build_vocab + build_sample on raw ids: (ids int32, sentence offsets int64,
    counts int64 in vocab order, words). Ties keep the raw id order (a stable
    sort; the ids are not strings, so the reference's hash-map tie order does
    not apply — the gates compare runs that share this vocabulary)."""
    counts = np.bincount(tok, minlength=len(names))
    order = np.argsort(-counts, kind="stable")
    V = int((counts >= min_count).sum())
    vr = order[:V]
    remap = np.full(len(names), -1, np.int64)
    remap[vr] = np.arange(V)
    ids = remap[tok]
    keep = ids >= 0
    lens = keep.reshape(n_sent, sent_len).sum(1)
    soff = np.zeros(n_sent + 1, np.int64)
    soff[1:] = np.cumsum(lens)
    return ids[keep].astype(np.int32), soff, counts[vr].astype(np.int64), [names[k] for k in vr]


def scores(words, E, qs, prs, dev=None, chunk=4096):
    """(3CosAdd analogy accuracy, Spearman similarity x 100) with torch on `dev`
    (cuda for the large vocabularies; cpu with a small `chunk` in the container)."""
    import torch

    from word2vec_amd.evaluate import similarity_score

    dev = dev or torch.device("cpu")
    idx = {w: k for k, w in enumerate(words)}
    En = torch.tensor(np.ascontiguousarray(E), device=dev)
    En = En / En.norm(dim=1, keepdim=True).clamp_min(1e-12)
    Q = torch.tensor([[idx[x] for x in q] for q in qs if all(x in idx for x in q)], device=dev)
    correct = 0
    for s in range(0, Q.shape[0], chunk):
        qa, qb, qc, qd = Q[s:s + chunk].T
        sims = (En[qb] - En[qa] + En[qc]) @ En.T
        r = torch.arange(qa.numel(), device=dev)
        for ex in (qa, qb, qc):
            sims[r, ex] = -float("inf")
        correct += int((sims.argmax(1) == qd).sum())
        del sims
    return 100.0 * correct / max(1, Q.shape[0]), similarity_score(words, E, prs)["spearman"]


def gpu_trainer(counts, ids, soff, raw, mode, dim, negative, alpha, W0, C0, S0, key, window=5, subsample=1e-4,
                table_size=100_000_000, iters=1, device=0, upload_corpus=True):
    """A DeviceTrainer (the C-ABI) for an id corpus, in the shipped throughput
    configuration: Philox, the parallel schedule, the library's default update
    policy (automatic hot rows, LDS-private rows, segments)."""
    from word2vec_amd import _native as N
    from word2vec_amd import host
    from word2vec_amd.device import Config, DeviceTrainer

    hs, cbow = mode.endswith("hs"), mode.startswith("cbow")
    keep = host.sample_probs(counts, subsample)
    bounds = host.table_bounds(counts, table_size) if negative else None
    codes = points = coff = None
    if hs:
        codes, points, coff = host.huffman(counts)
    cfg = Config(word_dim=dim, window=window, negative=negative, hs=hs, cbow=cbow, cbow_mean=True, iter=iters,
                 init_alpha=alpha, min_alpha=2.5e-6, table_size=table_size, device=device)
    t = DeviceTrainer(cfg)
    t.upload_vocab(keep, bounds, codes, points, coff)
    t.upload_model(W0, C0 if (negative or cbow) else None, S0)
    if upload_corpus:
        t.upload_corpus(ids, soff, int(raw))
    t.set_rng(N.W2V_RNG_PHILOX, key)
    t.set_schedule(N.W2V_SCHED_PARALLEL)
    t.set_progress(0)
    return t
