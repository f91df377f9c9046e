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


_ROWS, _COLS, _TOPIC, _ROLE = 50, 4, 8, 8  # planted_zipf_ids' grid


def _chunks(n_tokens, filler, planted, seed, dev, sent_len, chunk=1 << 26, planted_sents=1.0):
    """The raw ids of the corpus, chunk by chunk (deterministic in `seed`);
    only a fraction `planted_sents` of the sentences carry planted words (at
    `planted` of their positions: the relations stay dense inside windows
    while the corpus's planted total shrinks)."""
    import torch

    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    n_sent = n_tokens // sent_len
    n = n_sent * sent_len
    E0 = filler
    T0 = E0 + _ROWS * _COLS
    R0 = T0 + _ROWS * _TOPIC
    p = torch.arange(1, filler + 1, device=dev, dtype=torch.float64).reciprocal_()
    cdf = torch.cumsum(p, 0)
    cdf /= cdf[-1].clone()
    si = torch.randint(_ROWS, (n_sent,), generator=g, device=dev)
    sj = torch.randint(_COLS, (n_sent,), generator=g, device=dev)
    sp = (torch.rand(n_sent, generator=g, device=dev) < planted_sents) if planted_sents < 1.0 else None
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        m = e - s
        tok = torch.searchsorted(cdf, torch.rand(m, generator=g, device=dev, dtype=torch.float64), right=True)
        tok.clamp_(max=filler - 1)
        pick = torch.rand(m, generator=g, device=dev) < planted
        if sp is not None:
            pick &= sp[(torch.arange(s, e, device=dev) // sent_len)]
        pos = torch.nonzero(pick).squeeze(1)
        k = pos.numel()
        sent = (pos + s) // sent_len
        i, j = si[sent], sj[sent]
        kind = torch.rand(k, generator=g, device=dev)
        r1 = torch.rand(k, generator=g, device=dev)
        r2 = torch.rand(k, generator=g, device=dev)
        ri = torch.randint(_ROWS, (k,), generator=g, device=dev)
        rj = torch.randint(_COLS, (k,), generator=g, device=dev)
        rt = torch.randint(_TOPIC, (k,), generator=g, device=dev)
        rr = torch.randint(_ROLE, (k,), generator=g, device=dev)
        cross = r1 <= 0.25
        ei = torch.where(cross & (r2 >= 0.5), ri, i)
        ej = torch.where(cross & (r2 < 0.5), rj, j)
        tok[pos] = torch.where(kind < 0.34, E0 + ei * _COLS + ej,
                               torch.where(kind < 0.67, T0 + i * _TOPIC + rt, R0 + j * _ROLE + rr))
        yield s, e, tok


def planted_zipf_ids_torch(n_tokens, filler, planted, seed, dev, sent_len=1000, planted_sents=1.0):
    """planted_zipf_ids' law (Zipf(s=1) filler, the 50 x 4 planted grid) drawn
    with torch on `dev` (the GPU: 10 B tokens in seconds; not the same draws as
    the numpy generator), every rank in vocab (asserted: no OOV, so every
    sentence keeps its sent_len tokens). Two passes over the same draws (count,
    then map to vocab indices in count order): (ids int32 [n_sent, sent_len] on
    the host, counts int64 in vocab order, words, questions, pairs, raw
    tokens)."""
    import torch

    n_raw = filler + _ROWS * _COLS + _ROWS * _TOPIC + _COLS * _ROLE
    counts = torch.zeros(n_raw, dtype=torch.int64, device=dev)
    n = 0
    for s, e, tok in _chunks(n_tokens, filler, planted, seed, dev, sent_len, planted_sents=planted_sents):
        counts += torch.bincount(tok, minlength=n_raw)
        n = e
    counts_h = counts.cpu().numpy()
    order = np.argsort(-counts_h, kind="stable")
    V = int((counts_h >= 5).sum())
    assert V == n_raw, f"{n_raw - V} word types below min_count: the study assumes no OOV"
    remap = np.empty(n_raw, np.int32)
    remap[order] = np.arange(n_raw, dtype=np.int32)
    remap_d = torch.from_numpy(remap).to(dev)
    ids = np.empty(n, np.int32)
    for s, e, tok in _chunks(n_tokens, filler, planted, seed, dev, sent_len, planted_sents=planted_sents):
        ids[s:e] = remap_d[tok].cpu().numpy()
    names = ([f"f{k}" for k in range(filler)] + [f"e{a}_{b}" for a in range(_ROWS) for b in range(_COLS)]
             + [f"t{a}_{k}" for a in range(_ROWS) for k in range(_TOPIC)]
             + [f"r{b}_{k}" for b in range(_COLS) for k in range(_ROLE)])
    words = [names[k] for k in order]
    rng = np.random.default_rng(seed)
    qs = [(f"e{a}_{l}", f"e{a}_{b}", f"e{c}_{l}", f"e{c}_{b}") for a in range(_ROWS) for c in range(_ROWS) if a != c
          for b in range(_COLS) for l in range(_COLS) if b != l]
    prs = [(f"e{a}_{b}", f"e{c}_{d}", float((a == c) + (b == d))) for a in range(_ROWS) for b in range(_COLS)
           for c in range(_ROWS) for d in range(_COLS) if (a, b) < (c, d) and rng.random() < 0.05]
    return ids.reshape(-1, sent_len), counts_h[order].astype(np.int64), words, qs, prs, n


def train_replicas(data, R, gmode, rounds, dim=300, negative=5, mode="sg_ns", seed=1, dev=None):
    """One epoch of `data` (planted_zipf_ids_torch) by R replicas on one
    device (a same-device w2v_group: every replica a full-concurrency training
    handle, as on R GPUs; replica r trains the r-th contiguous 1/R of the
    shuffled sentence order as its own corpus, its counter following the
    global alpha schedule) exchanging `rounds` times per epoch in `gmode`
    (auto = Word2Vec::replica_mode's: average for <= 4 replicas of long shards, else sum for 2, adaptive for more; sat<beta> =
    W2V_GROUP_SATURATION; overlapped as the class does), or by one replica
    (R = 1). mode sg_ns or sg_sn (the
    shared-negatives minibatch). Returns ((analogy, similarity) of W or None
    if it diverged, train seconds)."""
    import time

    import torch

    from word2vec_amd import _native as N
    from word2vec_amd.replicas import NativeAverager

    ids, counts, words, qs, prs, raw = data
    n_sent, L = ids.shape
    V, d = counts.size, dim
    rng = np.random.default_rng(seed)
    W0 = ((rng.random((V, d), dtype=np.float32) - 0.5) / d).astype(np.float32)
    C0 = np.zeros((V, d), np.float32)
    perm = np.random.default_rng(1000 * seed).permutation(n_sent)
    key = (seed << 32) | 0x5EED
    reps = []
    for r in range(R):
        sh = np.sort(perm[n_sent * r // R: n_sent * (r + 1) // R])  # this replica's sentences (its own corpus)
        sid = ids.reshape(-1) if R == 1 else np.ascontiguousarray(ids[sh].reshape(-1))
        soff = np.arange(0, sh.size * L + 1, L, dtype=np.int64)
        t = gpu_trainer(counts, sid, soff, sh.size * L, "sg_ns", d, negative, 0.025, W0, C0, None, key + r)
        t.set_train_words(max(1, raw // R))
        if mode == "sg_sn":
            t.set_update(N.W2V_UPDATE_SHARED_NEGATIVES)
        t.set_order(perm.astype(np.int64) if R == 1 else
                    np.random.default_rng(7 + r).permutation(sh.size).astype(np.int64))
        reps.append((t, sh.size))
        del sid
    del W0, C0
    g = None
    if R > 1:
        # auto = Word2Vec::replica_mode (Word2Vec.cpp run_epochs_replicas): the mean for <= 4 replicas of
        # >= 64 x 4 M-word shards, else the sum for two, the adaptive divisor for more
        gm = (("average" if R <= 4 and raw // R >= 64 * 4_000_000 else "sum" if R <= 2 else "adaptive")
              if gmode == "auto" else gmode)
        if gm.startswith("sat"):  # sat<beta>: W2V_GROUP_SATURATION's per-row divisors
            g = NativeAverager([t for t, _ in reps], overlap=True, mode="sum")
            g.set_saturation(max(1, raw // R // rounds), float(gm[3:]))
        else:
            g = NativeAverager([t for t, _ in reps], overlap=True, mode=gm)
    torch.cuda.synchronize()
    t0 = time.time()
    glob = 0
    words_per_sent = L
    rounds = rounds if R > 1 else 1
    for r in range(rounds):
        wr = 0
        for t, m in reps:
            lo, hi = m * r // rounds, m * (r + 1) // rounds
            t.set_progress_async(glob // R)
            if hi > lo:
                t.train_slice_async(0, lo, hi - lo)
            wr += (hi - lo) * words_per_sent
        if g is not None:
            g.average()
        glob += wr
    if g is not None:
        g.finish()
    for t, _ in reps:
        t.synchronize()
    dt = time.time() - t0
    st = [t.read_stats() for t, _ in reps]
    diverged = any(s["nonfinite"] > 0 for s in st)
    W, _, _ = reps[0][0].download_model()
    if g is not None:
        g.close()
    for t, _ in reps:
        t.close()
    if diverged:
        return None, dt
    a, s = scores(words, W, qs, prs, dev)
    return (a, s), dt
