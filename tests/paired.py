"""Paired quality runs (north star level 3): the GPU and the
oracle train from the SAME initial weights on the SAME Philox draws (subsampling
decisions, window shrinks, negatives: a pure function of key, epoch, sentence,
position) over the SAME sentence order, so the only differences left are the
schedule (one wavefront vs the sequential oracle: fp32 summation order and the
LDS-aggregated flushes; full concurrency: Hogwild interleaving plus the update
policy). Seed-to-seed variance of the corpus (the oracle's own analogy score
spans ~5 points across seeds on the text8-like CBOW-HS workload) cancels in the
pairing. The oracle side is tests/golden/quality_paired_oracle.json
(tests/golden/gen_quality_paired_golden.py)."""
from __future__ import annotations

import numpy as np

from tests.golden.gen_quality_golden import CORPUS, ITERS, TRAIN, alpha
from tests.golden.gen_quality_zipf_golden import ZCORPUS, ZTRAIN, zalpha
from tests.harness import device_config, oracle_run
from tests.quality import planted_corpus, planted_zipf_corpus

# corpus -> seeds; text8_small is a text8-like corpus of 2 M tokens (20 K filler
# types, 30 % planted positions, so one epoch learns the relations), for the
# one-wavefront runs (one wave trains ~60 K words/s: 10 M tokens take minutes)
PAIRED_SEEDS = {"planted": (1, 2, 3), "text8_like": (1, 2, 3), "text8_small": (1,)}
PAIRED_MODES = {"planted": ("sg_ns", "sg_hs", "cbow_ns", "cbow_hs"), "text8_like": ("sg_ns", "cbow_hs"),
                "text8_small": ("sg_ns", "cbow_hs")}
ONE_WAVE_CORPORA = ("planted", "text8_small")
FULL_CORPORA = ("planted", "text8_like", "text8_small")


def corpus(name):
    if name == "planted":
        return planted_corpus(**CORPUS)
    if name == "text8_small":
        return planted_zipf_corpus(n_tokens=2_000_000, sent_len=1000, filler=20_000, planted_frac=0.3, seed=0)
    return planted_zipf_corpus(**ZCORPUS)


def params(name, mode):
    if name == "planted":
        return dict(iters=ITERS[mode], init_alpha=alpha(mode), **TRAIN)
    p = dict(ZTRAIN)
    return dict(iters=p.pop("iters"), init_alpha=zalpha(mode), **p)


def key_of(seed: int) -> int:
    return 0x5EED_0000_0000 + 7919 * seed


_ORACLES = {}


def setup(name, mode, seed, sents):
    """Oracle after build_vocab + init_weights (seeded) + build_sample, the
    per-epoch sentence orders and the Philox key of this (corpus, mode, seed).
    The vocabulary is built once per (corpus, mode) (build_vocab draws nothing
    from the generator, so re-seeding and re-running init_weights gives what a
    fresh oracle_run(seed=seed) gives)."""
    p = params(name, mode)
    k = (name, mode, id(sents))
    if k not in _ORACLES:
        _ORACLES.clear()
        _ORACLES[k] = oracle_run(sents, mode, seed=seed, train=False, **p)
        _ORACLES[k].build_sample()
    o = _ORACLES[k]
    o.seed(seed)
    o.init_weights()
    n = o.samples()[1].size - 1
    rng = np.random.default_rng(1000 + seed)
    orders = np.concatenate([rng.permutation(n) for _ in range(p["iters"])]).astype(np.int64)
    return o, orders, key_of(seed), p


def eval_matrix(mode):
    return 1 if mode == "cbow_hs" else 0  # the matrix main.cpp:198-201 saves


def gpu_cfg(o, mode, p):
    return device_config(o, mode, p["dim"], p["window"], p["iters"], p["table_size"], True, p["init_alpha"], 2.5e-6)


def train_gpu_paired(name, mode, seed, sents, max_waves=0, stats=None, policy=None):
    """The GPU side: the parallel schedule (Philox, default update policy;
    `policy` overrides it: hot_rows, private_rows, flush_centers,
    private_average, context_rows, context_flush) with at most `max_waves`
    wavefronts in flight (0 = all that fit), from the oracle's start on its
    draws. Returns (words, evaluated matrix)."""
    from tests.harness import device_from_oracle
    from word2vec_amd import _native as N

    o, orders, key, p = setup(name, mode, seed, sents)
    d = device_from_oracle(o, gpu_cfg(o, mode, p), initial=False)
    d.set_rng(N.W2V_RNG_PHILOX, key)
    d.set_schedule(N.W2V_SCHED_PARALLEL)
    d.set_max_waves(max_waves)
    pol = dict(policy or {})
    if "hot_rows" in pol:
        d.set_hot_rows(pol["hot_rows"])
    if "hot_tau_rows" in pol or "hot_tau_nodes" in pol:
        d.set_hot_auto(pol.get("hot_tau_rows", 0.0), pol.get("hot_tau_nodes", 1.0))
    if "private_rows" in pol:
        d.set_private_rows(pol["private_rows"])
    if "private_rate" in pol:
        d.set_private_rate(pol["private_rate"])
    if "flush_centers" in pol or "private_average" in pol:
        d.set_private_sync(pol.get("flush_centers", 0), pol.get("private_average", 8.0))
    if "context_rows" in pol or "context_flush" in pol:
        d.set_context_private(pol.get("context_rows", -1), pol.get("context_flush", 0))
    d.set_progress(0)
    n = orders.size // p["iters"]
    for e in range(p["iters"]):
        st = d.train_epoch(e, orders[e * n:(e + 1) * n])
        if stats is not None:
            stats.append(st)
    W, Cm, _ = d.download_model()
    d.close()
    words, _ = o.vocab()
    return words, (Cm if eval_matrix(mode) == 1 else W)
