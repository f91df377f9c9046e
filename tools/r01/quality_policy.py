"""Planted-corpus quality (the tests/test_gpu_quality.py gate: 3 seeds, mean
delta vs the sequential oracle golden) per mode under alternative update
policies, to pick per-mode defaults that keep the gate with the most speed.
usage: python tools/quality_policy.py [mode ...] [policy=NAME ...]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import json  # noqa: E402

import numpy as np  # noqa: E402

from tests.golden.gen_quality_golden import CORPUS, ITERS, TRAIN, alpha  # noqa: E402
from tests.harness import MODES  # noqa: E402
from tests.quality import planted_corpus  # noqa: E402
from word2vec_amd.evaluate import analogy_accuracy, similarity_score  # noqa: E402
from word2vec_amd.model import Word2Vec  # noqa: E402

GOLD = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
SENTS, QS, PAIRS = planted_corpus(**CORPUS)
POLICIES = [("default", {}), ("hot_rows=0", dict(hot_rows=0)), ("hot_rows=64", dict(hot_rows=64)),
            ("hot_rows=250", dict(hot_rows=250)), ("hot_rows=500", dict(hot_rows=500)), ("hot_rows=2000", dict(hot_rows=2000)),
            ("private off", dict(private_rows=0)), ("plain Hogwild", dict(hot_rows=0, private_rows=0, context_rows=0))]
CBOW_POLICIES = [("context rows off", dict(context_rows=0)), ("context flush 16", dict(context_flush=16)),
                 ("context flush 256", dict(context_flush=256)), ("context flush 1024", dict(context_flush=1024)),
                 ("context only", dict(private_rows=0)), ("context only flush 64", dict(private_rows=0, context_flush=64)),
                 ("both flush 64", dict(flush_centers=64, context_flush=64)),
                 ("both flush 16", dict(flush_centers=16, context_flush=16)),
                 ("context avg 1", dict(private_average=1.0)), ("context flush 32", dict(context_flush=32))]
HS_POLICIES = [("flush 32", dict(flush_centers=32)), ("flush 64", dict(flush_centers=64)),
               ("flush 128", dict(flush_centers=128))]
NS_POLICIES = [("flush 512", dict(flush_centers=512)), ("flush 1024", dict(flush_centers=1024)),
               ("flush 4096", dict(flush_centers=4096))]
ONLY = [p for p in sys.argv[1:] if p.startswith("policy=")]

for mode in [a for a in sys.argv[1:] if a in MODES] or list(MODES):
    m = MODES[mode]
    ref = np.array([[r["analogy"], r["similarity"]] for r in GOLD["scores"][mode]]).mean(0)
    pols = POLICIES + (CBOW_POLICIES if mode.startswith("cbow") else []) + (HS_POLICIES if mode.endswith("hs") else NS_POLICIES)
    if ONLY:
        pols = [p for p in pols if f"policy={p[0]}" in ONLY]
    for name, pol in pols:
        got = []
        for s in (11, 12, 13):
            w = Word2Vec(iter=ITERS[mode], window=5, min_count=TRAIN["min_count"], table_size=TRAIN["table_size"],
                         word_dim=TRAIN["dim"], negative=m["negative"], subsample_threshold=TRAIN["subsample"],
                         init_alpha=alpha(mode), min_alpha=2.5e-6, cbow_mean=True, train_method=m["train_method"],
                         model=m["model"], verbose=False, **pol)
            w.seed(s)
            w.build_vocab(SENTS)
            w.init_weights()
            w.train(SENTS)
            words, _ = w.vocab()
            E = w.matrix(1 if mode == "cbow_hs" else 0)
            if not np.isfinite(E).all():
                got.append([float("nan")] * 2)
                continue
            got.append([analogy_accuracy(words, E, QS)["accuracy"], similarity_score(words, E, PAIRS)["spearman"]])
        d = np.array(got).mean(0) - ref
        print(f"{mode:8s} {name:14s} delta analogy {d[0]:+6.2f} similarity {d[1]:+6.2f}", flush=True)
