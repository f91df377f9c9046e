#!/usr/bin/env python3
"""configs[4] (shared-negatives d512 / neg 15): quality at its own
hyper-parameters on the text8-like corpus for a given number of atomic rows
(`hot_rows`, default = the library's automatic rule with its 1000-row floor),
next to the reference's per-pair oracle golden
(tests/golden/quality_zipf_sg_ns_c5_oracle.json). One JSON line per run.
usage: c5_hot_probe.py HOT_ROWS[,HOT_ROWS...] [SEEDS] [MAX_WAVES[,...]] [ALPHA[,...]] [PRIVATE_ROWS[,...]]
       [PRIVATE_AVERAGE[,...]] [FLUSH_CENTERS[,...]]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from tests.golden.gen_quality_zipf_golden import ZCORPUS  # noqa: E402
from tests.quality import planted_zipf_corpus  # noqa: E402
from word2vec_amd.evaluate import analogy_accuracy, similarity_score  # noqa: E402
from word2vec_amd.model import Word2Vec  # noqa: E402


def main(hots="-2", seeds="11,12,13", waves="0", alphas="0", privs="-1", pavgs="8", flushes="0"):
    gold = json.loads((ROOT / "tests" / "golden" / "quality_zipf_sg_ns_c5_oracle.json").read_text())
    t = gold["train"]
    ref = np.array([[r["analogy"], r["similarity"]] for r in gold["scores"]]).mean(0)
    sents, qs, pairs = planted_zipf_corpus(**ZCORPUS)
    for hot, mw, al, pr, pa, fl in [(int(h), int(w), float(a), int(p), float(q), int(f)) for h in hots.split(",")
                                    for w in waves.split(",") for a in alphas.split(",") for p in privs.split(",")
                                    for q in pavgs.split(",") for f in flushes.split(",")]:
        got = []
        t0 = time.time()
        for seed in [int(s) for s in seeds.split(",")]:
            w = Word2Vec(iter=t["iters"], window=t["window"], min_count=t["min_count"], table_size=t["table_size"],
                         word_dim=t["dim"], negative=t["negative"], subsample_threshold=t["subsample"],
                         init_alpha=al if al > 0 else gold["alpha"], min_alpha=2.5e-6, cbow_mean=True,
                         train_method="ns", model="sg", shared_negatives=True, verbose=False, hot_rows=hot,
                         max_waves=mw, private_rows=pr, private_average=pa, flush_centers=fl)
            w.seed(seed)
            w.build_vocab(sents)
            w.init_weights()
            w.train(sents)
            words, _ = w.vocab()
            E = w.matrix(0)
            got.append([analogy_accuracy(words, E, qs)["accuracy"], similarity_score(words, E, pairs)["spearman"]])
        g = np.array(got).mean(0)
        print(json.dumps({"hot_rows": hot, "private_rows": pr, "private_average": pa, "flush_centers": fl,
                          "max_waves": mw, "alpha": al if al > 0 else gold["alpha"], "analogy": round(g[0], 2), "similarity": round(g[1], 2),
                          "d_analogy": round(g[0] - ref[0], 2), "d_similarity": round(g[1] - ref[1], 2),
                          "per_seed": np.round(got, 2).tolist(), "secs": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
