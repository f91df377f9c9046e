"""The sequential oracle (test infrastructure) on tools/r03/replica_study.py's
planted Zipf corpus at the headline's scale, paired with the study's one-GPU
replica (same corpus, init_weights draw, sentence order, Philox key): what the
reference scores there, for the hot-row threshold study.
usage: oracle_planted_big.py [seed] [tokens] [filler] [dim]"""
import importlib.util
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import oracle  # noqa: E402

spec = importlib.util.spec_from_file_location("replica_study", ROOT / "tools" / "r03" / "replica_study.py")
rs = importlib.util.module_from_spec(spec)
spec.loader.exec_module(rs)


def main(seed=1, tokens=50_000_000, filler=1_000_000, dim=300, planted=0.05):
    seed, tokens, filler, dim = int(seed), int(tokens), int(filler), int(dim)
    t0 = time.time()
    tok, n_sent, names, qs, prs = rs.planted_zipf_ids(tokens, filler=filler, planted_frac=float(planted), seed=0)
    raw = tok.size
    ids, soff, counts, words = rs.build(tok, n_sent, 1000, names)
    del tok
    V = counts.size
    o = oracle.Oracle(iter=1, window=5, min_count=5, table_size=100_000_000, word_dim=dim, negative=5,
                      subsample_threshold=1e-4, init_alpha=0.025, min_alpha=2.5e-6, cbow_mean=True,
                      train_method="ns", model="sg")
    o.set_vocab_counts(counts)
    rng = np.random.default_rng(seed)  # replica_study.train's W0 / C0
    o.set_matrix(0, ((rng.random((V, dim), dtype=np.float32) - 0.5) / dim).astype(np.float32))
    o.set_matrix(1, np.zeros((V, dim), np.float32))
    o.set_samples(ids, soff, raw)
    order = np.random.default_rng(1000 * seed).permutation(n_sent).astype(np.int64)
    t1 = time.time()
    o.train_philox(0, 1, order, (seed << 32) | 0x5EED, 0)
    t2 = time.time()
    a, s = rs.gpu_scores(words, o.matrix(0), qs, prs, torch.device("cpu"))
    print(json.dumps({"seed": seed, "tokens": raw, "V": int(V), "dim": dim, "oracle_analogy": round(a, 2),
                      "oracle_similarity": round(s, 2), "train_s": round(t2 - t1, 1), "total_s": round(time.time() - t0, 1)}),
          flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
