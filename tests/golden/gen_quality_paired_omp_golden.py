"""The reference's OpenMP Hogwild loop (Word2Vec.cpp:375-394, 16 threads as the
reference build runs on the GPU box's cores) on the paired-gate corpora
(tests/paired.py), from the same start, sentence orders and Philox draws as
the sequential golden (gen_quality_paired_golden.py): the threads'
concurrency is the only difference (oracle orc_train_philox_omp). Two runs per
seed (the loop is not deterministic). Test infrastructure; writes
tests/golden/quality_paired_omp16_oracle.json. From the repo root:
python tests/golden/gen_quality_paired_omp_golden.py [corpus ...]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
THREADS, RUNS = 16, 2


def one(name, mode, seed, sents, qs, pairs):
    from tests import paired
    from word2vec_amd.evaluate import analogy_accuracy, similarity_score

    runs, ts = [], []
    for _ in range(RUNS):
        o, orders, key, p = paired.setup(name, mode, seed, sents)  # re-seeds and re-draws the start
        t0 = time.time()
        o.train_philox_omp(THREADS, 0, p["iters"], orders, key, 0)
        ts.append(round(time.time() - t0, 1))
        words, _ = o.vocab()
        E = o.matrix(paired.eval_matrix(mode))
        runs.append([round(analogy_accuracy(words, E, qs)["accuracy"], 3),
                     round(similarity_score(words, E, pairs)["spearman"], 3)])
    a, s = np.mean(runs, 0)
    r = {"seed": seed, "key": key, "analogy": round(float(a), 3), "similarity": round(float(s), 3), "runs": runs,
         "threads": THREADS, "train_s": ts}
    print(name, mode, r, flush=True)
    return r


def main(only):
    from tests import paired

    f = ROOT / "tests" / "golden" / "quality_paired_omp16_oracle.json"
    out = json.loads(f.read_text()) if f.exists() else {}
    out["threads"], out["runs_per_seed"] = THREADS, RUNS
    for n, modes in paired.PAIRED_MODES.items():
        if only and n not in only:
            continue
        sents, qs, pairs = paired.corpus(n)
        out[n] = {m: [one(n, m, s, sents, qs, pairs) for s in paired.PAIRED_SEEDS[n]] for m in modes}
        f.write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main(set(sys.argv[1:]))
