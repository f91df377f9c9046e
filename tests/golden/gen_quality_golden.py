"""Oracle (sequential reference restatement) quality scores on the planted-
relation corpus, 3 seeds per mode -> tests/golden/quality_oracle.json.
Run from the repo root: python tests/golden/gen_quality_golden.py"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from tests.harness import oracle_run  # noqa: E402
from tests.quality import planted_corpus  # noqa: E402
from word2vec_amd.evaluate import analogy_accuracy, similarity_score  # noqa: E402

CORPUS = dict(sent_len=200, seed=0, rows=40, p_topic=0.10, p_role=0.10, p_cross=0.3, n_sent=3000)
TRAIN = dict(dim=64, window=5, table_size=10_000_000, min_count=5, subsample=1e-3)
ITERS = {"sg_ns": 2, "cbow_ns": 3, "sg_hs": 1, "cbow_hs": 3}
SEEDS = (1, 2, 3)


def alpha(mode):
    return 0.025 if mode.startswith("sg") else 0.05


def main():
    sents, qs, pairs = planted_corpus(**CORPUS)
    out = {"corpus": CORPUS, "train": TRAIN, "iters": ITERS, "seeds": SEEDS, "scores": {}}
    for mode, iters in ITERS.items():
        res = []
        for seed in SEEDS:
            o = oracle_run(sents, mode, iters=iters, seed=seed, init_alpha=alpha(mode), **TRAIN)
            words, _ = o.vocab()
            E = o.matrix(1 if mode == "cbow_hs" else 0)  # the matrix main.cpp:198-201 saves
            res.append({"analogy": analogy_accuracy(words, E, qs)["accuracy"],
                        "similarity": similarity_score(words, E, pairs)["spearman"]})
        out["scores"][mode] = res
        print(mode, res, flush=True)
    (ROOT / "tests" / "golden" / "quality_oracle.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
