"""Oracle scores on the text8-like planted corpus (tests/quality.planted_zipf_corpus),
SG-NS, 3 seeds -> tests/golden/quality_zipf_oracle.json (about 2 min per seed,
the seeds run in parallel processes). Run from the repo root."""
import json
import sys
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

ZCORPUS = dict(n_tokens=10_000_000, sent_len=1000, planted_frac=0.10, seed=0)
ZTRAIN = dict(dim=100, window=5, iters=1, table_size=100_000_000, min_count=5, subsample=1e-4)
ZMODE = "sg_ns"
ZSEEDS = (1, 2, 3)


def one(seed):
    from tests.harness import oracle_run
    from tests.quality import planted_zipf_corpus
    from word2vec_amd.evaluate import analogy_accuracy, similarity_score

    sents, qs, pairs = planted_zipf_corpus(**ZCORPUS)
    o = oracle_run(sents, ZMODE, seed=seed, init_alpha=0.025, **ZTRAIN)
    words, _ = o.vocab()
    E = o.matrix(0)
    return {"seed": seed, "analogy": analogy_accuracy(words, E, qs)["accuracy"],
            "similarity": similarity_score(words, E, pairs)["spearman"], "V": len(words)}


def main():
    with ProcessPoolExecutor(len(ZSEEDS)) as ex:
        res = list(ex.map(one, ZSEEDS))
    out = {"corpus": ZCORPUS, "train": ZTRAIN, "mode": ZMODE, "scores": res}
    (ROOT / "tests" / "golden" / "quality_zipf_oracle.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
