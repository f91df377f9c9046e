"""Oracle side of the paired quality runs (tests/paired.py): for each corpus
(planted, text8-like), mode and seed, the oracle trains in its Philox draw mode
from the seeded initial weights over the seeded sentence orders; the scores go
to tests/golden/quality_paired_oracle.json. The GPU tests
(tests/test_gpu_quality.py) train from the same start on the same draws.
About 1 min per text8-like run; runs in parallel processes. From the repo root:
python tests/golden/gen_quality_paired_golden.py [workers] [corpus ...]"""
import json
import sys
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def one(job):
    name, mode, seed = job
    from tests import paired
    from word2vec_amd.evaluate import analogy_accuracy, similarity_score

    sents, qs, pairs = paired.corpus(name)
    o, orders, key, p = paired.setup(name, mode, seed, sents)
    o.train_philox(0, p["iters"], orders, key, 0)
    words, _ = o.vocab()
    E = o.matrix(paired.eval_matrix(mode))
    r = {"seed": seed, "key": key, "analogy": analogy_accuracy(words, E, qs)["accuracy"],
         "similarity": similarity_score(words, E, pairs)["spearman"], "V": len(words)}
    print(name, mode, r, flush=True)
    return name, mode, r


def main(workers=4):
    from tests import paired

    import json as _json

    only = set(sys.argv[2:])  # corpus names to (re)generate; the rest is kept
    f = ROOT / "tests" / "golden" / "quality_paired_oracle.json"
    out = _json.loads(f.read_text()) if f.exists() and only else {}
    out["seeds"] = {k: list(v) for k, v in paired.PAIRED_SEEDS.items()}
    jobs = [(n, m, s) for n, modes in paired.PAIRED_MODES.items() if not only or n in only for m in modes
            for s in paired.PAIRED_SEEDS[n]]
    for n in paired.PAIRED_MODES:
        if not only or n in only:
            out[n] = {}
    with ProcessPoolExecutor(workers) as ex:
        for name, mode, r in ex.map(one, jobs):
            out[name].setdefault(mode, []).append(r)
    (ROOT / "tests" / "golden" / "quality_paired_oracle.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:2]])
