"""Sequential-oracle scores at the benchmarked workloads' own scale (VERDICT r03
"next" 2): the planted-relation Zipf corpus of tests/planted_ids.py sized and
shaped like the bench presets, trained by the oracle (oracle/w2v_oracle.cpp,
the reference's sequential loop, Word2Vec.cpp:251-353, 356-396) from the same
initial weights, sentence order and Philox draws the GPU gate
(tests/test_gpu_quality.py::test_quality_headline_scale) uses, so the GPU's
parallel schedule and update policy are the only difference.

  c3   configs[2] (bench default): SG-NS neg 5, d300, w5, subsample 1e-4,
       50 M tokens, Zipf(s=1) filler over 1 M ranks (V ~ 717 K), planted 0.05
  c2   configs[1]: CBOW-HS d200 on a text8-shaped corpus: 17 M tokens, filler
       p(r) ~ (r + 4)^-1.285 over 350 K ranks, 10 % planted positions: V 71.1 K
       at min_count 5, 256 K types, the most frequent word 5 % of tokens
       (text8: 71.3 K, 254 K, 6 %)
  c1   configs[0]: SG-NS neg 5 d100 on the same text8-shaped corpus
  c2ns the reference's CBOW-NS mode (neg 5, d200) on configs[1]'s corpus
  c1hs the reference's SG-HS mode (d100) on configs[0]'s corpus

usage (repo root): python tests/golden/gen_headline_planted_golden.py c3 [seeds]
  -> tests/golden/quality_headline_<workload>_oracle.json (one record per seed).
c3 takes ~37 min per seed on one core (seeds run in parallel processes).

The reference as it actually runs (VERDICT r05 "next" 2): its OpenMP Hogwild
loop (Word2Vec.cpp:375-394) on THREADS threads, same start, order and Philox
draws, so the threads' concurrency is the only difference from the sequential
golden (oracle orc_train_philox_omp):
  python tests/golden/gen_headline_planted_golden.py c3 [seeds] omp16
  -> tests/golden/quality_headline_<workload>_omp16_oracle.json, OMP_RUNS runs
     per seed (the loop is not deterministic), seeds one after another."""
import json
import sys
import time
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

TEXT8 = dict(n_tokens=17_000_000, filler=350_000, zipf_s=1.285, zipf_q=4.0, planted_frac=0.10)
WORKLOADS = {
    "c3": dict(corpus=dict(n_tokens=50_000_000, filler=1_000_000, planted_frac=0.05), mode="sg_ns", dim=300,
               negative=5, alpha=0.025),
    "c2": dict(corpus=TEXT8, mode="cbow_hs", dim=200, negative=0, alpha=0.05),
    "c1": dict(corpus=TEXT8, mode="sg_ns", dim=100, negative=5, alpha=0.025),
    # the reference's CBOW-NS mode (no BASELINE config of its own) on configs[1]'s corpus and width
    "c2ns": dict(corpus=TEXT8, mode="cbow_ns", dim=200, negative=5, alpha=0.05),
    # the reference's SG-HS mode on configs[0]'s corpus and width
    "c1hs": dict(corpus=TEXT8, mode="sg_hs", dim=100, negative=0, alpha=0.025),
    # SG-HS at configs[2]'s corpus and width
    "c3hs": dict(corpus=dict(n_tokens=50_000_000, filler=1_000_000, planted_frac=0.05), mode="sg_hs", dim=300,
                 negative=0, alpha=0.025),
    # SG-HS between text8's and configs[2]'s vocabularies (round 6 probe golden,
    # no gate: where does the large-vocabulary HS rule's threshold belong?
    # DESIGN.md §4.1): 20 M tokens, Zipf(s=1) filler over 300 K ranks, d200
    "mhs": dict(corpus=dict(n_tokens=20_000_000, filler=300_000, planted_frac=0.05), mode="sg_hs", dim=200,
                negative=0, alpha=0.025),
    # CBOW-HS at configs[2]'s corpus and width
    "c3cbhs": dict(corpus=dict(n_tokens=50_000_000, filler=1_000_000, planted_frac=0.05), mode="cbow_hs", dim=300,
                   negative=0, alpha=0.05),
}
TRAIN = dict(window=5, iters=1, table_size=100_000_000, min_count=5, subsample=1e-4)
SEEDS = (1, 2)


OMP_RUNS = 2


def golden_path(name, omp=0):
    tag = f"_omp{omp}" if omp else ""
    return ROOT / "tests" / "golden" / f"quality_headline_{name}{tag}_oracle.json"


def corpus(name):
    """(ids, sentence offsets, counts, words, raw tokens, questions, pairs)."""
    from tests.planted_ids import build, planted_zipf_ids

    tok, n_sent, names, qs, prs = planted_zipf_ids(**WORKLOADS[name]["corpus"], seed=0)
    raw = tok.size
    ids, soff, counts, words = build(tok, n_sent, 1000, names, TRAIN["min_count"])
    return ids, soff, counts, words, raw, qs, prs


def init(name, seed, V):
    """The paired start: W ~ U(-0.5, 0.5) / d from numpy (seed), C = 0 (NS) or
    drawn like W (CBOW-HS), synapses1 = 0; the sentence order; the
    Philox key."""
    w = WORKLOADS[name]
    d, hs = w["dim"], w["mode"].endswith("hs")
    rng = np.random.default_rng(seed)
    W0 = ((rng.random((V, d), dtype=np.float32) - 0.5) / d).astype(np.float32)
    C0 = ((rng.random((V, d), dtype=np.float32) - 0.5) / d).astype(np.float32) if hs else np.zeros((V, d), np.float32)
    S0 = np.zeros((V - 1, d), np.float32) if hs else None
    return W0, C0, S0, (seed << 32) | 0x5EED


def order_of(seed, n_sent):
    return np.random.default_rng(1000 * seed).permutation(n_sent).astype(np.int64)


def eval_matrix(name):
    return 1 if WORKLOADS[name]["mode"] == "cbow_hs" else 0  # the matrix main.cpp:198-201 saves


def one(args):
    name, seed, omp = args if len(args) == 3 else (*args, 0)
    import oracle
    from tests.planted_ids import scores

    w = WORKLOADS[name]
    t0 = time.time()
    ids, soff, counts, words, raw, qs, prs = corpus(name)
    V = counts.size
    o = oracle.Oracle(iter=TRAIN["iters"], window=TRAIN["window"], min_count=TRAIN["min_count"],
                      table_size=TRAIN["table_size"], word_dim=w["dim"], negative=w["negative"],
                      subsample_threshold=TRAIN["subsample"], init_alpha=w["alpha"], min_alpha=2.5e-6,
                      cbow_mean=True, train_method="hs" if w["mode"].endswith("hs") else "ns",
                      model="cbow" if w["mode"].startswith("cbow") else "sg")
    o.set_vocab_counts(counts)
    W0, C0, S0, key = init(name, seed, V)
    o.set_matrix(0, W0)
    o.set_matrix(1, C0)
    if S0 is not None:
        o.set_matrix(2, S0)
    del W0, C0, S0
    o.set_samples(ids, soff, raw)
    order = order_of(seed, soff.size - 1)
    if not omp:
        t1 = time.time()
        o.train_philox(0, 1, order, key, 0)
        t2 = time.time()
        a, s = scores(words, o.matrix(eval_matrix(name)), qs, prs, chunk=256)
        rec = {"seed": seed, "analogy": round(a, 3), "similarity": round(s, 3), "V": int(V), "raw_tokens": int(raw),
               "in_vocab": int(ids.size), "train_s": round(t2 - t1, 1), "total_s": round(time.time() - t0, 1)}
        print(json.dumps({"workload": name, **rec}), flush=True)
        return rec
    start = [o.matrix(k).copy() for k in (0, 1)] + ([o.matrix(2).copy()] if w["mode"].endswith("hs") else [])
    runs, ts = [], []
    for run in range(OMP_RUNS):
        for k, M in enumerate(start):
            o.set_matrix(k, M)
        t1 = time.time()
        o.train_philox_omp(omp, 0, 1, order, key, 0)
        ts.append(round(time.time() - t1, 1))
        runs.append([round(x, 3) for x in scores(words, o.matrix(eval_matrix(name)), qs, prs, chunk=256)])
    a, s = np.mean(runs, 0)
    rec = {"seed": seed, "analogy": round(float(a), 3), "similarity": round(float(s), 3), "runs": runs,
           "threads": omp, "V": int(V), "raw_tokens": int(raw), "in_vocab": int(ids.size), "train_s": ts,
           "total_s": round(time.time() - t0, 1)}
    print(json.dumps({"workload": name, **rec}), flush=True)
    return rec


def main(name, seeds=None, omp=None):
    seeds = tuple(int(s) for s in seeds.split(",")) if seeds else SEEDS
    threads = int(omp[3:]) if omp else 0
    if threads:
        recs = [one((name, s, threads)) for s in seeds]
        gen = f"tests/golden/gen_headline_planted_golden.py (the reference's OpenMP loop, {threads} threads, Philox draws)"
    else:
        with ProcessPoolExecutor(len(seeds)) as ex:
            recs = list(ex.map(one, [(name, s) for s in seeds]))
        gen = "tests/golden/gen_headline_planted_golden.py (sequential oracle, Philox draws)"
    w = WORKLOADS[name]
    out = {"workload": name, "corpus": w["corpus"], "mode": w["mode"], "dim": w["dim"], "negative": w["negative"],
           "alpha": w["alpha"], "train": TRAIN, "scores": recs, "generator": gen}
    golden_path(name, threads).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
