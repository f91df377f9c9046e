"""Oracle scores on the text8-like planted corpus (tests/quality.planted_zipf_corpus),
3 seeds: SG-NS -> tests/golden/quality_zipf_oracle.json, CBOW-HS (configs[1]'s
mode; `python tests/golden/gen_quality_zipf_golden.py cbow_hs`) ->
tests/golden/quality_zipf_cbow_hs_oracle.json, the shared-negatives
minibatch (`... sg_sn`) -> tests/golden/quality_zipf_sg_sn_oracle.json; configs[4]'s own
hyper-parameters (d512, negative 15): the reference's per-pair SG-NS (`... sg_ns_c5`) ->
tests/golden/quality_zipf_sg_ns_c5_oracle.json. About 2 min per seed at d100 (about
40 at d512 / neg 15), the seeds run in parallel processes. Run from the repo root."""
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
ZFILES = {"sg_ns": "quality_zipf_oracle.json", "cbow_hs": "quality_zipf_cbow_hs_oracle.json",
          "sg_sn": "quality_zipf_sg_sn_oracle.json", "sg_ns_c5": "quality_zipf_sg_ns_c5_oracle.json",
          "sg_sn_c5": "quality_zipf_sg_sn_c5_oracle.json"}
# configs[4]'s hyper-parameters (BASELINE.json): d512, negative 15
C5 = dict(dim=512, negative=15)


def zalpha(mode):
    return 0.025 if mode.startswith("sg") else 0.05


def zmatrix(mode):
    """The vectors evaluated: W, or C for CBOW-HS (tests/test_gpu_quality.train_gpu)."""
    return 1 if mode == "cbow_hs" else 0


def one(seed, mode=ZMODE):
    from tests.harness import oracle_run
    from tests.quality import planted_zipf_corpus
    from word2vec_amd.evaluate import analogy_accuracy, similarity_score

    sents, qs, pairs = planted_zipf_corpus(**ZCORPUS)
    if mode in ("sg_sn", "sg_sn_c5"):  # the shared-negatives minibatch, sequential (oracle sgsn_sentence)
        import numpy as np
        if mode == "sg_sn":  # neg 5 at ZTRAIN's d100
            o = oracle_run(sents, "sg_ns", seed=seed, init_alpha=zalpha(mode), train=False, **ZTRAIN)
        else:  # configs[4]'s d512 / negative 15
            from oracle import Oracle
            t = dict(ZTRAIN, dim=C5["dim"])
            o = Oracle(iter=t["iters"], window=t["window"], min_count=t["min_count"], table_size=t["table_size"],
                       word_dim=t["dim"], negative=C5["negative"], subsample_threshold=t["subsample"],
                       init_alpha=zalpha(mode), min_alpha=2.5e-6, cbow_mean=True, train_method="ns", model="sg")
            o.load_sentences(sents)
            o.seed(seed)
            o.build_vocab()
            o.init_weights()
        o.build_sample()
        o.set_shared_negatives(True)
        order = np.random.default_rng(seed).permutation(len(sents)).astype(np.int64)
        o.train_philox(0, 1, order, 0x5EED0000 + seed, 0)
    elif mode == "sg_ns_c5":  # the reference's per-pair SG-NS at configs[4]'s d512 / negative 15
        from oracle import Oracle
        t = dict(ZTRAIN, dim=C5["dim"])
        o = Oracle(iter=t["iters"], window=t["window"], min_count=t["min_count"], table_size=t["table_size"],
                   word_dim=t["dim"], negative=C5["negative"], subsample_threshold=t["subsample"],
                   init_alpha=zalpha(mode), min_alpha=2.5e-6, cbow_mean=True, train_method="ns", model="sg")
        o.load_sentences(sents)
        o.seed(seed)
        o.build_vocab()
        o.init_weights()
        o.train(record=False)
    else:
        o = oracle_run(sents, mode, seed=seed, init_alpha=zalpha(mode), **ZTRAIN)
    words, _ = o.vocab()
    E = o.matrix(zmatrix(mode))
    return {"seed": seed, "analogy": analogy_accuracy(words, E, qs)["accuracy"],
            "similarity": similarity_score(words, E, pairs)["spearman"], "V": len(words)}


def main(mode=ZMODE):
    with ProcessPoolExecutor(len(ZSEEDS)) as ex:
        res = list(ex.map(one, ZSEEDS, [mode] * len(ZSEEDS)))
    train = dict(ZTRAIN, **C5) if mode in ("sg_ns_c5", "sg_sn_c5") else ZTRAIN
    out = {"corpus": ZCORPUS, "train": train, "mode": mode, "alpha": zalpha(mode), "scores": res}
    (ROOT / "tests" / "golden" / ZFILES[mode]).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:2])
