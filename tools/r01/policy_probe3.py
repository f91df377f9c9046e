"""Quality of the update policies with workgroup-shared privatisation (16-wave
workgroups, flush every F workgroup centers): planted corpus (4 modes) and the
text8-like planted Zipf corpus (SG-NS). Usage: policy_probe3.py [small|zipf]..."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

from tests.golden.gen_quality_golden import CORPUS, ITERS, alpha  # noqa: E402
from tests.harness import MODES  # noqa: E402
from tests.quality import planted_corpus, planted_zipf_corpus  # noqa: E402
from word2vec_amd.evaluate import analogy_accuracy, similarity_score  # noqa: E402
from word2vec_amd.model import Word2Vec  # noqa: E402

KNOBS = ("W2V_PRIV_AVG", "W2V_MATRIX_ALLOC", "W2V_FRESH_LOADS", "W2V_DEBUG_MAX_BLOCKS", "W2V_FLUSH_EVERY", "W2V_BLOCK_WAVES")


def run(tag, sents, qs, pairs, mode, iters, dim, table, sub, a0, hot, priv, env, ref, waves=-1):
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(env)
    m = MODES[mode]
    w = Word2Vec(iter=iters, window=5, min_count=5, table_size=table, word_dim=dim, negative=m["negative"],
                 subsample_threshold=sub, init_alpha=a0, min_alpha=2.5e-6, cbow_mean=True,
                 train_method=m["train_method"], model=m["model"], hot_rows=hot, private_rows=priv, max_waves=waves)
    w.seed(11)
    w.build_vocab(sents)
    w.init_weights()
    w.train(sents)
    words, _ = w.vocab()
    E = w.matrix(1 if mode == "cbow_hs" else 0)
    print(f"{tag} {mode} hot={hot} priv={priv} waves={waves} {env}: analogy {analogy_accuracy(words, E, qs)['accuracy']:.2f} "
          f"sim {similarity_score(words, E, pairs)['spearman']:.2f} (oracle {ref[0]:.2f} {ref[1]:.2f})", flush=True)


which = sys.argv[1:] or ["small", "zipf"]
SWEEP2 = [(h, -1, {"W2V_FLUSH_EVERY": str(f)}) for h, f in ((-1, 4), (10000, 4), (1000, 4), (100, 4), (1000, 2), (1000, 8))]
if "sweep2" in which:
    S, Q, P = planted_corpus(**CORPUS)
    G = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
    for mode in MODES:
        ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"][mode]], axis=0)
        for hot, priv, env in SWEEP2[:3]:
            run("small", S, Q, P, mode, ITERS[mode], 64, 10_000_000, 1e-3, alpha(mode), hot, priv, env, ref)
    S, Q, P = planted_zipf_corpus(n_tokens=10_000_000, sent_len=1000, planted_frac=0.10, seed=0)
    G = json.loads((ROOT / "tests" / "golden" / "quality_zipf_oracle.json").read_text())
    ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"]], axis=0)
    for hot, priv, env in SWEEP2:
        run("zipf", S, Q, P, "sg_ns", 1, 100, 100_000_000, 1e-4, 0.025, hot, priv, env, ref)
if "hs" in which:
    S, Q, P = planted_corpus(**CORPUS)
    G = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
    for mode in ("sg_hs", "cbow_hs"):
        ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"][mode]], axis=0)
        for waves in (64, 128, 256, 512):
            for f in (1, 4):
                run("small", S, Q, P, mode, ITERS[mode], 64, 10_000_000, 1e-3, alpha(mode), -1, -1,
                    {"W2V_FLUSH_EVERY": str(f)}, ref, waves=waves)
        run("small", S, Q, P, mode, ITERS[mode], 64, 10_000_000, 1e-3, alpha(mode), -1, 0, {}, ref, waves=128)
if "alloc" in which:
    S, Q, P = planted_corpus(**CORPUS)
    G = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
    for mode, waves in (("sg_hs", 64), ("sg_hs", 1024), ("sg_ns", -1)):
        ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"][mode]], axis=0)
        for alloc in ("uncached", "finegrained", "default"):
            for priv in (0, -1):
                run("small", S, Q, P, mode, ITERS[mode], 64, 10_000_000, 1e-3, alpha(mode), -1, priv,
                    {"W2V_MATRIX_ALLOC": alloc}, ref, waves=waves)
if "avg" in which:
    S, Q, P = planted_corpus(**CORPUS)
    G = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
    for mode in ("sg_hs", "cbow_hs"):
        ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"][mode]], axis=0)
        for waves in (1024, 1 << 20):
            for avg, f in ((1, 4), (8, 4), (1, 16), (8, 16)):
                run("small", S, Q, P, mode, ITERS[mode], 64, 10_000_000, 1e-3, alpha(mode), -1, -1,
                    {"W2V_FLUSH_EVERY": str(f), "W2V_PRIV_AVG": str(avg)}, ref, waves=waves)
    for mode in ("sg_ns", "cbow_ns"):
        ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"][mode]], axis=0)
        for avg, f in ((1, 16), (8, 16), (1, 64), (8, 64)):
            run("small", S, Q, P, mode, ITERS[mode], 64, 10_000_000, 1e-3, alpha(mode), 1000, -1,
                {"W2V_FLUSH_EVERY": str(f), "W2V_PRIV_AVG": str(avg)}, ref)
    S, Q, P = planted_zipf_corpus(n_tokens=10_000_000, sent_len=1000, planted_frac=0.10, seed=0)
    G = json.loads((ROOT / "tests" / "golden" / "quality_zipf_oracle.json").read_text())
    ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"]], axis=0)
    for avg, f in ((1, 16), (8, 16), (1, 64), (8, 64)):
        run("zipf", S, Q, P, "sg_ns", 1, 100, 100_000_000, 1e-4, 0.025, 1000, -1,
            {"W2V_FLUSH_EVERY": str(f), "W2V_PRIV_AVG": str(avg)}, ref)
if "avg2" in which:
    S, Q, P = planted_corpus(**CORPUS)
    G = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
    for mode in ("sg_ns", "cbow_ns"):
        ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"][mode]], axis=0)
        for hot, f in ((1000, 256), (1000, 1024), (0, 64), (0, 256)):
            run("small", S, Q, P, mode, ITERS[mode], 64, 10_000_000, 1e-3, alpha(mode), hot, -1,
                {"W2V_FLUSH_EVERY": str(f), "W2V_PRIV_AVG": "8"}, ref)
    S, Q, P = planted_zipf_corpus(n_tokens=10_000_000, sent_len=1000, planted_frac=0.10, seed=0)
    G = json.loads((ROOT / "tests" / "golden" / "quality_zipf_oracle.json").read_text())
    ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"]], axis=0)
    for hot, f in ((1000, 256), (1000, 1024), (0, 64), (0, 256)):
        run("zipf", S, Q, P, "sg_ns", 1, 100, 100_000_000, 1e-4, 0.025, hot, -1,
            {"W2V_FLUSH_EVERY": str(f), "W2V_PRIV_AVG": "8"}, ref)
SWEEP = [(-1, -1, {"W2V_BLOCK_WAVES": str(b), "W2V_FLUSH_EVERY": str(f)}) for b, f in ((4, 1), (4, 4), (16, 1), (16, 4), (16, 16))]
if "sweep" in which:
    S, Q, P = planted_corpus(**CORPUS)
    G = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
    ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"]["sg_ns"]], axis=0)
    for hot, priv, env in SWEEP:
        run("small", S, Q, P, "sg_ns", ITERS["sg_ns"], 64, 10_000_000, 1e-3, alpha("sg_ns"), hot, priv, env, ref)
    S, Q, P = planted_zipf_corpus(n_tokens=10_000_000, sent_len=1000, planted_frac=0.10, seed=0)
    G = json.loads((ROOT / "tests" / "golden" / "quality_zipf_oracle.json").read_text())
    ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"]], axis=0)
    for hot, priv, env in SWEEP:
        run("zipf", S, Q, P, "sg_ns", 1, 100, 100_000_000, 1e-4, 0.025, hot, priv, env, ref)
if "small" in which:
    S, Q, P = planted_corpus(**CORPUS)
    G = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
    for mode in MODES:
        ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"][mode]], axis=0)
        for hot, priv, env in [(-1, -1, {}), (-1, -1, {"W2V_FLUSH_EVERY": "64"})]:
            run("small", S, Q, P, mode, ITERS[mode], 64, 10_000_000, 1e-3, alpha(mode), hot, priv, env, ref)
if "zipf" in which:
    S, Q, P = planted_zipf_corpus(n_tokens=10_000_000, sent_len=1000, planted_frac=0.10, seed=0)
    G = json.loads((ROOT / "tests" / "golden" / "quality_zipf_oracle.json").read_text())
    ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"]], axis=0)
    for hot, priv, env in [(-1, -1, {}), (10000, -1, {}), (1000, -1, {}), (-1, -1, {"W2V_FLUSH_EVERY": "64"})]:
        run("zipf", S, Q, P, "sg_ns", 1, 100, 100_000_000, 1e-4, 0.025, hot, priv, env, ref)
