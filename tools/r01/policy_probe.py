"""Quality + speed of update policies / allocation modes (experiment driver)."""
import os, sys, time, json, subprocess
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np
from tests.golden.gen_quality_golden import CORPUS, ITERS, TRAIN, alpha
from tests.harness import MODES
from tests.quality import planted_corpus
from word2vec_amd.evaluate import analogy_accuracy, similarity_score
from word2vec_amd.model import Word2Vec
sents, qs, pairs = planted_corpus(**CORPUS)
GOLD = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
configs = [("default", {}), ("uncached", {"W2V_MATRIX_ALLOC": "uncached"}), ("fresh", {"W2V_FRESH_LOADS": "1"}),
           ("uncached+fresh", {"W2V_MATRIX_ALLOC": "uncached", "W2V_FRESH_LOADS": "1"})]
modes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["sg_ns", "cbow_hs"]
for name, env in configs:
    for k in ("W2V_MATRIX_ALLOC", "W2V_FRESH_LOADS"):
        os.environ.pop(k, None)
    os.environ.update(env)
    for mode in modes:
        m = MODES[mode]
        ref = np.mean([[r["analogy"], r["similarity"]] for r in GOLD["scores"][mode]], axis=0)
        for hot, priv in [(0, 0), (-1, 0)]:
            w = Word2Vec(iter=ITERS[mode], window=5, min_count=5, table_size=10_000_000, word_dim=64, negative=m["negative"],
                         subsample_threshold=1e-3, init_alpha=alpha(mode), min_alpha=2.5e-6, cbow_mean=True,
                         train_method=m["train_method"], model=m["model"], hot_rows=hot, private_rows=priv)
            w.seed(11); w.build_vocab(sents); w.init_weights(); w.train(sents)
            words, _ = w.vocab()
            E = w.matrix(1 if mode == "cbow_hs" else 0)
            print(f"{name:15s} {mode} hot={hot} priv={priv}: analogy {analogy_accuracy(words, E, qs)['accuracy']:.2f} "
                  f"sim {similarity_score(words, E, pairs)['spearman']:.2f} (oracle {ref[0]:.2f} {ref[1]:.2f})", flush=True)
