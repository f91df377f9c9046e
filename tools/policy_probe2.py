"""Quality of plain updates with write-through (sc1) loads/stores, and of HS under concurrency caps."""
import os, sys, json
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
def run(mode, hot, priv, env):
    for k in ("W2V_FRESH_LOADS", "W2V_DEBUG_MAX_BLOCKS", "W2V_FLUSH_EVERY"):
        os.environ.pop(k, None)
    os.environ.update(env)
    m = MODES[mode]
    ref = np.mean([[r["analogy"], r["similarity"]] for r in GOLD["scores"][mode]], axis=0)
    w = Word2Vec(iter=ITERS[mode], window=5, min_count=5, table_size=10_000_000, word_dim=64, negative=m["negative"],
                 subsample_threshold=1e-3, init_alpha=alpha(mode), min_alpha=2.5e-6, cbow_mean=True,
                 train_method=m["train_method"], model=m["model"], hot_rows=hot, private_rows=priv)
    w.seed(11); w.build_vocab(sents); w.init_weights(); w.train(sents)
    words, _ = w.vocab()
    E = w.matrix(1 if mode == "cbow_hs" else 0)
    print(f"{mode} hot={hot} priv={priv} {env}: analogy {analogy_accuracy(words, E, qs)['accuracy']:.2f} "
          f"sim {similarity_score(words, E, pairs)['spearman']:.2f} (oracle {ref[0]:.2f} {ref[1]:.2f})", flush=True)
for F in (1, 2, 4, 8, 16):
    for mode in ("sg_ns", "cbow_hs"):
        run(mode, -1, -1, {"W2V_FLUSH_EVERY": str(F)})
