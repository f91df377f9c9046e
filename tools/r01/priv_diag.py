import os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np
from tests.golden.gen_quality_golden import CORPUS, ITERS, TRAIN, alpha
from tests.harness import MODES
from tests.quality import planted_corpus
from word2vec_amd.evaluate import analogy_accuracy
from word2vec_amd.model import Word2Vec
sents, qs, pairs = planted_corpus(**CORPUS)
mode = "sg_ns"; m = MODES[mode]
for hot, priv, cap in [(-1, 0, 0), (-1, -1, 0), (-1, -1, 1), (-1, -1, 4), (-1, 2, 0), (-1, 64, 0)]:
    os.environ["W2V_DEBUG_MAX_BLOCKS"] = str(cap)
    w = Word2Vec(iter=2, window=5, min_count=5, table_size=10_000_000, word_dim=64, negative=5, subsample_threshold=1e-3,
                 init_alpha=0.025, min_alpha=2.5e-6, cbow_mean=True, train_method="ns", model="sg", hot_rows=hot, private_rows=priv)
    w.seed(11); w.build_vocab(sents); w.init_weights(); w.train(sents)
    words, counts = w.vocab()
    W, Cm = w.matrix(0), w.matrix(1)
    acc = analogy_accuracy(words, W, qs)["accuracy"]
    print(f"hot {hot} priv {priv} cap {cap}: acc {acc:.2f} |W| max {np.abs(W).max():.3g} nan {np.isnan(W).sum()} "
          f"|C| max {np.abs(Cm).max():.3g} nan {np.isnan(Cm).sum()} C[0:3] norms {np.linalg.norm(Cm[:3],axis=1)} C[100] {np.linalg.norm(Cm[100]):.3g}", flush=True)
