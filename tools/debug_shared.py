"""Debug: shared-negatives kernel vs oracle on tiny hand-made sentences (GPU)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np
from oracle import Oracle
from tests.harness import device_from_oracle
from word2vec_amd import _native as N
from word2vec_amd.device import Config

KEY = 77
def run(sents, dim, window, K):
    o = Oracle(iter=1, window=window, min_count=1, table_size=1000, word_dim=dim, negative=K,
               subsample_threshold=0.0, init_alpha=0.5, min_alpha=1e-4, train_method="ns", model="sg")
    o.load_sentences(sents); o.seed(1); o.build_vocab(); o.init_weights(); o.build_sample()
    rng = np.random.default_rng(5)
    o.set_matrix(1, ((rng.random((o.V, dim)) - 0.5)).astype(np.float32))
    o.set_matrix(0, ((rng.random((o.V, dim)) - 0.5)).astype(np.float32))
    o.set_shared_negatives(True)
    cfg = Config(word_dim=dim, window=window, negative=K, hs=False, cbow=False, iter=1, init_alpha=0.5,
                 min_alpha=1e-4, table_size=1000)
    d = device_from_oracle(o, cfg, initial=False)
    d.set_update(N.W2V_UPDATE_SHARED_NEGATIVES); d.set_rng(N.W2V_RNG_PHILOX, KEY)
    d.set_schedule(N.W2V_SCHED_SEQUENTIAL); d.set_progress(0)
    W0, C0 = o.matrix(0), o.matrix(1)
    order = np.arange(len(sents))
    o.train_philox(0, 1, order, KEY, 0)
    st = d.train_epoch(0, order)
    W, Cm, _ = d.download_model()
    words, _ = o.vocab()
    print("case", sents, "dim", dim, "win", window, "K", K, st)
    for name, g, w, i in (("W", W, o.matrix(0), W0), ("C", Cm, o.matrix(1), C0)):
        for r in range(o.V):
            dg, dw = g[r] - i[r], w[r] - i[r]
            e = np.abs(dg - dw).max()
            if np.abs(dw).max() > 0 or np.abs(dg).max() > 0:
                print(f"  {name}[{words[r]}] |dw|={np.abs(dw).max():.4g} |dg|={np.abs(dg).max():.4g} err={e:.3g}",
                      "ratio", np.round((dg[:8] / np.where(dw[:8] == 0, 1, dw[:8])), 3))
    d.close()

run([["a", "b"]], 64, 1, 1)
run([["a", "b", "c"]], 64, 1, 1)
run([["a", "b", "a"]], 64, 1, 1)
run([["a", "b", "c", "d", "e", "f"]], 64, 2, 3)
run([["a", "b"]], 128, 1, 1)
