"""Quality of the per-pair kernel (SG-NS, the reference's update) vs wavefronts in
flight, on the text8-like planted corpus: where does the GPU's margin over the
sequential oracle come from? usage: python tools/quality_concurrency.py"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import json  # noqa: E402

import numpy as np  # noqa: E402

from tests.golden.gen_quality_zipf_golden import ZCORPUS, ZTRAIN  # noqa: E402
from tests.quality import planted_zipf_corpus  # noqa: E402
from word2vec_amd.evaluate import analogy_accuracy, similarity_score  # noqa: E402
from word2vec_amd.model import Word2Vec  # noqa: E402

ZGOLD = json.loads((ROOT / "tests" / "golden" / "quality_zipf_oracle.json").read_text())
ref = np.array([[r["analogy"], r["similarity"]] for r in ZGOLD["scores"]]).mean(0)
s, q, p = planted_zipf_corpus(**ZCORPUS)
policies = [("default policy", {}), ("plain Hogwild", dict(hot_rows=0, private_rows=0))]
for name, pol in policies:
    for mw in (1, 16, 256, 2048, 0):
        w = Word2Vec(iter=ZTRAIN["iters"], window=5, min_count=5, table_size=ZTRAIN["table_size"],
                     word_dim=ZTRAIN["dim"], negative=5, subsample_threshold=ZTRAIN["subsample"], init_alpha=0.025,
                     min_alpha=2.5e-6, cbow_mean=True, train_method="ns", model="sg", verbose=False, max_waves=mw,
                     **pol)
        w.seed(11)
        w.build_vocab(s)
        w.init_weights()
        w.train(s)
        words, _ = w.vocab()
        E = w.matrix(0)
        print(f"{name}, max_waves {mw}: analogy {analogy_accuracy(words, E, q)['accuracy']:.2f} "
              f"similarity {similarity_score(words, E, p)['spearman']:.2f} (sequential oracle {ref[0]:.2f} "
              f"{ref[1]:.2f})", flush=True)
