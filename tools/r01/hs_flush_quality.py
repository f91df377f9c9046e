"""Quality of the HS modes vs the flush interval of the LDS-private Huffman
nodes: text8-like corpus (CBOW-HS, 3 seeds, against its oracle golden).
usage: python tools/hs_flush_quality.py [flush ...]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

from tests.golden.gen_quality_zipf_golden import ZCORPUS, ZTRAIN  # noqa: E402
from tests.quality import planted_zipf_corpus  # noqa: E402
from word2vec_amd.evaluate import analogy_accuracy, similarity_score  # noqa: E402
from word2vec_amd.model import Word2Vec  # noqa: E402

G = json.loads((ROOT / "tests" / "golden" / "quality_zipf_cbow_hs_oracle.json").read_text())
ref = np.mean([[r["analogy"], r["similarity"]] for r in G["scores"]], axis=0)
zs, zq, zp = planted_zipf_corpus(**ZCORPUS)
for fl in [int(a) for a in sys.argv[1:]] or (0, 32, 64):
    got = []
    for seed in (11, 12, 13):
        w = Word2Vec(iter=ZTRAIN["iters"], window=5, min_count=5, table_size=ZTRAIN["table_size"],
                     word_dim=ZTRAIN["dim"], negative=0, subsample_threshold=ZTRAIN["subsample"], init_alpha=0.05,
                     min_alpha=2.5e-6, cbow_mean=True, train_method="hs", model="cbow", verbose=False,
                     flush_centers=fl)
        w.seed(seed)
        w.build_vocab(zs)
        w.init_weights()
        w.train(zs)
        words, _ = w.vocab()
        E = w.matrix(1)
        got.append([analogy_accuracy(words, E, zq)["accuracy"], similarity_score(words, E, zp)["spearman"]])
    got = np.array(got)
    print(f"cbow_hs text8-like flush {fl}: per seed {got.round(2).tolist()} mean delta {(got.mean(0) - ref).round(2)}",
          flush=True)
