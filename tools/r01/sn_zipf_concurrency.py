"""Shared-negatives quality on the text8-like corpus (V ~98K, neg 5, the
test_gpu_quality gate) vs workgroups in flight, 3 seeds each.
usage: python tools/sn_zipf_concurrency.py [max_waves ...] [seeds=11,12] [hot_rows=N]"""
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

ZGOLD = json.loads((ROOT / "tests" / "golden" / "quality_zipf_oracle.json").read_text())
ref = np.mean([[r["analogy"], r["similarity"]] for r in ZGOLD["scores"]], axis=0)
zs, zq, zp = planted_zipf_corpus(**ZCORPUS)
args = [a for a in sys.argv[1:] if not a.startswith(("seeds=", "hot_rows="))]
hot = next((int(a[9:]) for a in sys.argv[1:] if a.startswith("hot_rows=")), 1000)
seeds = next((tuple(int(x) for x in a[6:].split(",")) for a in sys.argv[1:] if a.startswith("seeds=")), (11, 12, 13))
for mw in [int(a) for a in args] or (0, 512, 256):
    got = []
    for seed in seeds:
        w = Word2Vec(iter=ZTRAIN["iters"], window=5, min_count=5, table_size=ZTRAIN["table_size"],
                     word_dim=ZTRAIN["dim"], negative=5, subsample_threshold=ZTRAIN["subsample"], init_alpha=0.025,
                     min_alpha=2.5e-6, cbow_mean=True, train_method="ns", model="sg", shared_negatives=True,
                     verbose=False, max_waves=mw, hot_rows=hot)
        w.seed(seed)
        w.build_vocab(zs)
        w.init_weights()
        w.train(zs)
        words, _ = w.vocab()
        E = w.matrix(0)
        got.append([analogy_accuracy(words, E, zq)["accuracy"], similarity_score(words, E, zp)["spearman"]])
    got = np.array(got)
    print(f"hot_rows {hot} max_waves {mw}: per seed {got.round(2).tolist()} mean delta {(got.mean(0) - ref).round(2)}", flush=True)
