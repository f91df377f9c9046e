"""configs[4] shared-negatives: speed (bench) and text8-like / planted quality vs
the LDS-private C rows (private_rows, flush_centers); quality = mean of 3 seeds.
usage: python tools/sn_private_sweep.py [rows,flush ...]"""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

from tests.golden.gen_quality_golden import CORPUS, ITERS, TRAIN  # noqa: E402
from tests.golden.gen_quality_zipf_golden import ZCORPUS, ZTRAIN  # noqa: E402
from tests.quality import planted_corpus, planted_zipf_corpus  # noqa: E402
from word2vec_amd.evaluate import analogy_accuracy, similarity_score  # noqa: E402
from word2vec_amd.model import Word2Vec  # noqa: E402

P = planted_corpus(**CORPUS)
Z = planted_zipf_corpus(**ZCORPUS)
cases = [(0, 0), (8, 16), (8, 64), (8, 256), (4, 64), (2, 64)]
if len(sys.argv) > 1:
    cases = [tuple(int(x) for x in c.split(",")) for c in sys.argv[1:]]
for pr, fl in cases:
    res = []
    for (s, q, p), it, dim, ts, sub in ((P, ITERS["sg_ns"], TRAIN["dim"], TRAIN["table_size"], TRAIN["subsample"]),
                                        (Z, ZTRAIN["iters"], ZTRAIN["dim"], ZTRAIN["table_size"], ZTRAIN["subsample"])):
        got = []
        for seed in (11, 12, 13):
            w = Word2Vec(iter=it, window=5, min_count=5, table_size=ts, word_dim=dim, negative=5,
                         subsample_threshold=sub, init_alpha=0.025, min_alpha=2.5e-6, cbow_mean=True,
                         train_method="ns", model="sg", shared_negatives=True, verbose=False, private_rows=pr,
                         flush_centers=fl)
            w.seed(seed)
            w.build_vocab(s)
            w.init_weights()
            w.train(s)
            words, _ = w.vocab()
            E = w.matrix(0)
            got.append((analogy_accuracy(words, E, q)["accuracy"], similarity_score(words, E, p)["spearman"]))
        res.append(tuple(round(float(x), 2) for x in np.mean(got, axis=0)))
    b = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--mode", "sg_sn", "--dim", "512", "--negative", "15",
                        "--cpu-seconds", "0", "--steps", "1", "--private-rows", str(pr), "--flush-centers", str(fl)],
                       capture_output=True, text=True)
    v = json.loads(b.stdout.strip().splitlines()[-1])["value"] if b.returncode == 0 else b.stderr[-300:]
    print(f"private_rows {pr} flush {fl}: planted {res[0]} text8-like {res[1]} bench {v}", flush=True)
