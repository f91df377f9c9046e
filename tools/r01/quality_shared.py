"""Quality of the shared-negatives minibatch (GPU, parallel) against the oracle's
per-pair reference goldens, on the planted corpus and the text8-like corpus."""
import json
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

GOLD = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
ZGOLD = json.loads((ROOT / "tests" / "golden" / "quality_zipf_oracle.json").read_text())


def run(sents, qs, pairs, neg, iters, dim, table, sub, seed, shared, alpha=0.025):
    w = Word2Vec(iter=iters, window=5, min_count=5, table_size=table, word_dim=dim, negative=neg,
                 subsample_threshold=sub, init_alpha=alpha, min_alpha=2.5e-6, cbow_mean=True, train_method="ns",
                 model="sg", shared_negatives=shared, verbose=False)
    w.seed(seed)
    w.build_vocab(sents)
    w.init_weights()
    w.train(sents)
    words, _ = w.vocab()
    E = w.matrix(0)
    return analogy_accuracy(words, E, qs)["accuracy"], similarity_score(words, E, pairs)["spearman"]


sents, qs, pairs = planted_corpus(**CORPUS)
ref = np.mean([[r["analogy"], r["similarity"]] for r in GOLD["scores"]["sg_ns"]], axis=0)
for shared in (False, True):
    for neg in (5, 15):
        got = np.mean([run(sents, qs, pairs, neg, ITERS["sg_ns"], TRAIN["dim"], TRAIN["table_size"], TRAIN["subsample"],
                           s, shared) for s in (11, 12, 13)], axis=0)
        print(f"planted shared={shared} neg={neg}: gpu {got.round(2)} oracle(neg5 per-pair) {ref.round(2)}", flush=True)
zs, zq, zp = planted_zipf_corpus(**ZCORPUS)
zref = np.mean([[r["analogy"], r["similarity"]] for r in ZGOLD["scores"]], axis=0)
for shared in (False, True):
    for neg in (5, 15):
        got = run(zs, zq, zp, neg, ZTRAIN["iters"], ZTRAIN["dim"], ZTRAIN["table_size"], ZTRAIN["subsample"], 11,
                  shared)
        print(f"text8-like shared={shared} neg={neg}: gpu {np.round(got, 2)} oracle(neg5 per-pair) {zref.round(2)}",
              flush=True)
