"""Probe (not a test): configs[4]'s shared-negatives quality gate
(tests/test_gpu_quality.py::test_quality_shared_negatives_not_below_oracle)
at other LDS-private row counts. Usage: python -m tests.probes.sn_quality_probe -1 8 6"""
import sys

import numpy as np

from tests.golden.gen_quality_golden import ITERS, TRAIN
from tests.golden.gen_quality_zipf_golden import ZCORPUS, ZTRAIN
from tests.quality import planted_zipf_corpus
from tests.test_gpu_quality import GOLD, PAIRS, QS, SENTS, ZGOLD
from word2vec_amd.evaluate import analogy_accuracy, similarity_score
from word2vec_amd.model import Word2Vec


def train(sents, iters, dim, table, sub, seed, private_rows):
    w = Word2Vec(iter=iters, window=5, min_count=5, table_size=table, word_dim=dim, negative=5,
                 subsample_threshold=sub, init_alpha=0.025, min_alpha=2.5e-6, cbow_mean=True, train_method="ns",
                 model="sg", shared_negatives=True, verbose=False, private_rows=private_rows)
    w.seed(seed)
    w.build_vocab(sents)
    w.init_weights()
    w.train(sents)
    words, _ = w.vocab()
    return words, w.matrix(0)


def main(prs):
    zs = planted_zipf_corpus(**ZCORPUS)
    for corpus in ("planted", "text8-like"):
        if corpus == "planted":
            sents, qs, pairs = SENTS, QS, PAIRS
            args = (ITERS["sg_ns"], TRAIN["dim"], TRAIN["table_size"], TRAIN["subsample"])
            ref = np.array([[r["analogy"], r["similarity"]] for r in GOLD["scores"]["sg_ns"]]).mean(0)
        else:
            sents, qs, pairs = zs
            args = (ZTRAIN["iters"], ZTRAIN["dim"], ZTRAIN["table_size"], ZTRAIN["subsample"])
            ref = np.array([[r["analogy"], r["similarity"]] for r in ZGOLD["scores"]]).mean(0)
        for pr in prs:
            got = []
            for seed in (11, 12, 13):
                words, E = train(sents, *args, seed, pr)
                got.append([analogy_accuracy(words, E, qs)["accuracy"], similarity_score(words, E, pairs)["spearman"]])
            got = np.array(got).mean(0)
            print(f"shared-negatives {corpus} private_rows={pr}: gpu {got.round(2)} oracle {ref.round(2)} "
                  f"delta {(got - ref).round(2)}", flush=True)


if __name__ == "__main__":
    main([int(x) for x in sys.argv[1:]] or [-1, 8])
