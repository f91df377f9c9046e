"""End-to-end quality gate (north star level 3): vectors trained by the GPU
path (parallel Hogwild wavefronts, Philox draws) score within ±1 point of the
oracle (sequential reference restatement) on analogy (3CosAdd accuracy) and
word similarity (Spearman x100), on the planted-relation corpus. Means over
seeds on both sides (oracle golden: tests/golden/quality_oracle.json)."""
import json
from pathlib import Path

import numpy as np
import pytest

from tests.golden.gen_quality_golden import CORPUS, ITERS, TRAIN, alpha
from tests.harness import MODES
from tests.quality import planted_corpus
from word2vec_amd.evaluate import analogy_accuracy, similarity_score
from word2vec_amd.model import Word2Vec

pytestmark = pytest.mark.gpu
GOLD = json.loads((Path(__file__).parent / "golden" / "quality_oracle.json").read_text())
SENTS, QS, PAIRS = planted_corpus(**CORPUS)


def gpu_scores(mode, seed):
    m = MODES[mode]
    w = Word2Vec(iter=ITERS[mode], window=TRAIN["window"], min_count=TRAIN["min_count"],
                 table_size=TRAIN["table_size"], word_dim=TRAIN["dim"], negative=m["negative"],
                 subsample_threshold=TRAIN["subsample"], init_alpha=alpha(mode), min_alpha=2.5e-6, cbow_mean=True,
                 train_method=m["train_method"], model=m["model"])
    w.seed(seed)
    w.build_vocab(SENTS)
    w.init_weights()
    w.train(SENTS)
    words, _ = w.vocab()
    E = w.matrix(1 if mode == "cbow_hs" else 0)
    return analogy_accuracy(words, E, QS)["accuracy"], similarity_score(words, E, PAIRS)["spearman"]


@pytest.mark.parametrize("mode", list(MODES))
def test_quality_within_one_point_of_oracle(mode):
    got = np.array([gpu_scores(mode, s) for s in (11, 12, 13)])
    ref = np.array([[r["analogy"], r["similarity"]] for r in GOLD["scores"][mode]])
    d_analogy = got[:, 0].mean() - ref[:, 0].mean()
    d_sim = got[:, 1].mean() - ref[:, 1].mean()
    print(f"{mode}: gpu {got.mean(0)} oracle {ref.mean(0)} delta analogy {d_analogy:+.2f} sim {d_sim:+.2f}")
    assert abs(d_analogy) <= 1.0, (mode, got, ref)
    assert abs(d_sim) <= 1.0, (mode, got, ref)
