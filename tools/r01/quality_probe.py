"""GPU quality across update policies on the planted-relation corpus (vs the oracle golden)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

from tests.golden.gen_quality_golden import CORPUS, ITERS, TRAIN, alpha  # noqa: E402
from tests.harness import MODES  # noqa: E402
from tests.quality import planted_corpus  # noqa: E402
from word2vec_amd.evaluate import analogy_accuracy, similarity_score  # noqa: E402
from word2vec_amd.model import Word2Vec  # noqa: E402

GOLD = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
sents, qs, pairs = planted_corpus(**CORPUS)
policies = [(-1, -1), (-1, 0), (0, -1), (0, 0), (10000, -1), (200, -1)]
out = {}
for mode in MODES:
    ref = np.mean([[r["analogy"], r["similarity"]] for r in GOLD["scores"][mode]], axis=0)
    for hot, priv in policies:
        m = MODES[mode]
        w = Word2Vec(iter=ITERS[mode], window=TRAIN["window"], min_count=TRAIN["min_count"],
                     table_size=TRAIN["table_size"], word_dim=TRAIN["dim"], negative=m["negative"],
                     subsample_threshold=TRAIN["subsample"], init_alpha=alpha(mode), min_alpha=2.5e-6,
                     cbow_mean=True, train_method=m["train_method"], model=m["model"], hot_rows=hot, private_rows=priv)
        w.seed(11)
        w.build_vocab(sents)
        w.init_weights()
        w.train(sents)
        words, _ = w.vocab()
        E = w.matrix(1 if mode == "cbow_hs" else 0)
        a = analogy_accuracy(words, E, qs)["accuracy"]
        s = similarity_score(words, E, pairs)["spearman"]
        out[f"{mode} hot={hot} priv={priv}"] = (round(a, 2), round(s, 2), round(ref[0], 2), round(ref[1], 2))
        print(mode, hot, priv, "gpu", round(a, 2), round(s, 2), "oracle", round(ref[0], 2), round(ref[1], 2), flush=True)
json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "/dev/stdout", "w"), indent=1)
