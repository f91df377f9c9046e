"""Quality of plain updates with write-through (sc1) loads/stores, and of HS under concurrency caps."""
import os, sys, json
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np
from tests.golden.gen_quality_golden import CORPUS, ITERS, TRAIN, alpha
from tests.harness import MODES
from tests.quality import planted_corpus
from word2vec_amd.evaluate import analogy_accuracy, similarity_score
from word2vec_amd.model import Word2Vec
sents, qs, pairs = planted_corpus(**CORPUS)
GOLD = json.loads((ROOT / "tests" / "golden" / "quality_oracle.json").read_text())
def run(mode, hot, priv, env):
    for k in ("W2V_FRESH_LOADS", "W2V_DEBUG_MAX_BLOCKS", "W2V_FLUSH_EVERY"):
        os.environ.pop(k, None)
    os.environ.update(env)
    m = MODES[mode]
    ref = np.mean([[r["analogy"], r["similarity"]] for r in GOLD["scores"][mode]], axis=0)
    w = Word2Vec(iter=ITERS[mode], window=5, min_count=5, table_size=10_000_000, word_dim=64, negative=m["negative"],
                 subsample_threshold=1e-3, init_alpha=alpha(mode), min_alpha=2.5e-6, cbow_mean=True,
                 train_method=m["train_method"], model=m["model"], hot_rows=hot, private_rows=priv)
    w.seed(11); w.build_vocab(sents); w.init_weights(); w.train(sents)
    words, _ = w.vocab()
    E = w.matrix(1 if mode == "cbow_hs" else 0)
    print(f"{mode} hot={hot} priv={priv} {env}: analogy {analogy_accuracy(words, E, qs)['accuracy']:.2f} "
          f"sim {similarity_score(words, E, pairs)['spearman']:.2f} (oracle {ref[0]:.2f} {ref[1]:.2f})", flush=True)
for F in (1, 2, 4, 8, 16):
    for mode in ("sg_ns", "cbow_hs"):
        run(mode, -1, -1, {"W2V_FLUSH_EVERY": str(F)})

# realistic text8-like corpus (10M tokens, 10K sentences, V~98K), SG-NS
from tests.quality import planted_zipf_corpus  # noqa: E402
ZS, ZQ, ZP = planted_zipf_corpus(n_tokens=10_000_000, sent_len=1000, planted_frac=0.10, seed=0)


def zrun(hot, priv, env):
    for k in ("W2V_FRESH_LOADS", "W2V_DEBUG_MAX_BLOCKS", "W2V_FLUSH_EVERY"):
        os.environ.pop(k, None)
    os.environ.update(env)
    w = Word2Vec(iter=1, window=5, min_count=5, table_size=100_000_000, word_dim=100, negative=5,
                 subsample_threshold=1e-4, init_alpha=0.025, min_alpha=2.5e-6, cbow_mean=True,
                 train_method="ns", model="sg", hot_rows=hot, private_rows=priv)
    w.seed(11); w.build_vocab(ZS); w.init_weights(); w.train(ZS)
    words, _ = w.vocab()
    E = w.matrix(0)
    print(f"ZIPF sg_ns hot={hot} priv={priv} {env}: analogy {analogy_accuracy(words, E, ZQ)['accuracy']:.2f} "
          f"sim {similarity_score(words, E, ZP)['spearman']:.2f} (oracle ~71)", flush=True)


for hot, priv, env in [(0, 0, {}), (-1, 0, {}), (-1, -1, {"W2V_FLUSH_EVERY": "8"}), (10000, -1, {"W2V_FLUSH_EVERY": "8"}),
                       (10000, -1, {"W2V_FLUSH_EVERY": "1"}), (0, -1, {"W2V_FLUSH_EVERY": "8"})]:
    zrun(hot, priv, env)
