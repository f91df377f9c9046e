"""Cost of the lifted hyper-parameter limits (ns_word_many's
duplicate test and cbow_center_huge's span walk are quadratic in negative / 64
and in the window). The parallel schedule, Philox draws, one epoch over a
Zipf corpus (100 sentences x 1000 tokens, d 64), per setting: wall
time, kept centers, targets, and the time per target row update relative to
the small path's. One JSON line per setting.

usage: limits_cost_probe.py [neg|win ...]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from tests.corpus import zipf_sentences  # noqa: E402
from tests.harness import device_from_oracle, oracle_run  # noqa: E402
from word2vec_amd import _native as N  # noqa: E402
from word2vec_amd.device import Config  # noqa: E402

SENTS = None


def run(mode, window, negative, timeout_s=60.0):
    global SENTS
    if SENTS is None:
        SENTS = zipf_sentences(100, 1000, 20000, seed=61)
    o = oracle_run(SENTS, mode, dim=64, window=5, iters=1, table_size=1_000_000, train=False)
    o.build_sample()
    cfg = Config(word_dim=64, window=window, negative=negative, hs=False, cbow=mode == "cbow_ns", cbow_mean=True,
                 iter=1, init_alpha=0.0025, min_alpha=2.5e-6, table_size=1_000_000)
    d = device_from_oracle(o, cfg, initial=False)
    d.set_rng(N.W2V_RNG_PHILOX, 5)
    d.set_schedule(N.W2V_SCHED_PARALLEL)
    d.set_progress(0)
    order = np.random.default_rng(3).permutation(len(SENTS))
    d.train_epoch(0, order)  # warm-up (code objects, table)
    d.set_progress(0)
    d.reset_stats()
    t0 = time.perf_counter()
    st = d.train_epoch(0, order)
    dt = time.perf_counter() - t0
    d.close()
    return {"mode": mode, "window": window, "negative": negative, "secs": round(dt, 4),
            "words_per_s": round(st["words"] / dt), "centers": st["centers"], "targets": st["targets"],
            "ns_per_target": round(dt * 1e9 / max(1, st["targets"]), 2), "nonfinite": st["nonfinite"]}


if __name__ == "__main__":
    what = sys.argv[1:] or ["neg", "win"]
    if "neg" in what:
        for neg in (5, 63, 64, 256, 1024, 2048, 4096):
            print(json.dumps(run("sg_ns", 5, neg)), flush=True)
    if "win" in what:
        for win in (5, 127, 128, 256, 512, 1024, 2048):
            print(json.dumps(run("cbow_ns", win, 5)), flush=True)
