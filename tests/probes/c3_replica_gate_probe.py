"""Sizing VERDICT r04 "next" 4: configs[3]'s shape (V 1 M filler ranks, SG-NS
d300 w5 neg5, subsample 1e-4) in the hard regime (planted words in a fraction
of the sentences), eight same-device replicas through the C++ class's
defaults (gpu_devices = {0 x 8}: auto mode, automatic cadence, overlap)
against one replica, the single-replica score taken as the mean of `ones`
runs (Hogwild run-to-run spread). One JSON line per run, then the deltas.

usage: c3_replica_gate_probe.py [--tokens 2.5e9] [--planted 0.05] [--planted-sents 0.08] [--ones 2] [--eights 1]
                                [--variants mode:rounds ...]
A variant runs the eight replicas with replica_mode `mode` (auto, sum, average,
row_average, adaptive) at `rounds` exchanges per epoch (0 = automatic)."""
import argparse
import json
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from tests.planted_ids import planted_zipf_ids_torch  # noqa: E402
from tests.test_gpu_replicas import _class_on_ids  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=2.5e9)
    ap.add_argument("--planted", type=float, default=0.05)
    ap.add_argument("--planted-sents", type=float, default=0.08)
    ap.add_argument("--ones", type=int, default=2)
    ap.add_argument("--eights", type=int, default=1)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--variants", nargs="*", default=[])
    a = ap.parse_args()
    t0 = time.time()
    data = planted_zipf_ids_torch(int(a.tokens), 1_000_000, a.planted, a.seed, torch.device("cuda", 0),
                                  planted_sents=a.planted_sents)
    print(json.dumps({"tokens": data[5], "V": int(data[1].size), "gen_s": round(time.time() - t0, 1)}), flush=True)
    with tempfile.TemporaryDirectory() as td:
        vp = Path(td) / "vocab.txt"
        vp.write_text("".join(f"{i} {c} {t}\n" for i, (t, c) in enumerate(zip(data[2], data[1]))))
        res = {"one": [], "eight": []}
        runs = [("one", None, a.ones, None), ("eight", [0] * 8, a.eights, None)]
        runs += [(v, [0] * 8, 1, v) for v in a.variants]
        for name, devs, n, var in runs:
            res.setdefault(name, [])
            for k in range(n):
                t0 = time.time()
                s = _class_on_ids_v(data, vp, devs, a.seed, var)
                res[name].append(s)
                print(json.dumps({"run": name, "k": k, "analogy": round(s[0], 2), "similarity": round(s[1], 2),
                                  "secs": round(time.time() - t0, 1)}), flush=True)
    one = np.mean(res["one"], 0)
    out = {"one_mean": one.round(2).tolist(), "one_spread": np.ptp(res["one"], 0).round(2).tolist()}
    for name in res:
        if name != "one" and res[name]:
            out[f"delta_{name}"] = (np.mean(res[name], 0) - one).round(2).tolist()
    print(json.dumps(out), flush=True)


def _class_on_ids_v(data, vp, devs, seed, var):
    """_class_on_ids with a replica_mode / cadence variant."""
    if var is None:
        return _class_on_ids(data, vp, devs, seed=seed, dim=300)
    from tests.planted_ids import scores
    from word2vec_amd.model import Word2Vec

    mode, rounds = var.split(":")
    ids, counts, words, qs, prs, raw = data
    sync = 0 if int(rounds) == 0 else max(1, raw // 8 // int(rounds))
    w = Word2Vec(iter=1, window=5, min_count=5, table_size=100_000_000, word_dim=300, negative=5,
                 subsample_threshold=1e-4, init_alpha=0.025, min_alpha=2.5e-6, cbow_mean=True, train_method="ns",
                 model="sg", gpu_devices=devs, sync_words=sync, replica_mode=mode, verbose=False)
    w.seed(seed)
    w.read_vocab(vp)
    w.make_table()
    w.precalc_sampling()
    w.init_weights()
    n_sent, L = ids.shape
    w.train_ids(ids.reshape(-1), np.arange(0, n_sent * L + 1, L, dtype=np.int64), raw)
    return scores(words, w.matrix(0), qs, prs, torch.device("cuda", 0))


if __name__ == "__main__":
    main()
