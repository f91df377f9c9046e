"""Sizing VERDICT r04 "next" 4: configs[3]'s shape (V 1 M filler ranks, SG-NS
d300 w5 neg5, subsample 1e-4) in the hard regime (planted words in a fraction
of the sentences), eight same-device replicas through the C++ class's
defaults (gpu_devices = {0 x 8}: auto mode, automatic cadence, overlap)
against one replica, the single-replica score taken as the mean of `ones`
runs (Hogwild run-to-run spread). One JSON line per run, then the deltas.

usage: c3_replica_gate_probe.py [--tokens 2.5e9] [--planted 0.05] [--planted-sents 0.08] [--ones 2] [--eights 1]"""
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
    a = ap.parse_args()
    t0 = time.time()
    data = planted_zipf_ids_torch(int(a.tokens), 1_000_000, a.planted, a.seed, torch.device("cuda", 0),
                                  planted_sents=a.planted_sents)
    print(json.dumps({"tokens": data[5], "V": int(data[1].size), "gen_s": round(time.time() - t0, 1)}), flush=True)
    with tempfile.TemporaryDirectory() as td:
        vp = Path(td) / "vocab.txt"
        vp.write_text("".join(f"{i} {c} {t}\n" for i, (t, c) in enumerate(zip(data[2], data[1]))))
        res = {"one": [], "eight": []}
        for name, devs, n in (("one", None, a.ones), ("eight", [0] * 8, a.eights)):
            for k in range(n):
                t0 = time.time()
                s = _class_on_ids(data, vp, devs, seed=a.seed, dim=300)
                res[name].append(s)
                print(json.dumps({"run": name, "k": k, "analogy": round(s[0], 2), "similarity": round(s[1], 2),
                                  "secs": round(time.time() - t0, 1)}), flush=True)
    one, eight = np.mean(res["one"], 0), np.mean(res["eight"], 0)
    print(json.dumps({"one_mean": one.round(2).tolist(), "one_spread": np.ptp(res["one"], 0).round(2).tolist(),
                      "eight_mean": eight.round(2).tolist(), "delta": (eight - one).round(2).tolist()}), flush=True)


if __name__ == "__main__":
    main()
