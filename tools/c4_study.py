#!/usr/bin/env python3
"""configs[3] at its own scale on ONE GPU (VERDICT r03 "next" 1): a 10 B-token
planted-relation Zipf corpus (V = 1 M filler ranks, SG-NS d300 w5 neg5,
subsample 1e-4, one epoch), trained by ONE replica and by R replicas on the
same device (a same-device w2v_group: every replica a full-concurrency training
handle, as on R GPUs; each trains a contiguous 1/R of the shuffled sentence
order as its own corpus) exchanging at the class's automatic cadence (64
exchanges per epoch: Word2Vec::sync_words = 0), in the mode Word2Vec::replica_mode
picks (auto: average for R > 2) or another. The corpus is generated on the
GPU (torch; tests/planted_ids.py's law: Zipf filler, entity / topic / role
words of a 50 x 4 grid planted at `planted` of the positions); 1000-token
sentences, no OOV (every rank occurs >= 5 times at 10 B tokens).

usage: c4_study.py [--tokens 1e10] [--planted 0.001] [--runs 1:auto,8:auto,8:sum]
       [--dim 300] [--mode sg_ns|sg_sn] [--negative 5] [--rounds 64] [--seed 1]
One JSON line per run: R, mode, analogy, similarity, delta to the R = 1 run,
train seconds (device), words/s."""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from tests.planted_ids import planted_zipf_ids_torch as gen_corpus, train_replicas  # noqa: E402


def run(args, data, R, gmode, dev, rounds):
    return train_replicas(data, R, gmode, rounds, args.dim, args.negative, args.mode, args.seed, dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=1e10)
    ap.add_argument("--filler", type=int, default=1_000_000)
    ap.add_argument("--planted", type=float, default=0.05)
    ap.add_argument("--planted-sents", type=float, default=1.0,
                    help="fraction of the sentences that carry planted words (at --planted of their positions)")
    ap.add_argument("--dim", type=int, default=300)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--mode", default="sg_ns", choices=["sg_ns", "sg_sn"])
    ap.add_argument("--rounds", type=int, default=64, help="exchanges per epoch (the class's automatic cadence)")
    ap.add_argument("--runs", default="1:auto,8:auto",
                    help="R:mode[:rounds][,...] (mode auto|sum|average|row_average|adaptive; rounds per epoch, "
                         "default --rounds)")
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.time()
    data = gen_corpus(int(args.tokens), args.filler, args.planted, args.seed, dev, planted_sents=args.planted_sents)
    print(json.dumps({"corpus_tokens": data[5], "V": int(data[1].size), "planted": args.planted, "planted_sents": args.planted_sents, "dim": args.dim,
                      "mode": args.mode, "negative": args.negative, "rounds_per_epoch": args.rounds,
                      "gen_s": round(time.time() - t0, 1)}), flush=True)
    base = None
    for spec in args.runs.split(","):
        f = spec.split(":")
        R, gm = int(f[0]), f[1]
        rounds = int(f[2]) if len(f) > 2 else args.rounds
        res, dt = run(args, data, R, gm, dev, rounds)
        rec = {"R": R, "gmode": gm, "rounds_per_epoch": rounds if R > 1 else 0, "train_s": round(dt, 2),
               "words_per_s": round(data[5] / dt, 1)}
        if res is None:
            rec["diverged"] = True
        else:
            rec.update(analogy=round(res[0], 2), similarity=round(res[1], 2))
            if R == 1:
                base = res
            elif base is not None:
                rec.update(d_analogy=round(res[0] - base[0], 2), d_similarity=round(res[1] - base[1], 2))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
