#!/usr/bin/env python3
"""Replica-exchange quality study on ONE GPU (VERDICT r02 "next" 1).

R replicas (R DeviceTrainer handles on cuda:0, one same-device w2v_group) each
train a contiguous shard of every epoch's shuffled sentence order at full
concurrency and exchange their updates every 1/rounds of an epoch (SUM,
AVERAGE or ROW_AVERAGE; blocking or overlapped), exactly as bench.py --gpus R
and Word2Vec::gpu_devices do across GPUs. Compared against ONE replica that
trains every sentence, at equal tokens, on a planted-relation Zipf corpus
(the text8-like gate corpus of tests/quality.py, scaled up, generated as ids
with numpy). Output: one JSON line per run (analogy, similarity, delta to the
single replica of the same seed).

usage: replica_study.py [--tokens N] [--replicas 8] [--rounds 1,8,32,128]
                        [--gmodes sum,average,row_average] [--seeds 1,2]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from word2vec_amd import _native as N  # noqa: E402
from word2vec_amd import host  # noqa: E402
from word2vec_amd.device import Config, DeviceTrainer  # noqa: E402
from word2vec_amd.replicas import NativeAverager  # noqa: E402
from tests.planted_ids import build, planted_zipf_ids, scores  # noqa: E402


def gpu_scores(words, E, qs, prs, dev):
    return scores(words, E, qs, prs, dev)


def train(args, R, rounds, gmode, overlap, seed, data, dev):
    ids, soff, counts, words, mode = data
    n = soff.size - 1
    hs = mode == "cbow_hs"
    cbow = mode.startswith("cbow")
    neg = 0 if hs else 5
    keep = host.sample_probs(counts, 1e-4)
    bounds = host.table_bounds(counts, 100_000_000) if neg else None
    codes = points = coff = None
    if hs:
        codes, points, coff = host.huffman(counts)
    V, d = counts.size, args.dim
    rng = np.random.default_rng(seed)
    W0 = ((rng.random((V, d), dtype=np.float32) - 0.5) / d).astype(np.float32)
    C0 = ((rng.random((V, d), dtype=np.float32) - 0.5) / d).astype(np.float32) if hs else \
        (np.zeros((V, d), np.float32) if (neg or cbow) else None)
    S0 = np.zeros((V - 1, d), np.float32) if hs else None
    a0 = (0.05 if cbow else 0.025) * (args.lr_scale if R > 1 else 1.0)  # linear LR scaling of the replicas
    cfg = Config(word_dim=d, window=5, negative=neg, hs=hs, cbow=cbow, cbow_mean=True, iter=args.iters,
                 init_alpha=a0, min_alpha=2.5e-6, table_size=100_000_000, device=0)
    reps = []
    for _ in range(R):
        t = DeviceTrainer(cfg)
        t.upload_vocab(keep, bounds, codes, points, coff)
        t.upload_model(W0, C0, S0)
        t.upload_corpus(ids, soff, int(args.raw_tokens))
        t.set_train_words(max(1, int(args.raw_tokens) // R))
        t.set_rng(N.W2V_RNG_PHILOX, (seed << 32) | 0x5EED)
        t.set_schedule(N.W2V_SCHED_PARALLEL)
        if args.hot_tau > 0:  # automatic hot rows at this threshold (0 = the library's rule by vocabulary)
            t.set_hot_auto(args.hot_tau, 1.0)
        if args.max_waves > 0:  # the same total concurrency for every R
            t.set_max_waves(max(1, args.max_waves // R))
        reps.append(t)
    g = None
    if R > 1:
        if gmode.startswith("sat"):  # sat<beta>: W2V_GROUP_SATURATION
            g = NativeAverager(reps, overlap=overlap, mode="sum")
            g.split_rows = g.set_saturation(max(1, int(args.raw_tokens) // R // rounds), float(gmode[3:]))
        elif gmode.startswith("split"):  # split<n*>: mean for rows saturated within a round (>= n* updates)
            g = NativeAverager(reps, overlap=overlap, mode="sum")
            g.split_rows = g.set_split(max(1, int(args.raw_tokens) // R // rounds), float(gmode[5:]))
        else:
            g = NativeAverager(reps, overlap=overlap, mode=gmode)
    lens = np.diff(soff)
    glob = 0
    t0 = time.time()
    for ep in range(args.iters):
        order = np.random.default_rng(1000 * seed + ep).permutation(n).astype(np.int64)
        shards = [order[n * i // R: n * (i + 1) // R] for i in range(R)]
        cums = []
        for t, sh in zip(reps, shards):
            t.set_order(sh)
            cums.append(np.concatenate([[0], np.cumsum(lens[sh])]))
        # `rounds` full exchanges per epoch; with --hot-rows K, hot-row exchanges
        # (W / C rows [0, K), the nodes nearest the root) at --hot-rounds per epoch between them
        sub = max(rounds, args.hot_rounds) if args.hot_rows > 0 else rounds
        per_full = max(1, sub // rounds)
        for r in range(sub):
            words_r = 0
            for t, sh, cu in zip(reps, shards, cums):
                m = sh.size
                lo, hi = m * r // sub, m * (r + 1) // sub
                t.set_progress_async(glob // R)
                if hi > lo:
                    t.train_slice_async(ep, lo, hi - lo)
                words_r += int(cu[hi] - cu[lo])
            if g is not None:
                g.average(0 if (r + 1) % per_full == 0 else args.hot_rows)
            glob += words_r
        if g is not None:
            g.finish()
        for t in reps:
            t.synchronize()
    dt = time.time() - t0
    Wf, Cf, _ = reps[0].download_model()
    diverged = any(t.read_stats()["nonfinite"] > 0 for t in reps)
    if g is not None:
        g.close()
    for t in reps:
        t.close()
    return (None if diverged else (Cf if hs else Wf)), dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=50_000_000)
    ap.add_argument("--filler", type=int, default=200_000)
    ap.add_argument("--dim", type=int, default=100)
    ap.add_argument("--iters", type=int, default=1)
    ap.add_argument("--mode", default="sg_ns")
    ap.add_argument("--replicas", default="8")
    ap.add_argument("--rounds", default="1,8,32,128")
    ap.add_argument("--gmodes", default="sum,average,row_average")
    ap.add_argument("--overlap", type=int, default=1)
    ap.add_argument("--seeds", default="1")
    ap.add_argument("--planted-frac", type=float, default=0.10)
    ap.add_argument("--hot-rows", type=int, default=0, help="hot rows exchanged between the full exchanges (0 = none)")
    ap.add_argument("--hot-rounds", type=int, default=0, help="hot-row exchanges per epoch")
    ap.add_argument("--hot-tau", type=float, default=0.0, help="automatic hot-row threshold (0 = by vocabulary)")
    ap.add_argument("--lr-scale", type=float, default=1.0, help="init_alpha x this for R > 1 (linear scaling rule)")
    ap.add_argument("--max-waves", type=int, default=0, help="cap the waves of all R replicas together (each gets max_waves // R; 0 = full chip each)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.time()
    tok, n_sent, names, qs, prs = planted_zipf_ids(args.tokens, filler=args.filler, planted_frac=args.planted_frac,
                                                   seed=0)
    args.raw_tokens = tok.size
    ids, soff, counts, words = build(tok, n_sent, 1000, names)
    del tok
    print(json.dumps({"corpus_tokens": int(args.raw_tokens), "in_vocab": int(ids.size), "V": int(counts.size),
                      "sentences": int(n_sent), "gen_s": round(time.time() - t0, 1), "mode": args.mode,
                      "dim": args.dim, "iters": args.iters, "planted_frac": args.planted_frac,
                      "max_waves": args.max_waves, "lr_scale": args.lr_scale, "hot_tau": args.hot_tau}), flush=True)
    data = (ids, soff, counts, words, args.mode)
    for seed in [int(s) for s in args.seeds.split(",")]:
        hr = args.hot_rows
        args.hot_rows = 0
        E, dt = train(args, 1, 1, "sum", False, seed, data, dev)
        args.hot_rows = hr
        a1, s1 = gpu_scores(words, E, qs, prs, dev)
        print(json.dumps({"seed": seed, "R": 1, "analogy": round(a1, 2), "similarity": round(s1, 2),
                          "train_s": round(dt, 2)}), flush=True)
        for R in [int(x) for x in args.replicas.split(",") if x]:
            for rounds in [int(x) for x in args.rounds.split(",") if x]:
                for gm in args.gmodes.split(","):
                    E, dt = train(args, R, rounds, gm, bool(args.overlap), seed, data, dev)
                    if E is None:
                        print(json.dumps({"seed": seed, "R": R, "rounds_per_epoch": rounds, "gmode": gm,
                                          "hot_rows": args.hot_rows, "hot_rounds": args.hot_rounds,
                                          "overlap": bool(args.overlap), "diverged": True}), flush=True)
                        continue
                    a, s = gpu_scores(words, E, qs, prs, dev)
                    print(json.dumps({"seed": seed, "R": R, "rounds_per_epoch": rounds, "gmode": gm,
                                      "hot_rows": args.hot_rows, "hot_rounds": args.hot_rounds,
                                      "overlap": bool(args.overlap), "analogy": round(a, 2),
                                      "similarity": round(s, 2), "d_analogy": round(a - a1, 2),
                                      "d_similarity": round(s - s1, 2), "train_s": round(dt, 2)}), flush=True)


if __name__ == "__main__":
    main()
