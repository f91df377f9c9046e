#!/usr/bin/env python3
"""Throughput bench for the Word2Vec hot path on MI355X.

Workload (BASELINE.json configs[2], the 1-GPU headline config): skip-gram,
negative sampling neg=5, dim=300, window=5, subsample 1e-4, min_count 5, on a
synthetic Zipf(s=1) corpus over 1M word ranks in 1000-token sentences (the
1B-Word corpus is not available offline). One "step" = one training pass
(epoch) of the hot path over this rank's shard, inputs already resident in HBM.
With N GPUs (torchrun), every rank trains its own shard of the same size on a
full model replica and the replicas are averaged by the library's RCCL group
(include/w2v_dev.h w2v_group_*, overlapped with the next round) after every
step (weak scaling); torch.distributed (gloo) carries only control messages.

Prints ONE JSON line on rank 0 (metric/value/unit/... + roofline + cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

MODES = {
    "sg_ns": dict(cbow=False, hs=False),
    "sg_hs": dict(cbow=False, hs=True),
    "cbow_ns": dict(cbow=True, hs=False),
    "cbow_hs": dict(cbow=True, hs=True),
    # configs[4]: shared-negatives minibatch SGNS on the matrix cores (run with --dim 512 --negative 15)
    "sg_sn": dict(cbow=False, hs=False, shared=True),
}
MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X dense f32-input MFMA (MI355X_MICROARCH.md)
# configs[3] (10 B tokens over N GPUs) under Word2Vec::sync_words = 0 (the
# class's automatic cadence, 64 exchanges per epoch: Word2Vec.cpp
# kAutoReplicaRounds): one exchange per 10e9 / N / 64 words of a replica's
# shard, in the class's auto mode for that shard (Word2Vec::replica_mode: the
# mean for N <= 4 — 2.5-5 B-word shards —, the adaptive divisor for more).
# bench.py --gpus N is configs[3]'s per-GPU step, so it exchanges at that
# cadence and in that mode — what the product runs on that workload.
CONFIG3_TOKENS = 10_000_000_000
AUTO_ROUNDS, AUTO_AVERAGE_WORDS, AUTO_AVERAGE_REPLICAS = 64, 4_000_000, 4  # include/Word2Vec.h
AUTO_ADAPTIVE_ROUNDS = 128  # Word2Vec::kAutoAdaptiveRounds: the adaptive divisor's cadence


def config3_sync_words(world, mode="adaptive"):
    rounds = AUTO_ADAPTIVE_ROUNDS if mode == "adaptive" else AUTO_ROUNDS
    return CONFIG3_TOKENS // max(1, world) // rounds


def auto_replica_mode(world, shard_words=None):
    """Word2Vec::replica_mode auto (Word2Vec.cpp run_epochs_replicas) for
    `world` replicas of configs[3]'s shards (or shards of `shard_words`)."""
    shard = CONFIG3_TOKENS // max(1, world) if shard_words is None else shard_words
    if world <= AUTO_AVERAGE_REPLICAS and shard >= AUTO_ROUNDS * AUTO_AVERAGE_WORDS:
        return "average"
    return "sum" if world <= 2 else "adaptive"

# BASELINE.json configs on this bench's synthetic Zipf corpora (text8 and the
# 1B-Word corpus are not available offline): --config cN sets these fields.
CONFIGS = {
    # text8-shaped (configs[0] / [1]): 17 M tokens, p(r) ~ (r + 4)^-1.30 over 350 K ranks gives V ~ 71 K at
    # min_count 5, ~254 K types, the most frequent word 6 % of tokens (text8: 71,290 / 253,854 / 6.2 %)
    "c1": dict(mode="sg_ns", dim=100, negative=5, vocab=350_000, zipf_s=1.30, zipf_q=4.0, tokens=17_000_000),
    "c2": dict(mode="cbow_hs", dim=200, negative=0, vocab=350_000, zipf_s=1.30, zipf_q=4.0, tokens=17_000_000),
    "c3": dict(mode="sg_ns", dim=300, negative=5, vocab=1_000_000, tokens=50_000_000),  # 1B-Word stand-in (default)
    "c4": dict(mode="sg_ns", dim=300, negative=5, vocab=1_000_000, tokens=50_000_000),  # per GPU of the N-GPU run
    "c5": dict(mode="sg_sn", dim=512, negative=15, vocab=1_000_000, tokens=50_000_000),  # shared-negatives MFMA
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=list(CONFIGS), default=None,
                    help="BASELINE.json config preset (the defaults of --mode/--dim/--negative/--vocab/--tokens/...)")
    ap.add_argument("--mode", default="sg_ns", choices=list(MODES))
    ap.add_argument("--dim", type=int, default=300)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--vocab", type=int, default=1_000_000, help="Zipf rank range (V before min_count)")
    ap.add_argument("--tokens", type=int, default=50_000_000, help="raw tokens per GPU per step")
    ap.add_argument("--sent-len", type=int, default=1000)
    ap.add_argument("--zipf-s", type=float, default=1.0, help="corpus law p(rank) ~ (rank + q)^-s (1 = Zipf)")
    ap.add_argument("--zipf-q", type=float, default=0.0, help="Zipf-Mandelbrot offset q of the corpus law")
    ap.add_argument("--subsample", type=float, default=1e-4)
    ap.add_argument("--min-count", type=int, default=5)
    ap.add_argument("--table-size", type=int, default=100_000_000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget (0 = skip)")
    # update policy of the parallel schedule (include/w2v_dev.h); defaults = the library's
    ap.add_argument("--hot-rows", type=int, default=-2,
                    help="rows updated with atomics (-2 auto from the corpus statistics, -1 all, 0 none = plain "
                         "Hogwild RMW, k = k most frequent)")
    ap.add_argument("--hot-auto", type=float, nargs=2, default=[0.0, 1.0], metavar=("ROWS", "NODES"),
                    help="thresholds of the automatic hot rows (expected updates in flight of a W / C row, a node; "
                         "rows 0 = the library default, 1)")
    ap.add_argument("--private-rows", type=int, default=-1,
                    help="hottest output rows privatised per workgroup in LDS (-1 auto, 0 off)")
    ap.add_argument("--private-rate", type=float, default=None,
                    help="privatise only rows updated >= this many times per center (default: the library's)")
    ap.add_argument("--flush-centers", type=int, default=0,
                    help="workgroup centers between private-row flushes (0 = auto)")
    ap.add_argument("--private-average", type=float, default=8.0,
                    help="concurrency the private rows' summed deltas are scaled to (0 = plain sum)")
    ap.add_argument("--context-rows", type=int, default=-1,
                    help="CBOW: hottest context rows privatised in LDS (-1 auto, 0 off)")
    ap.add_argument("--context-flush", type=int, default=0, help="CBOW: centers between context-row flushes (0 auto)")
    ap.add_argument("--max-waves", type=int, default=0, help="wavefronts in flight (0 = all that fit)")
    ap.add_argument("--own-model", action="store_true",
                    help="N=1 only: let the library allocate the matrices instead of torch")
    ap.add_argument("--sync-every", type=int, default=0,
                    help="N>1: exchange every this many sentences of a shard (0 = by --sync-words)")
    ap.add_argument("--sync-words", type=int, default=0,
                    help="N>1: exchange every this many in-vocab words of a shard (0: the class's automatic "
                         "cadence on configs[3], 64 exchanges per epoch of a 10 B / N-token shard)")
    ap.add_argument("--replica-mode", default="auto", choices=["auto", "sum", "average", "row_average", "adaptive"],
                    help="N>1: how the replicas' updates combine (auto: as Word2Vec::replica_mode on configs[3]'s "
                         "shards: average for <= 4 ranks, adaptive for more; DESIGN.md §6.2)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: average the replicas in place on the training stream instead of from a snapshot "
                         "on a communication stream overlapped with the next round")
    pre, _ = ap.parse_known_args()
    if pre.config:  # the preset's values are defaults: flags given explicitly still win (e.g. --mode)
        ap.set_defaults(**CONFIGS[pre.config])
    return ap.parse_args()


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # W2V_BENCH_SHARE_GPU=1 rehearses the N>1 path on a one-GPU box: every rank
    # on cuda:0, gloo instead of RCCL (numbers from such a run are not bench lines)
    share = os.environ.get("W2V_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # control plane only (vocab counts, the group id, barriers, max time):
        # the replicas are averaged by the library's own RCCL group
        dist.init_process_group("gloo")

    from word2vec_amd import _native as N
    from word2vec_amd import host
    from word2vec_amd.device import Config, DeviceTrainer
    from word2vec_amd.replicas import (agree_rounds, global_round_words, local_round_words, make_averager, n_rounds,
                                       train_rounds)

    mode = MODES[args.mode]
    neg = 0 if mode["hs"] else args.negative
    d = args.dim

    # ---- synthetic corpus shard (on the GPU, seeded per rank) ------------------
    t0 = time.time()
    n_sent = args.tokens // args.sent_len
    n_tok = n_sent * args.sent_len
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed * 1000 + rank)
    p = torch.arange(1, args.vocab + 1, device=dev, dtype=torch.float64).add_(args.zipf_q).pow_(-args.zipf_s)
    cdf = torch.cumsum(p, 0)
    cdf /= cdf[-1].clone()
    ranks = torch.empty(n_tok, dtype=torch.int64, device=dev)
    chunk = 1 << 24
    for s in range(0, n_tok, chunk):
        e = min(n_tok, s + chunk)
        u = torch.rand(e - s, generator=g, device=dev, dtype=torch.float64)
        ranks[s:e] = torch.searchsorted(cdf, u, right=True).clamp_(max=args.vocab - 1)
        del u
    counts = torch.bincount(ranks, minlength=args.vocab)
    if world > 1:  # one vocab for all replicas (built over the whole corpus)
        cc = counts.cpu()
        dist.all_reduce(cc)
        counts = cc.to(dev)
    order = torch.argsort(counts, descending=True, stable=True)
    V = int((counts >= args.min_count).sum())
    vocab_ranks = order[:V]
    remap = torch.full((args.vocab,), -1, dtype=torch.int64, device=dev)
    remap[vocab_ranks] = torch.arange(V, device=dev)
    ids = remap[ranks]
    del ranks
    inv = ids >= 0
    lens = inv.view(n_sent, args.sent_len).sum(1)
    soff = torch.zeros(n_sent + 1, dtype=torch.int64, device=dev)
    soff[1:] = torch.cumsum(lens, 0)
    ids_iv = ids[inv].to(torch.int32)
    del ids, inv
    counts_v = counts[vocab_ranks].cpu().numpy().astype(np.int64)
    ids_h = ids_iv.cpu().numpy()
    soff_h = soff.cpu().numpy()
    del ids_iv
    log(f"[bench] corpus: {n_tok} raw tokens/rank, {ids_h.size} in-vocab, V={V}, {time.time() - t0:.1f}s")

    # ---- host products (bit-exact restatements) + device residency -------------
    t0 = time.time()
    keep = host.sample_probs(counts_v, args.subsample)
    bounds = host.table_bounds(counts_v, args.table_size) if neg > 0 else None
    codes = points = coff = None
    if mode["hs"]:
        codes, points, coff = host.huffman(counts_v)
    iters_total = args.warmup + args.steps
    cfg = Config(word_dim=d, window=args.window, negative=neg, hs=mode["hs"], cbow=mode["cbow"],
                 cbow_mean=True, iter=iters_total, init_alpha=0.025 if not mode["cbow"] else 0.05,
                 min_alpha=2.5e-6, table_size=args.table_size, device=local)
    tr = DeviceTrainer(cfg)
    stream = torch.cuda.Stream(device=dev)  # the kernels, the events and RCCL all run on this stream
    torch.cuda.set_stream(stream)
    tr.set_stream(stream.cuda_stream)
    tr.upload_vocab(keep, bounds, codes, points, coff)
    pitch = tr.row_pitch()  # the kernels' row width (64 x floats per lane), zero padding
    vrows = V
    gW = torch.Generator(device=dev)
    gW.manual_seed(args.seed)  # identical initial replicas on every rank
    W = torch.zeros(vrows, pitch, dtype=torch.float32, device=dev)
    W[:V, :d] = (torch.rand(V, d, generator=gW, device=dev) - 0.5) / d
    Cm = torch.zeros(vrows, pitch, dtype=torch.float32, device=dev) if (neg > 0 or mode["cbow"]) else None
    if Cm is not None and mode["cbow"] and mode["hs"]:
        Cm[:V, :d] = (torch.rand(V, d, generator=gW, device=dev) - 0.5) / d
    S = torch.zeros(max(vrows, 1), pitch, dtype=torch.float32, device=dev) if mode["hs"] else None
    if args.own_model and world == 1:
        Wn = W[:, :d].cpu().numpy()
        Cn = Cm[:, :d].cpu().numpy() if Cm is not None else None
        Sn = S[:, :d].cpu().numpy() if S is not None else None
        tr.upload_model(Wn, Cn, Sn)
        del Wn, Cn, Sn
        W = Cm = S = None
    else:
        tr.bind_model(W.data_ptr(), Cm.data_ptr() if Cm is not None else None,
                      S.data_ptr() if S is not None else None, pitch)
    # alpha follows the global schedule: train_words = (global raw tokens) / world
    # with each round's counter at (global words) / world (replicas.train_rounds)
    tr.upload_corpus(ids_h, soff_h, n_tok)
    tr.set_rng(N.W2V_RNG_PHILOX, (args.seed << 32) | (rank + 1))
    if mode.get("shared"):
        tr.set_update(N.W2V_UPDATE_SHARED_NEGATIVES)
    tr.set_schedule(N.W2V_SCHED_PARALLEL)
    tr.set_hot_rows(args.hot_rows)
    tr.set_hot_auto(*args.hot_auto)
    tr.set_private_rows(args.private_rows)
    if args.private_rate is not None:
        tr.set_private_rate(args.private_rate)
    tr.set_private_sync(args.flush_centers, args.private_average)
    tr.set_max_waves(args.max_waves)
    tr.set_context_private(args.context_rows, args.context_flush)
    tr.set_progress(0)
    torch.cuda.synchronize()
    log(f"[bench] resident in HBM ({time.time() - t0:.1f}s)")

    mats = [m for m in (W, Cm, S) if m is not None]
    if not mats:
        assert world == 1
    # N = 1: no-op; one rank per GPU: the native RCCL group (the group id broadcast from rank 0);
    # W2V_BENCH_SHARE_GPU (ranks share cuda:0, RCCL needs one rank per GPU): one-rank native groups + gloo mean
    rmode = args.replica_mode if args.replica_mode != "auto" else auto_replica_mode(world)
    averager, rmode_used = make_averager(tr, mats, world, rank, rmode, not args.no_overlap, share)
    if args.sync_every > 0 or world == 1:
        rounds = n_rounds(n_sent * world, world, args.sync_every)
    else:  # every rank's shard has ~ the same words, but not exactly: agree on the largest round count
        rounds = max(1, -(-int(ids_h.size) // max(1, args.sync_words or config3_sync_words(world, rmode))))
        rounds = agree_rounds(rounds, world)  # a rank that ran a different number of exchanges would hang the group
    order_dev = torch.arange(n_sent, dtype=torch.int64, device=dev)  # this rank's shard, in order
    round_words = global_round_words(local_round_words(soff_h, range(n_sent), rounds), world)
    progress = 0

    def step(epoch, evs=None):
        nonlocal progress
        progress = train_rounds(tr, averager, order_dev, epoch, rounds, progress, round_words, world, evs)

    for w in range(args.warmup):
        step(w)
    averager.finish()
    torch.cuda.synchronize()
    st0 = tr.read_stats()
    events = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k, events)
    averager.finish()  # the last (overlapped) average is folded in inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    st1 = tr.read_stats()
    kern_ms = [a.elapsed_time(b) for a, b in events]
    delta = {k: st1[k] - st0[k] for k in st1}
    # every step trains this rank's whole shard once (the device word counter is
    # moved to the global count at each averaging round, so count from the shard)
    assert delta["sentences"] == n_sent * args.steps, delta
    words_local = int(ids_h.size) * args.steps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        wsum = torch.tensor([words_local], dtype=torch.int64)
        dist.all_reduce(wsum)
        words_total = int(wsum.item())
    else:
        words_total = words_local
    for m in mats:
        assert torch.isfinite(m).all().item(), "non-finite weights"

    value = words_total / elapsed
    # algorithmic HBM bytes per launch: fp32 rows read+written
    if mode["cbow"] or mode.get("shared"):  # unique context rows (CBOW inputs / minibatch W rows)
        row_moves = 2 * delta["contexts"] + 2 * delta["targets"]
    else:
        row_moves = 2 * delta["centers"] + 2 * delta["targets"]
    n_launch = max(1, len(events))
    bytes_per_launch = (4 * d * row_moves + 4 * delta["draws"]) / n_launch
    avg_kernel_s = float(np.mean(kern_ms)) / 1e3
    achieved = bytes_per_launch / avg_kernel_s / 1e9
    traffic, traffic_src, traffic_ms = pmc_traffic(args)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                "kernel": "train_epoch_kernel", "avg_launch_ms": round(avg_kernel_s * 1e3, 3),
                "algorithmic_bytes_per_launch": int(bytes_per_launch),
                # the rocprofv3 average of the profile `traffic` comes from (another lease's box: MI355X
                # boxes differ by up to ~10 %), next to this run's own HIP-event average
                "profile_box_ms": traffic_ms}
    if mode.get("shared"):
        # MFMA work issued per kept center: three 16 x 16 x pitch f32 GEMMs (L, dW, dC)
        flops = 3 * 2 * 16 * 16 * pitch * delta["centers"] / n_launch
        tf = flops / avg_kernel_s / 1e12
        roofline["kernel"] = "train_shared_neg_kernel"
        # useful work: the unpadded M x T x d products of each center's three GEMMs; the
        # kernel counts sum M (contexts) and sum T (targets), and T is ~neg + 1 for
        # every center, so sum M T ~= sum M x mean T
        useful = 3 * 2 * d * delta["contexts"] * (delta["targets"] / max(1, delta["centers"])) / n_launch
        tu = useful / avg_kernel_s / 1e12
        roofline["mfma"] = {"issued_tflops": round(tf, 2), "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                            "frac": round(tf / MFMA_F32_PEAK_TFLOPS, 4), "dtype": "f32 (v_mfma_f32_16x16x4_f32)",
                            "useful_tflops": round(tu, 2), "useful_frac": round(tu / MFMA_F32_PEAK_TFLOPS, 4),
                            "useful_note": "6 d sum(M T) over unpadded tiles (M unique contexts, T center + "
                                           "negatives), sum(M T) ~= sum M x mean T"}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args, counts_v, ids_h, soff_h, neg, mode)
        cpu["gpu_over_cpu"] = round(value / max(cpu["value"], 1e-9), 1)
        cpu["gpu_over_cpu_per_thread_rng"] = round(value / max(cpu["per_thread_rng_value"], 1e-9), 1)

    if rank == 0:
        out = {
            "metric": (f"trained words/sec, dim={d} " + ("CBOW" if mode["cbow"] else "SG") + ("-HS" if mode["hs"] else ("-NS" if mode["cbow"] else "NS"))
                       + (" shared-negatives minibatch" if mode.get("shared") else "")
                       + " (per-GPU replica, RCCL all-reduce of the replicas' updates for N>1)"),
            "value": round(value, 1),
            "unit": "words/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic",
            "config": {
                "workload": f"{args.mode} neg{neg} d{d} w{args.window} subsample {args.subsample} min_count "
                            f"{args.min_count}; synthetic Zipf(s={args.zipf_s:g}"
                            + (f", q={args.zipf_q:g}" if args.zipf_q else "") + f") over {args.vocab} ranks "
                            + {"c1": "standing in for text8 (configs[0]'s workload)",
                               "c2": "standing in for text8 (configs[1])",
                               "c4": "per GPU of configs[3]",
                               "c5": "(configs[4], shared-negatives minibatch)"}.get(
                                   args.config, "(configs[4], shared-negatives minibatch)" if mode.get("shared") else
                                   "standing in for 1B-Word (configs[2])") + f"; {args.sent_len}-token sentences",
                "baseline_config": args.config or ("c5" if mode.get("shared") else "c3"),
                "traffic_key": traffic_key(args),
                "tokens_per_gpu_per_step": n_tok,
                "in_vocab_tokens_per_gpu_per_step": int(ids_h.size),
                "vocab_size": V,
                "global_batch": n_tok * world,
                "parallelism": (f"dp{world}: full replica per GPU, corpus shard per GPU, RCCL all-reduce "
                                f"of the updates, {rmode_used}, "
                                f"{'overlapped' if not args.no_overlap else 'blocking'}, x{rounds} per step "
                                f"(every {int(ids_h.size) // rounds} words of a shard)"
                                if world > 1 else "dp1"),
                "hot_rows": args.hot_rows,
                "private_rows": args.private_rows,
                "flush_centers": args.flush_centers,
                "private_average": args.private_average,
                "max_waves": args.max_waves,
                "context_rows": args.context_rows,
                "context_flush": args.context_flush,
                "kept_centers_per_step": int(delta["centers"] / args.steps),
                "env_knobs": tr.knobs(),
                "hot_auto": args.hot_auto,
                "policy_used": tr.policy(),
                "targets_per_step": int(delta["targets"] / args.steps),
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if world > 1:
        log(f"[bench] replica exchange: {rmode_used}, group {averager.info()}")
        averager.close()
    tr.close()


def pmc_traffic(args):
    """HBM bytes per launch of this workload's dominant kernel from the committed
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh + tools/pmc_summary.py;
    2 x FETCH + WRITE, MI355X_MICROARCH.md's gfx950 correction), with the profile
    it came from: (bytes, source) or (None, None)."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None, None, None
    try:
        rec = json.loads(f.read_text()).get(traffic_key(args))
    except (OSError, ValueError):
        return None, None, None
    if isinstance(rec, dict):
        return rec.get("traffic"), rec.get("source"), rec.get("avg_duration_ms_rocprof")
    return None, None, None


def traffic_key(args) -> str:
    """profiles/pmc_traffic.json key of this workload (tools/pmc_summary.py)."""
    k = f"{args.mode}_d{args.dim}_n{args.tokens}"
    if args.zipf_s != 1.0 or args.zipf_q != 0.0 or args.vocab != 1_000_000:
        k += f"_v{args.vocab}_s{args.zipf_s:g}_q{args.zipf_q:g}"
    return k


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_topology() -> dict:
    """What the CPU legs may use: the process's affinity set (the threads the
    legs run), the machine's logical CPUs, sockets / physical cores of the
    affinity set (sysfs), the cgroup CPU quota and where OMP_NUM_THREADS came
    from (it is not used to size the legs)."""
    aff = sorted(os.sched_getaffinity(0))
    pkgs, cores = set(), set()
    for c in aff:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            pkg = open(base + "physical_package_id").read().strip()
            core = open(base + "core_id").read().strip()
        except OSError:
            continue
        pkgs.add(pkg)
        cores.add((pkg, core))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"affinity_cpus": len(aff), "host_cpus": os.cpu_count(), "sockets": len(pkgs) or None,
            "physical_cores": len(cores) or None, "cgroup_cpu_quota": quota,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(args, counts_v, ids_h, soff_h, neg, mode):
    """The reference's OpenMP training loop (Word2Vec.cpp:375-394; restated in
    oracle/w2v_oracle.cpp with its per-call hash map / set, static schedule,
    shared alpha) compiled with the reference's own flags (main.cpp:2: -Ofast
    -march=native -funroll-loops -fopenmp, built on this host), timed on ALL
    the host cores this process may use (OMP_NUM_THREADS =
    nproc): the CPUs of its affinity set (len(os.sched_getaffinity(0))),
    capped by the cgroup's CPU quota where there is one — on the GPU box the
    affinity set is the whole 256-CPU machine but the quota is 16 CPUs, and
    256 threads on 16 CPUs' time measure the scheduler, not the reference
    (r03z: 0.08 M words/s, below one thread's 0.16 M); the environment's
    OMP_NUM_THREADS is reported, not used. Over a bounded prefix of the same
    shard (same params):
      value                     those threads, ONE shared mt19937 (the reference's data race)
      per_thread_rng_value      the same, one mt19937 per thread
      single_thread_value       one thread"""
    import oracle

    topo = host_topology()
    threads = topo["affinity_cpus"]
    if topo["cgroup_cpu_quota"]:
        threads = max(1, min(threads, int(-(-topo["cgroup_cpu_quota"] // 1))))
    path, flags = oracle.build_fast()
    native = oracle.BaselineLib(path)

    def make():
        o = oracle.Oracle(iter=1, window=args.window, min_count=args.min_count, table_size=args.table_size,
                          word_dim=args.dim, negative=neg, subsample_threshold=args.subsample, init_alpha=0.025,
                          min_alpha=2.5e-6, cbow_mean=True, train_method="hs" if mode["hs"] else "ns",
                          model="cbow" if mode["cbow"] else "sg", native=native)
        o.set_vocab_counts(counts_v)
        o.seed(args.seed)
        return o

    def timed(o, nthreads, budget, shared, seed):
        # calibrate on a prefix with a few sentences per thread (a static
        # schedule), then time a prefix sized to the budget
        n_cal = int(min(soff_h.size - 1, max(32, 4 * nthreads)))
        o.set_samples(ids_h[: soff_h[n_cal]], soff_h[: n_cal + 1], int(n_cal * args.sent_len))
        o.init_weights()
        t = time.perf_counter()
        w = o.train_omp(nthreads, n_cal, seed, shared)
        rate = w / max(time.perf_counter() - t, 1e-6)
        n = int(min(soff_h.size - 1, max(n_cal, rate * budget / max(1, args.sent_len))))
        o.set_samples(ids_h[: soff_h[n]], soff_h[: n + 1], int(n * args.sent_len))
        o.init_weights()
        t = time.perf_counter()
        w = o.train_omp(nthreads, n, seed + 1, shared)
        dt = time.perf_counter() - t
        return w, dt, n

    o = make()
    w, dt, n = timed(o, threads, args.cpu_seconds, True, 11)
    wp, dtp, n_p = timed(o, threads, args.cpu_seconds / 2, False, 21)
    w1, dt1, n1 = timed(o, 1, args.cpu_seconds / 3, True, 31)
    return {"value": round(w / dt, 1), "unit": "words/s", "cores": threads, "kind": "port",
            "per_thread_rng_value": round(wp / dtp, 1),
            "single_thread_value": round(w1 / dt1, 1),
            "cpu": cpu_model(), **topo, "flags": flags,
            "sample": f"{n} sentences ({w} in-vocab tokens) of the same shard, {dt:.1f}s: the reference's OpenMP "
                      f"loop restated (oracle/w2v_oracle.cpp orc_train_omp_shared), built with {flags}, "
                      f"{threads} threads (the process's usable CPUs: its affinity set, {topo['affinity_cpus']} "
                      f"CPUs, capped by the cgroup quota, {topo['cgroup_cpu_quota']}) sharing one mt19937 as the "
                      f"reference does; per_thread_rng_value: {n_p} sentences, {dtp:.1f}s, one mt19937 per "
                      f"thread; single_thread_value: {n1} sentences, {dt1:.1f}s"
                      + ("; the reference's per-pair update: the shared-negatives minibatch has no reference CPU path"
                         if mode.get("shared") else "")}


if __name__ == "__main__":
    main()
