"""Update-policy variants of the GPU's parallel schedule on the paired quality
gates at the benchmarked scale (tests/test_gpu_quality.py): per golden seed,
the GPU trains from the golden run's own start under each variant and the
delta to the oracle's score is printed (one JSON line per variant).

usage: policy_probe.py <c3|c2|c1|c5> <variant> [<variant> ...]
  variant = name[:setter=value[,setter=value...]], setters: tau (hot-row
  threshold, rows), tau_nodes, hot (hot_rows), priv (private_rows), avg
  (private_average), flush (flush_centers), ctx (context_rows), ctxflush,
  waves (max_waves); e.g. default tau1:tau=1 priv32:priv=32; a key W2V_* is an
  experiment knob set in the environment while the variant's handles are created
Test infrastructure (reads the committed goldens; runs no oracle)."""
import contextlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def _kv(spec):
    return dict(x.split("=") for x in spec.split(",") if x) if spec else {}


@contextlib.contextmanager
def knobs(spec):
    """W2V_* keys of a variant in the environment (read at w2v_dev_create)."""
    env = {k: v for k, v in _kv(spec).items() if k.startswith("W2V_")}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def apply(t, spec):
    kv = _kv(spec)
    if "tau" in kv or "tau_nodes" in kv:
        t.set_hot_auto(float(kv.get("tau", 0)), float(kv.get("tau_nodes", 1)))
    if "hot" in kv:
        t.set_hot_rows(int(kv["hot"]))
    if "priv" in kv:
        t.set_private_rows(int(kv["priv"]))
    if "avg" in kv or "flush" in kv:
        t.set_private_sync(int(kv.get("flush", 0)), float(kv.get("avg", 8)))
    if "ctx" in kv or "ctxflush" in kv:
        t.set_context_private(int(kv.get("ctx", -1)), int(kv.get("ctxflush", 0)))
    if "waves" in kv:
        t.set_max_waves(int(kv["waves"]))


def headline(name, variants):
    from tests.golden import gen_headline_planted_golden as G
    from tests.planted_ids import gpu_trainer, scores
    from word2vec_amd._native import DevError

    gold = json.loads(G.golden_path(name).read_text())
    w = G.WORKLOADS[name]
    ids, soff, counts, words, raw, qs, prs = G.corpus(name)
    for v in variants:
        nm, _, spec = v.partition(":")
        got, ref, pol, t0 = [], [], None, time.time()
        for r in gold["scores"]:
            W0, C0, S0, key = G.init(name, r["seed"], counts.size)
            with knobs(spec):
                t = gpu_trainer(counts, ids, soff, raw, w["mode"], w["dim"], w["negative"], w["alpha"], W0, C0, S0,
                                key)
            apply(t, spec)
            try:
                st = t.train_epoch(0, G.order_of(r["seed"], soff.size - 1))
            except DevError as e:  # a diverged variant is a result, not the probe's end
                print(f"  {nm} seed {r['seed']}: {e}", file=sys.stderr, flush=True)
                st = {"nonfinite": -1}
            pol = t.policy()
            W, Cm, _ = t.download_model()
            t.close()
            E = Cm if G.eval_matrix(name) == 1 else W
            got.append(scores(words, E, qs, prs, torch.device("cuda", 0)) if st["nonfinite"] == 0 else (np.nan, np.nan))
            ref.append([r["analogy"], r["similarity"]])
            print(f"  {nm} seed {r['seed']}: {np.round(np.array(got[-1]) - ref[-1], 2).tolist()} "
                  f"({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
        report(name, nm, spec, got, ref, pol, t0)


def c5(variants):
    from oracle import Oracle

    from tests.golden.gen_quality_zipf_golden import ZCORPUS
    from tests.harness import device_from_oracle
    from tests.quality import planted_zipf_corpus
    from word2vec_amd import _native as N
    from word2vec_amd.device import Config
    from word2vec_amd.evaluate import analogy_accuracy, similarity_score

    gold = json.loads((ROOT / "tests" / "golden" / "quality_zipf_sg_sn_c5_oracle.json").read_text())
    t_ = gold["train"]
    sents, qs, pairs = planted_zipf_corpus(**ZCORPUS)
    starts = []
    for r in gold["scores"]:
        o = Oracle(iter=1, window=t_["window"], min_count=t_["min_count"], table_size=t_["table_size"],
                   word_dim=t_["dim"], negative=t_["negative"], subsample_threshold=t_["subsample"],
                   init_alpha=gold["alpha"], min_alpha=2.5e-6, cbow_mean=True, train_method="ns", model="sg")
        o.load_sentences(sents)
        o.seed(r["seed"])
        o.build_vocab()
        o.init_weights()
        o.build_sample()
        starts.append((r, o))
    for v in variants:
        nm, _, spec = v.partition(":")
        got, ref, pol, t0 = [], [], None, time.time()
        for r, o in starts:
            cfg = Config(word_dim=t_["dim"], window=t_["window"], negative=t_["negative"], hs=False, cbow=False,
                         cbow_mean=True, iter=1, init_alpha=gold["alpha"], min_alpha=2.5e-6,
                         table_size=t_["table_size"])
            with knobs(spec):
                d = device_from_oracle(o, cfg, initial=False)
            d.set_update(N.W2V_UPDATE_SHARED_NEGATIVES)
            d.set_rng(N.W2V_RNG_PHILOX, 0x5EED0000 + r["seed"])
            d.set_schedule(N.W2V_SCHED_PARALLEL)
            d.set_progress(0)
            apply(d, spec)
            d.train_epoch(0, np.random.default_rng(r["seed"]).permutation(len(sents)).astype(np.int64))
            pol = d.policy()
            W, _, _ = d.download_model()
            d.close()
            words, _ = o.vocab()
            got.append([analogy_accuracy(words, W, qs)["accuracy"], similarity_score(words, W, pairs)["spearman"]])
            ref.append([r["analogy"], r["similarity"]])
        report("c5", nm, spec, got, ref, pol, t0)


def report(name, nm, spec, got, ref, pol, t0):
    got, ref = np.array(got, float), np.array(ref, float)
    d = got - ref
    print(json.dumps({"workload": name, "variant": nm, "spec": spec, "gpu": got.mean(0).round(2).tolist(),
                      "oracle": ref.mean(0).round(2).tolist(), "delta": d.mean(0).round(2).tolist(),
                      "per_seed": d.round(2).tolist(), "policy": pol, "secs": round(time.time() - t0, 1)}),
          flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "c5":
        c5(sys.argv[2:])
    else:
        headline(sys.argv[1], sys.argv[2:])
