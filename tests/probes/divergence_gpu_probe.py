"""VERDICT r04 "next" 2, GPU side: the r04a input (window 150, negative 80,
alpha 0.025, d 64, V 1,807; profiles/r04a_gpu_tests.log:714-747) through the
parallel schedule at several wave caps and update policies. The sequential
oracle stays finite on it (tests/probes/divergence_probe.py). One JSON line
per run: non-finite sigma arguments, max |W|, max |C|.

usage: divergence_gpu_probe.py [variant ...]   variant = name[:setter=value,...]
(setters of tests/probes/policy_probe.py: waves, hot, priv, avg, flush, tau, W2V_* knobs)"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from tests.corpus import zipf_sentences  # noqa: E402
from tests.harness import device_from_oracle, oracle_run  # noqa: E402
from tests.probes.policy_probe import apply, knobs  # noqa: E402
from word2vec_amd import _native as N  # noqa: E402
from word2vec_amd.device import Config  # noqa: E402


def run(mode, spec, alpha=0.025, vmax=2000):
    sents = zipf_sentences(200, 400, vmax, seed=51, ragged=True)
    o = oracle_run(sents, mode, dim=64, window=150, iters=1, table_size=100_000, train=False)
    o.build_sample()
    cfg = Config(word_dim=64, window=150, negative=80, hs=False, cbow=mode == "cbow_ns", cbow_mean=True, iter=1,
                 init_alpha=alpha, min_alpha=2.5e-6, table_size=100_000)
    with knobs(spec):
        d = device_from_oracle(o, cfg, initial=False)
    d.set_rng(N.W2V_RNG_PHILOX, 99)
    d.set_schedule(N.W2V_SCHED_PARALLEL)
    d.set_progress(0)
    apply(d, spec)
    t0 = time.time()
    err = ""
    try:
        st = d.train_epoch(0, np.random.default_rng(3).permutation(o.samples()[1].size - 1))
    except N.DevError as e:
        err = str(e)
        st = d.read_stats()
    pol = d.policy()
    W, Cm, _ = d.download_model()
    d.close()
    fw, fc = np.isfinite(W), np.isfinite(Cm)
    return {"mode": mode, "spec": spec, "alpha": alpha, "V": int(W.shape[0]), "words": st.get("words"),
            "nonfinite_sigma": st.get("nonfinite"), "nonfinite_values": int((~fw).sum() + (~fc).sum()),
            "max_abs_W": float(np.abs(W[fw]).max()) if fw.any() else None,
            "max_abs_C": float(np.abs(Cm[fc]).max()) if fc.any() else None,
            "policy": pol, "error": err[:120], "secs": round(time.time() - t0, 2)}


if __name__ == "__main__":
    variants = sys.argv[1:] or ["full", "w512:waves=512", "w128:waves=128", "w64:waves=64", "w32:waves=32",
                                "w16:waves=16", "w8:waves=8"]
    for mode in ("cbow_ns", "sg_ns"):
        for v in variants:
            nm, _, spec = v.partition(":")
            r = run(mode, spec)
            r["variant"] = nm
            print(json.dumps(r), flush=True)
