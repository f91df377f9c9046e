"""VERDICT r04 "next" 2: does the SEQUENTIAL reference diverge on the input
that diverged on the GPU in r04a (profiles/r04a_gpu_tests.log:714-747)?

Input: zipf_sentences(200, 400, 2000, seed=51, ragged=True), window 150,
negative 80, alpha 0.025, d 64, subsample 1e-3, min_count 2, table 1e5.
The oracle (w2v_oracle.cpp) trains it one epoch in two draw modes:
  * REF: the reference's own mt19937 stream (Word2Vec.cpp:356-396);
  * PHILOX: the device's Philox draws (key 99, the r04a test's), sequential;
  * OMP<T>: the reference's own OpenMP Hogwild loop (Word2Vec.cpp:375-394,
    orc_train_omp_shared) on T threads sharing the model, one mt19937 per
    thread (the reference shares one, a data race);
and reports, per matrix, whether every value is finite and the largest |x|,
plus the largest |sigma argument| reached is inferred from the row norms
(max |W_i| * max |C_j|).

CPU only. Usage: python -m tests.probes.divergence_probe [--alpha A]"""
from __future__ import annotations

import argparse
import time

import numpy as np

from oracle import Oracle
from tests.corpus import zipf_sentences


def run(mode, alpha, draws, vmax=2000, window=150, negative=80, dim=64):
    sents = zipf_sentences(200, 400, vmax, seed=51, ragged=True)
    o = Oracle(iter=1, window=window, min_count=2, table_size=100_000, word_dim=dim, negative=negative,
               subsample_threshold=1e-3, init_alpha=alpha, min_alpha=2.5e-6, cbow_mean=True, train_method="ns",
               model="cbow" if mode == "cbow_ns" else "sg")
    o.load_sentences(sents)
    o.seed(1234)
    o.build_vocab()
    o.init_weights()
    o.build_sample()
    t0 = time.time()
    if draws == "ref":
        o.train(record=False)
    elif draws.startswith("omp"):
        o.init_weights()  # Word2Vec.cpp:358 (train() re-initialises)
        o.train_omp(int(draws[3:]), o.samples()[1].size - 1, seed=1234, shared_rng=False)
    else:
        order = np.random.default_rng(3).permutation(o.samples()[1].size - 1)
        o.train_philox(0, 1, order, 99, 0)
    dt = time.time() - t0
    W, Cm = o.matrix(0), o.matrix(1)
    fin = bool(np.isfinite(W).all() and np.isfinite(Cm).all())
    wn = float(np.nanmax(np.abs(W))) if np.isfinite(W).any() else float("nan")
    cn = float(np.nanmax(np.abs(Cm))) if np.isfinite(Cm).any() else float("nan")
    nonfin = int((~np.isfinite(W)).sum() + (~np.isfinite(Cm)).sum())
    rn = np.linalg.norm(np.nan_to_num(W), axis=1).max() * np.linalg.norm(np.nan_to_num(Cm), axis=1).max()
    print(f"{mode:8s} {draws:6s} alpha {alpha:g} V {o.V} words {o.current_words}: finite {fin} "
          f"non-finite values {nonfin} max|W| {wn:.3g} max|C| {cn:.3g} max|W_i||C_j| {rn:.3g} ({dt:.1f} s)",
          flush=True)
    return fin


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--alpha", type=float, nargs="*", default=[0.025, 0.0025])
    ap.add_argument("--vmax", type=int, default=2000)
    ap.add_argument("--draws", nargs="*", default=["ref", "philox"], help="ref, philox, omp<T>")
    ap.add_argument("--modes", nargs="*", default=["cbow_ns", "sg_ns"])
    a = ap.parse_args()
    for alpha in a.alpha:
        for mode in a.modes:
            for draws in a.draws:
                run(mode, alpha, draws, vmax=a.vmax)


if __name__ == "__main__":
    main()
