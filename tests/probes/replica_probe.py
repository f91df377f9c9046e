"""GPU probe: where does data-parallel replica training lose quality? Runs the
planted corpus (tests/paired.py setup: oracle vocab, seeded init, Philox key)
through variants of slicing and exchanging, and prints analogy / similarity.
usage (GPU box): python tests/probes/replica_probe.py [mode] [seed] [rounds] [corpus] [short]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

from tests import paired  # noqa: E402
from tests.harness import device_from_oracle  # noqa: E402
from word2vec_amd import _native as N  # noqa: E402
from word2vec_amd.evaluate import analogy_accuracy, similarity_score  # noqa: E402
from word2vec_amd.replicas import NativeAverager  # noqa: E402


def main(mode="sg_ns", seed=1, rounds=8, corpus="planted", short="0"):
    seed, rounds = int(seed), int(rounds)
    sents, qs, pairs = paired.corpus(corpus)
    o, orders, key, p = paired.setup(corpus, mode, seed, sents)
    off = o.samples()[1]
    n = off.size - 1
    words, _ = o.vocab()
    T = int(off[-1])  # in-vocab tokens (train_words proxy)

    def handle():
        d = device_from_oracle(o, paired.gpu_cfg(o, mode, p), initial=False)
        d.set_rng(N.W2V_RNG_PHILOX, key)
        d.set_schedule(N.W2V_SCHED_PARALLEL)
        return d

    def score(d, tag, t0):
        W, Cm, _ = d.download_model()
        E = Cm if paired.eval_matrix(mode) == 1 else W
        print(f"{tag:48s} analogy {analogy_accuracy(words, E, qs)['accuracy']:6.2f} "
              f"similarity {similarity_score(words, E, pairs)['spearman']:6.2f}  {time.time() - t0:.1f}s", flush=True)

    lens = np.diff(off)

    def run(R, slices, exchange=None, gmode="row_average", overlap=False, shards=True, pol=None):
        t0 = time.time()
        ds = [handle() for _ in range(R)]
        for d in ds:
            pol = pol or {}
            if "hot_rows" in pol:
                d.set_hot_rows(pol["hot_rows"])
            if "private_rows" in pol:
                d.set_private_rows(pol["private_rows"])
            if "private_average" in pol or "flush_centers" in pol:
                d.set_private_sync(pol.get("flush_centers", 0), pol.get("private_average", 8.0))
            if "context_rows" in pol:
                d.set_context_private(pol["context_rows"], 0)
            if "max_waves" in pol:
                d.set_max_waves(pol["max_waves"])
        for d in ds:
            d.set_train_words(max(1, o.train_words // R))
        g = NativeAverager(ds, overlap=overlap, mode=gmode) if exchange else None
        glob = 0
        for e in range(p["iters"]):
            order = orders[e * n:(e + 1) * n]
            parts = [order[n * i // R:n * (i + 1) // R] for i in range(R)] if shards else [order] * R
            for d, part in zip(ds, parts):
                d.set_order(part)
            for r in range(slices):
                w = 0
                for d, part in zip(ds, parts):
                    m = part.size
                    lo, hi = m * r // slices, m * (r + 1) // slices
                    d.set_progress_async(glob // R)
                    if hi > lo:
                        d.train_slice_async(e, lo, hi - lo)
                    w += int(lens[part[lo:hi]].sum())
                if g is not None and exchange == "round":
                    g.average()
                glob += w
            if g is not None and exchange == "epoch":
                g.average()
            if g is not None:
                g.finish()
            for d in ds:
                d.synchronize()
        tag = f"R={R} slices={slices} exchange={exchange} mode={gmode} overlap={overlap} {pol or ''}"
        score(ds[0], tag, t0)
        if g is not None:
            g.close()
        for d in ds:
            d.close()

    del T
    if short == "5":  # two replicas, summed every 1/64 epoch, against one model
        run(1, 1)
        run(1, rounds)
        run(2, rounds, "round", "sum")
        run(2, rounds, "round", "sum", overlap=True)
        run(1, 1, pol={"max_waves": 1})
        run(2, rounds, "round", "sum", pol={"max_waves": 1})
        return
    if short == "4":  # one wavefront per replica: the exchange logic without the parallel policy
        one = {"max_waves": 1}
        run(1, 1, pol=one)
        run(2, 4, "round", "sum", pol=one)
        run(2, 4, "round", "row_average", pol=one)
        run(2, 1, "round", "sum", pol=one)
        run(2, 4, "round", "sum", overlap=True, pol=one)
        return
    if short == "3":
        run(1, 1)
        run(1, 4)
        run(1, 16)
        run(2, 1, "round")
        run(2, 4, "round")
        run(2, 4, "round", overlap=True)
        run(2, 4, "round", "sum")
        return
    if short == "2":
        run(1, 1)
        run(1, 1, pol={"max_waves": 2512})
        run(1, 4)
        run(1, 4, pol={"max_waves": 2048})
        run(1, 4, pol={"max_waves": 1024})
        run(1, 4, pol={"private_average": 0.0})
        run(1, 4, pol={"private_rows": 0, "context_rows": 0})
        run(1, 16)
        run(1, 16, pol={"max_waves": 512})
        return
    if short == "1":
        run(1, 1)
        run(1, rounds)
        for gm in ("row_average", "sum", "average"):
            run(2, 1, "round", gm)
            run(2, rounds, "round", gm)
            run(2, rounds, "round", gm, overlap=True)
        return
    run(1, 1)
    run(1, rounds)
    run(1, rounds, pol={"private_average": 0.0})
    run(1, rounds, pol={"private_average": 1.0})
    run(1, rounds, pol={"private_rows": 0, "context_rows": 0})
    run(1, rounds, pol={"hot_rows": -1})
    run(1, rounds, pol={"hot_rows": -1, "private_rows": 0, "context_rows": 0})
    run(2, rounds, None)
    for gm in ("row_average", "sum", "average"):
        run(2, rounds, "round", gm)
        run(2, rounds, "round", gm, overlap=True)
    run(2, 4 * rounds, "round")
    run(2, 4 * rounds, "round", overlap=True)
    run(2, 1, "round")
    run(2, 1, "round", overlap=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
