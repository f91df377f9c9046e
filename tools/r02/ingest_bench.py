"""Corpus ingestion throughput: the host readers (csrc/host/corpus.cpp, host
threads) against the GPU ingest (include/w2v_ingest.h) on one synthetic
text8-like file (Zipf words, 64 MiB block repeated to --mib). Prints one JSON
line per path: seconds and tokens/s for the vocab count (build_vocab_file) and
for the id mapping (file_samples), and checks both give the same samples.

    python tools/r02/ingest_bench.py --mib 1024 --threads 16
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def make_file(path: str, mib: int, seed: int = 0) -> None:
    rng = np.random.default_rng(seed)
    vmax = 250_000
    p = 1.0 / np.arange(1, vmax + 1) ** 1.0
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    words = np.array([f"w{r}" for r in range(vmax)], dtype=object)
    block = []
    size = 0
    while size < 64 << 20:
        ids = np.searchsorted(cdf, rng.random(1 << 20), side="right").clip(0, vmax - 1)
        s = " ".join(words[ids]) + " "
        block.append(s)
        size += len(s)
    data = "".join(block).encode()
    with open(path, "wb") as f:
        left = mib << 20
        while left > 0:
            n = min(left, len(data))
            # cut after a space so words stay whole
            while n < len(data) and data[n - 1:n] != b" ":
                n += 1
            f.write(data[:n])
            left -= n


def run(gpu: bool, path: str, threads: int, chunk: int):
    from word2vec_amd.model import Word2Vec

    m = Word2Vec(iter=1, window=5, min_count=5, table_size=1000, word_dim=16, negative=5, train_method="ns",
                 model="sg", verbose=False, gpu_ingest=gpu, ingest_chunk_bytes=chunk)
    t0 = time.perf_counter()
    m.build_vocab_file(path, "text8", threads)
    t1 = time.perf_counter()
    ids, off, tw = m.file_samples(path, "text8", threads)
    t2 = time.perf_counter()
    return dict(count_s=t1 - t0, map_s=t2 - t1, tokens=int(tw), vocab=int(m.V)), (ids, off, tw)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="ingest_")
    path = os.path.join(d, "corpus.txt")
    t = time.perf_counter()
    make_file(path, a.mib)
    print(f"# wrote {os.path.getsize(path) >> 20} MiB in {time.perf_counter() - t:.1f}s", flush=True)
    lines = []
    res = {}
    for gpu in (True, False, True):   # first GPU run pays the context / code-object load
        r, s = run(gpu, path, a.threads, a.chunk)
        r.update(path="gpu" if gpu else f"host_{a.threads}threads", bytes=os.path.getsize(path),
                 count_tok_per_s=r["tokens"] / r["count_s"], map_tok_per_s=r["tokens"] / r["map_s"],
                 total_gb_per_s=2 * os.path.getsize(path) / (r["count_s"] + r["map_s"]) / 1e9)
        res[gpu] = s
        print(json.dumps(r), flush=True)
        lines.append(r)
    same = (res[True][2] == res[False][2] and np.array_equal(res[True][1], res[False][1])
            and np.array_equal(res[True][0], res[False][0]))
    print(json.dumps({"identical_samples": bool(same)}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"runs": lines, "identical_samples": bool(same)}, f, indent=1)
    os.remove(path)
    os.rmdir(d)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
