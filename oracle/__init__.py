"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (w2v_oracle.cpp).

Importable by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the checker. The product (word2vec_amd/) never imports this package.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"


def build(force: bool = False) -> Path:
    src = HERE / "w2v_oracle.cpp"
    if force or not LIB.exists() or LIB.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["make", "-C", str(HERE), "-s"], check=True)
    return LIB


_P, _I32, _I64, _U32, _U64, _F = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_float
_SIG = {
    "orc_new": (_P, [_I32, _I32, _I32, _I32, _I32, _I32, _F, _F, _F, _I32, _I32, _I32]),
    "orc_free": (None, [_P]),
    "orc_seed": (None, [_P, _U32]),
    "orc_load_text": (None, [_P, C.c_char_p, _I64]),
    "orc_build_vocab": (None, [_P]),
    "orc_vocab_size": (_I64, [_P]),
    "orc_vocab_word": (C.c_char_p, [_P, _I64]),
    "orc_vocab_counts": (None, [_P, _P]),
    "orc_sample_probs": (None, [_P, _P]),
    "orc_huffman_total": (_I64, [_P]),
    "orc_huffman": (None, [_P, _P, _P, _P]),
    "orc_table_size": (_I64, [_P]),
    "orc_table": (None, [_P, _P]),
    "orc_table_bounds": (None, [_P, _P]),
    "orc_init_weights": (None, [_P]),
    "orc_matrix_rows": (_I64, [_P, _I32]),
    "orc_get_matrix": (None, [_P, _I32, _I32, _P]),
    "orc_set_matrix": (None, [_P, _I32, _P, _I64]),
    "orc_build_sample": (None, [_P]),
    "orc_n_tokens": (_I64, [_P]),
    "orc_n_sentences": (_I64, [_P]),
    "orc_samples": (None, [_P, _P, _P]),
    "orc_train_words": (_I64, [_P]),
    "orc_current_words": (_I64, [_P]),
    "orc_last_alpha": (_F, [_P]),
    "orc_train": (None, [_P, _I32]),
    "orc_stream_size": (_I64, [_P]),
    "orc_stream": (None, [_P, _P, _P, _P]),
    "orc_train_replay": (None, [_P, _I32, _P, _P, _P, _I64]),
    "orc_train_philox": (None, [_P, _I32, _I32, _P, _U64, _I64]),
    "orc_train_philox_omp": (None, [_P, _I32, _I32, _I32, _P, _U64, _I64]),
    "orc_philox": (None, [_P, _U64, _P]),
    "orc_set_shared_negatives": (None, [_P, _I32]),
    "orc_train_omp": (_I64, [_P, _I32, _I64, _U32]),
    "orc_train_omp_shared": (_I64, [_P, _I32, _I64, _U32, _I32]),
    "orc_set_vocab_counts": (None, [_P, _P, _I64]),
    "orc_set_samples": (None, [_P, _P, _P, _I64, _I64]),
    "orc_train_sentence": (None, [_P, _P, _I64, _F, _I32]),
    "orc_negative_sampling": (None, [_P, _I64, _P, _P, _I32, _F]),
    "orc_hierarchical_softmax": (None, [_P, _I64, _P, _P, _F]),
}

_lib = None


def _bind(path) -> C.CDLL:
    L = C.CDLL(str(path))
    for k, (r, a) in _SIG.items():
        f = getattr(L, k)
        f.restype, f.argtypes = r, a
    return L


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        build()
        _lib = _bind(LIB)
    return _lib


# The CPU-baseline build: the same restatement compiled with the reference's
# own flags (main.cpp:2: -Ofast -march=native -funroll-loops -fopenmp). Used
# ONLY by bench.py's cpu_baseline leg for timing — -Ofast changes the float
# bits of the host products, so parity never uses it.
REF_FLAGS = ["-std=c++11", "-Ofast", "-march=native", "-funroll-loops", "-fopenmp"]
PORTABLE_FLAGS = ["-std=c++11", "-Ofast", "-march=x86-64-v3", "-funroll-loops", "-fopenmp"]
FAST_LIB = HERE / "liboracle_fast.so"  # prebuilt with PORTABLE_FLAGS (Makefile), for boxes without g++


def build_fast(out_dir=None):
    """Compile the baseline build with REF_FLAGS for THIS host's CPU (-march=native
    must be compiled where it runs). Returns (path, flags); falls back to the
    prebuilt portable build when no compiler is available."""
    import hashlib
    import os
    import shutil
    import tempfile

    src = HERE / "w2v_oracle.cpp"
    cxx = shutil.which(os.environ.get("CXX", "g++")) or shutil.which("g++")
    if cxx:
        tag = hashlib.sha1(src.read_bytes() + " ".join(REF_FLAGS).encode()).hexdigest()[:12]
        out = Path(out_dir or tempfile.gettempdir()) / f"w2v_cpu_baseline_{tag}.so"
        if not out.exists():
            tmp = out.with_suffix(f".{os.getpid()}.so")
            r = subprocess.run([cxx, *REF_FLAGS, "-fPIC", "-shared", "-o", str(tmp), str(src)],
                               capture_output=True, text=True)
            if r.returncode == 0:
                os.replace(tmp, out)
        if out.exists():
            return out, " ".join(REF_FLAGS)
    return FAST_LIB, " ".join(PORTABLE_FLAGS) + " (prebuilt)"


class BaselineLib:
    """Context for Oracle(..., lib=...): the reference-flags build."""

    def __init__(self, path):
        self.L = _bind(path)


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Oracle:
    """Sequential restatement of lache/word2vec's Word2Vec (see w2v_oracle.cpp)."""

    def __init__(self, iter=1, window=5, min_count=5, table_size=100_000_000, word_dim=200, negative=0,
                 subsample_threshold=1e-3, init_alpha=0.025, min_alpha=1e-6, cbow_mean=False,
                 train_method="hs", model="cbow", native=None):
        self.L = native.L if native is not None else lib()
        self.dim = word_dim
        self.hs = train_method == "hs"
        self.cbow = model == "cbow"
        self.negative = negative
        self.h = self.L.orc_new(iter, window, min_count, table_size, word_dim, negative, subsample_threshold,
                                init_alpha, min_alpha, int(cbow_mean), int(self.hs), int(self.cbow))

    def __del__(self):
        try:
            self.L.orc_free(self.h)
        except Exception:
            pass

    def seed(self, s: int):
        self.L.orc_seed(self.h, s)

    def load_sentences(self, sentences):
        text = "\n".join(" ".join(s) for s in sentences).encode()
        self.L.orc_load_text(self.h, text, len(text))

    def build_vocab(self):
        self.L.orc_build_vocab(self.h)

    @property
    def V(self) -> int:
        return self.L.orc_vocab_size(self.h)

    def vocab(self):
        V = self.V
        words = [self.L.orc_vocab_word(self.h, i).decode() for i in range(V)]
        counts = np.empty(V, np.int64)
        self.L.orc_vocab_counts(self.h, _p(counts))
        return words, counts

    def sample_probs(self):
        out = np.empty(self.V, np.float32)
        self.L.orc_sample_probs(self.h, _p(out))
        return out

    def huffman(self):
        n = self.L.orc_huffman_total(self.h)
        codes = np.empty(max(n, 1), np.uint8)
        points = np.empty(max(n, 1), np.int32)
        off = np.empty(self.V + 1, np.int64)
        self.L.orc_huffman(self.h, _p(codes), _p(points), _p(off))
        return codes[:n], points[:n], off

    def table(self):
        out = np.empty(self.L.orc_table_size(self.h), np.uint32)
        self.L.orc_table(self.h, _p(out))
        return out

    def table_bounds(self):
        out = np.empty(self.V + 1, np.int64)
        self.L.orc_table_bounds(self.h, _p(out))
        return out

    def init_weights(self):
        self.L.orc_init_weights(self.h)

    def matrix(self, which: int, initial: bool = False):
        rows = self.L.orc_matrix_rows(self.h, which)
        if initial:
            rows = {0: self.V, 1: self.V if self._has_c() else 0, 2: self.V - 1 if self.hs else 0}[which]
        out = np.empty((rows, self.dim), np.float32)
        if rows:
            self.L.orc_get_matrix(self.h, which, int(initial), _p(out))
        return out

    def _has_c(self):
        return self.cbow or self.negative > 0 or not self.hs

    def set_matrix(self, which: int, m):
        m = np.ascontiguousarray(m, dtype=np.float32)
        self.L.orc_set_matrix(self.h, which, _p(m), m.shape[0])

    def build_sample(self):
        self.L.orc_build_sample(self.h)

    def samples(self):
        ids = np.empty(max(self.L.orc_n_tokens(self.h), 1), np.int32)
        off = np.empty(self.L.orc_n_sentences(self.h) + 1, np.int64)
        self.L.orc_samples(self.h, _p(ids), _p(off))
        return ids[: off[-1]], off

    @property
    def train_words(self):
        return self.L.orc_train_words(self.h)

    @property
    def current_words(self):
        return self.L.orc_current_words(self.h)

    def train(self, record: bool = True):
        self.L.orc_train(self.h, int(record))

    def stream(self, iters: int):
        n = self.L.orc_stream_size(self.h)
        ns = self.L.orc_n_sentences(self.h)
        s = np.empty(max(n, 1), np.uint32)
        off = np.empty(max(ns * iters, 1), np.int64)
        orders = np.empty(max(ns * iters, 1), np.int64)
        self.L.orc_stream(self.h, _p(s), _p(off), _p(orders))
        return s[:n], off[: ns * iters], orders[: ns * iters]

    def train_replay(self, epochs, orders, stream, offsets, cw0=0):
        orders = np.ascontiguousarray(orders, np.int64)
        stream = np.ascontiguousarray(stream, np.uint32)
        offsets = np.ascontiguousarray(offsets, np.int64)
        self.L.orc_train_replay(self.h, epochs, _p(orders), _p(stream), _p(offsets), cw0)

    def train_philox(self, epoch0, epochs, orders, key, cw0=0):
        orders = np.ascontiguousarray(orders, np.int64)
        self.L.orc_train_philox(self.h, epoch0, epochs, _p(orders), key, cw0)

    def train_philox_omp(self, threads, epoch0, epochs, orders, key, cw0=0):
        """The reference's OpenMP loop (Word2Vec.cpp:375-394, static schedule,
        Hogwild updates) on `threads` threads with the Philox draws: differs
        from train_philox only by the threads' concurrency."""
        orders = np.ascontiguousarray(orders, np.int64)
        self.L.orc_train_philox_omp(self.h, threads, epoch0, epochs, _p(orders), key, cw0)

    def set_shared_negatives(self, on: bool = True):
        """Shared-negatives minibatch skip-gram (configs[4]) for later training calls."""
        self.L.orc_set_shared_negatives(self.h, int(bool(on)))

    def train_omp(self, threads: int, n_sent_limit: int, seed: int = 1, shared_rng: bool = False) -> int:
        """The reference's OpenMP loop on `threads` threads over the first
        n_sent_limit sentences; shared_rng = one unsynchronised mt19937 for all
        threads, as the reference (a data race), else one per thread."""
        return self.L.orc_train_omp_shared(self.h, threads, n_sent_limit, seed, int(bool(shared_rng)))

    def set_vocab_counts(self, counts):
        c = np.ascontiguousarray(counts, np.int64)
        self.L.orc_set_vocab_counts(self.h, _p(c), c.size)

    def set_samples(self, ids, off, train_words):
        ids = np.ascontiguousarray(ids, np.int32)
        off = np.ascontiguousarray(off, np.int64)
        self.L.orc_set_samples(self.h, _p(ids), _p(off), off.size - 1, int(train_words))

    def train_sentence(self, ids, alpha: float, cbow: bool):
        ids = np.ascontiguousarray(ids, np.int32)
        self.L.orc_train_sentence(self.h, _p(ids), ids.size, alpha, int(cbow))

    def negative_sampling(self, word, x, grad, which, alpha):
        x = np.ascontiguousarray(x, np.float32)
        g = np.array(grad, np.float32)
        self.L.orc_negative_sampling(self.h, word, _p(x), _p(g), which, alpha)
        return g

    def hierarchical_softmax(self, word, x, grad, alpha):
        x = np.ascontiguousarray(x, np.float32)
        g = np.array(grad, np.float32)
        self.L.orc_hierarchical_softmax(self.h, word, _p(x), _p(g), alpha)
        return g


def philox(ctr, key: int):
    c = np.ascontiguousarray(ctr, np.uint32)
    out = np.empty(4, np.uint32)
    lib().orc_philox(_p(c), key, _p(out))
    return out
