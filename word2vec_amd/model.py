"""Python view of the C++ Word2Vec class (include/Word2Vec.h via include/w2v_model.h).

Same constructor arguments and method names as the reference class
(/root/reference/Word2Vec.h:61-90); the C++ object does the work and its hot
path runs in the HIP kernels. Used by the tests and for scripting.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from .host import HOST_LIB

_lib = None
# Word2Vec::replica_mode values (include/w2v_dev.h W2V_GROUP_*)
REPLICA_MODES = {"auto": -1, "sum": 0, "average": 1, "row_average": 2, "adaptive": 3}


def _load():
    global _lib
    if _lib is None:
        if not HOST_LIB.exists():
            raise RuntimeError(f"word2vec_amd: {HOST_LIB} is missing; run make -C word2vec_amd/csrc")
        L = C.CDLL(str(HOST_LIB), mode=C.RTLD_GLOBAL)
        P, I32, I64, F, S = C.c_void_p, C.c_int32, C.c_int64, C.c_float, C.c_char_p
        sig = {
            "w2v_model_new": (P, [I32, I32, I32, I32, I32, I32, F, F, F, I32, I32, S, S]),
            "w2v_model_free": (None, [P]),
            "w2v_model_last_error": (S, [P]),
            "w2v_model_seed": (None, [P, C.c_uint32]),
            "w2v_model_options": (None, [P, I32, I32, I32]),
            "w2v_model_update_policy": (None, [P, I64, I32, I32, F, I64]),
            "w2v_model_context_policy": (None, [P, I32, I32]),
            "w2v_model_set_shared_negatives": (None, [P, I32]),
            "w2v_model_replicas": (None, [P, P, I32, I64, I32]),
            "w2v_model_replica_mode": (None, [P, I32]),
            "w2v_model_set_gpu_ingest": (None, [P, I32, I64]),
            "w2v_model_build_vocab": (C.c_int, [P, S, I64]),
            "w2v_model_train": (C.c_int, [P, S, I64]),
            "w2v_model_train_ids": (C.c_int, [P, P, P, I64, I64]),
            "w2v_model_init_weights": (C.c_int, [P]),
            "w2v_model_build_vocab_file": (C.c_int, [P, S, S, I32]),
            "w2v_model_train_file": (C.c_int, [P, S, S, I32]),
            "w2v_model_file_samples": (C.c_int, [P, S, S, I32, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64)]),
            "w2v_model_copy_samples": (C.c_int, [P, P, P]),
            "w2v_model_vocab_size": (I64, [P]),
            "w2v_model_word": (S, [P, I64]),
            "w2v_model_word_count": (I64, [P, I64]),
            "w2v_model_sample_probability": (F, [P, I64]),
            "w2v_model_path_length": (I64, [P, I64]),
            "w2v_model_path": (C.c_int, [P, I64, P, P]),
            "w2v_model_table_length": (I64, [P]),
            "w2v_model_table": (C.c_int, [P, P]),
            "w2v_model_rows": (I64, [P, I32]),
            "w2v_model_get_matrix": (C.c_int, [P, I32, P]),
            "w2v_model_set_matrix": (C.c_int, [P, I32, P, I64, I64]),
            "w2v_model_train_sentence": (C.c_int, [P, P, I64, F, I32]),
            "w2v_model_negative_sampling": (C.c_int, [P, I64, P, P, I32, F]),
            "w2v_model_hierarchical_softmax": (C.c_int, [P, I64, P, P, F]),
            "w2v_model_save": (C.c_int, [P, S, I32, I32]),
            "w2v_model_load": (C.c_int, [P, S, I32]),
            "w2v_model_save_vocab": (C.c_int, [P, S]),
            "w2v_model_create_huffman_tree": (C.c_int, [P]),
            "w2v_model_make_table": (C.c_int, [P]),
            "w2v_model_precalc_sampling": (C.c_int, [P]),
            "w2v_model_save_checkpoint": (C.c_int, [P, S]),
            "w2v_model_load_checkpoint": (C.c_int, [P, S]),
            "w2v_model_set_checkpoint_path": (C.c_int, [P, S]),
            "w2v_model_epochs_done": (I64, [P]),
            "w2v_model_epoch_seconds": (C.c_double, [P, I64]),
            "w2v_model_current_words": (I64, [P]),
            "w2v_model_replica_rounds": (I64, [P]),
            "w2v_model_replica_max_diff": (C.c_double, [P]),
            "w2v_model_read_vocab": (C.c_int, [P, S]),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype, f.argtypes = r, a
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _text(sentences) -> bytes:
    return "\n".join(" ".join(s) for s in sentences).encode()


class Word2Vec:
    """Mirror of the reference class; matrices are exposed as numpy copies."""

    W_, C_, SYN1 = 0, 1, 2

    def __init__(self, iter=1, window=5, min_count=5, table_size=100_000_000, word_dim=200, negative=0,
                 subsample_threshold=0.001, init_alpha=0.025, min_alpha=1e-6, cbow_mean=False, num_threads=1,
                 train_method="hs", model="cbow", gpu_device=0, replay_rng=False, verbose=False, hot_rows=-2,
                 private_rows=-1, flush_centers=0, private_average=8.0, max_waves=0, shared_negatives=False,
                 context_rows=-1, context_flush=0, gpu_devices=None, sync_words=0, overlap_average=True,
                 replica_mode="auto", gpu_ingest=False, ingest_chunk_bytes=0, checkpoint_path=""):
        self.L = _load()
        self.word_dim = word_dim
        self.h = self.L.w2v_model_new(iter, window, min_count, table_size, word_dim, negative, subsample_threshold,
                                      init_alpha, min_alpha, int(cbow_mean), num_threads, train_method.encode(),
                                      model.encode())
        if not self.h:
            raise RuntimeError("w2v_model_new failed")
        self.L.w2v_model_options(self.h, gpu_device, int(replay_rng), int(verbose))
        self.L.w2v_model_update_policy(self.h, int(hot_rows), int(private_rows), int(flush_centers),
                                       float(private_average), int(max_waves))
        self.L.w2v_model_set_shared_negatives(self.h, int(bool(shared_negatives)))
        self.L.w2v_model_context_policy(self.h, int(context_rows), int(context_flush))
        if gpu_devices:
            devs = np.ascontiguousarray(gpu_devices, np.int32)
            self.L.w2v_model_replicas(self.h, _p(devs), devs.size, int(sync_words), int(bool(overlap_average)))
            self.L.w2v_model_replica_mode(self.h, REPLICA_MODES.get(replica_mode, replica_mode))
        self.L.w2v_model_set_gpu_ingest(self.h, int(bool(gpu_ingest)), int(ingest_chunk_bytes))
        if checkpoint_path:
            self.set_checkpoint_path(checkpoint_path)

    def __del__(self):
        try:
            self.L.w2v_model_free(self.h)
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.L.w2v_model_last_error(self.h).decode(errors='replace')}")

    # reference API ---------------------------------------------------------
    def seed(self, s: int):
        """generator.seed(s) (the reference seeds from std::random_device)."""
        self.L.w2v_model_seed(self.h, s)

    def build_vocab(self, sentences):
        t = _text(sentences)
        self._chk(self.L.w2v_model_build_vocab(self.h, t, len(t)), "build_vocab")

    def init_weights(self):
        self._chk(self.L.w2v_model_init_weights(self.h), "init_weights")

    def train(self, sentences):
        t = _text(sentences)
        self._chk(self.L.w2v_model_train(self.h, t, len(t)), "train")

    def build_vocab_file(self, path, format="lines", threads=0):
        """Word2Vec::build_vocab_file: the vocab of a corpus file, bit-exact with build_vocab(line_docs(path))
        ("lines") or with the reference CLI's text8 reader ("text8")."""
        self._chk(self.L.w2v_model_build_vocab_file(self.h, str(path).encode(), format.encode(), int(threads)),
                  "build_vocab_file")

    def train_file(self, path, format="lines", threads=0):
        self._chk(self.L.w2v_model_train_file(self.h, str(path).encode(), format.encode(), int(threads)),
                  "train_file")

    def file_samples(self, path, format="lines", threads=0):
        """(ids, offsets, train_words): build_sample of a corpus file as token ids."""
        nt, ns, tw = C.c_int64(), C.c_int64(), C.c_int64()
        self._chk(self.L.w2v_model_file_samples(self.h, str(path).encode(), format.encode(), int(threads),
                                                C.byref(nt), C.byref(ns), C.byref(tw)), "file_samples")
        ids = np.empty(nt.value, np.int32)
        off = np.empty(ns.value + 1, np.int64)
        self._chk(self.L.w2v_model_copy_samples(self.h, _p(ids), _p(off)), "copy_samples")
        return ids, off, tw.value

    def train_ids(self, ids, offsets, train_words):
        ids = np.ascontiguousarray(ids, np.int32)
        off = np.ascontiguousarray(offsets, np.int64)
        self._chk(self.L.w2v_model_train_ids(self.h, _p(ids), _p(off), off.size - 1, int(train_words)), "train_ids")

    def train_sentence(self, ids, alpha: float, cbow: bool):
        ids = np.ascontiguousarray(ids, np.int32)
        self._chk(self.L.w2v_model_train_sentence(self.h, _p(ids), ids.size, float(alpha), int(cbow)),
                  "train_sentence")

    def negative_sampling(self, word: int, x, grad, which: int, alpha: float):
        x = np.array(x, np.float32)
        g = np.array(grad, np.float32)
        self._chk(self.L.w2v_model_negative_sampling(self.h, word, _p(x), _p(g), which, float(alpha)),
                  "negative_sampling")
        return g

    def hierarchical_softmax(self, word: int, x, grad, alpha: float):
        x = np.array(x, np.float32)
        g = np.array(grad, np.float32)
        self._chk(self.L.w2v_model_hierarchical_softmax(self.h, word, _p(x), _p(g), float(alpha)),
                  "hierarchical_softmax")
        return g

    def save_word2vec(self, path, which=0, binary=False):
        self._chk(self.L.w2v_model_save(self.h, str(path).encode(), which, int(binary)), "save_word2vec")

    def load_word2vec(self, path, binary=False):
        self._chk(self.L.w2v_model_load(self.h, str(path).encode(), int(binary)), "load_word2vec")

    def save_checkpoint(self, path):
        self._chk(self.L.w2v_model_save_checkpoint(self.h, str(path).encode()), "save_checkpoint")

    def load_checkpoint(self, path):
        """Restore W / C / synapses1, current_words, the schedule position and the generator: a mid-schedule
        checkpoint's next train runs the remaining epochs, a whole-schedule one starts a new schedule on the
        loaded weights (include/Word2Vec.h)."""
        self._chk(self.L.w2v_model_load_checkpoint(self.h, str(path).encode()), "load_checkpoint")

    def set_checkpoint_path(self, path):
        """Write a checkpoint after every epoch of train ("" = off; "%d" in the path = the epochs done)."""
        self._chk(self.L.w2v_model_set_checkpoint_path(self.h, str(path).encode()), "set_checkpoint_path")

    @property
    def epochs_done(self) -> int:
        return self.L.w2v_model_epochs_done(self.h)

    @property
    def epoch_seconds(self) -> list:
        """Wall seconds of each device epoch of the last train call."""
        out = []
        while (t := self.L.w2v_model_epoch_seconds(self.h, len(out))) >= 0:
            out.append(t)
        return out

    @property
    def replica_rounds(self) -> int:
        """Exchanges the replicas (gpu_devices) ran in the last train call."""
        return self.L.w2v_model_replica_rounds(self.h)

    @property
    def replica_max_diff(self) -> float:
        """max |M_i - M_0| / max |M_0| over the replicas after the last exchange (-1: not measured)."""
        return self.L.w2v_model_replica_max_diff(self.h)

    @property
    def current_words(self) -> int:
        return self.L.w2v_model_current_words(self.h)

    def save_vocab(self, path):
        self._chk(self.L.w2v_model_save_vocab(self.h, str(path).encode()), "save_vocab")

    def read_vocab(self, path):
        self._chk(self.L.w2v_model_read_vocab(self.h, str(path).encode()), "read_vocab")

    def create_huffman_tree(self):
        self._chk(self.L.w2v_model_create_huffman_tree(self.h), "create_huffman_tree")

    def make_table(self):
        self._chk(self.L.w2v_model_make_table(self.h), "make_table")

    def precalc_sampling(self):
        self._chk(self.L.w2v_model_precalc_sampling(self.h), "precalc_sampling")

    # introspection ---------------------------------------------------------
    @property
    def V(self) -> int:
        return self.L.w2v_model_vocab_size(self.h)

    def vocab(self):
        V = self.V
        words = [self.L.w2v_model_word(self.h, i).decode("utf-8", errors="surrogateescape") for i in range(V)]  # indices in range: never NULL
        counts = np.array([self.L.w2v_model_word_count(self.h, i) for i in range(V)], np.int64)
        return words, counts

    def sample_probs(self):
        return np.array([self.L.w2v_model_sample_probability(self.h, i) for i in range(self.V)], np.float32)

    def huffman(self):
        V = self.V
        lens = np.array([self.L.w2v_model_path_length(self.h, i) for i in range(V)], np.int64)
        off = np.zeros(V + 1, np.int64)
        off[1:] = np.cumsum(lens)
        codes = np.zeros(max(int(off[-1]), 1), np.uint8)
        points = np.zeros(max(int(off[-1]), 1), np.int32)
        for i in range(V):
            if lens[i]:
                c = np.zeros(lens[i], np.uint8)
                p = np.zeros(lens[i], np.int32)
                self.L.w2v_model_path(self.h, i, _p(c), _p(p))
                codes[off[i]:off[i + 1]] = c
                points[off[i]:off[i + 1]] = p
        return codes[: off[-1]], points[: off[-1]], off

    def table(self):
        out = np.empty(self.L.w2v_model_table_length(self.h), np.uint32)
        self.L.w2v_model_table(self.h, _p(out))
        return out

    def matrix(self, which: int):
        rows = self.L.w2v_model_rows(self.h, which)
        out = np.empty((max(rows, 0), self.word_dim), np.float32)
        if rows > 0:
            self.L.w2v_model_get_matrix(self.h, which, _p(out))
        return out

    def set_matrix(self, which: int, m):
        m = np.ascontiguousarray(m, np.float32)
        if m.ndim != 2 or m.shape[1] != self.word_dim:
            raise ValueError(f"set_matrix: expected (rows, {self.word_dim}), got {m.shape}")
        self._chk(self.L.w2v_model_set_matrix(self.h, which, _p(m), m.shape[0], m.shape[1]), "set_matrix")
