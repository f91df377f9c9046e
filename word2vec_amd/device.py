"""Python handle over the C-ABI (include/w2v_dev.h): HBM-resident training state.

This is the thin plumbing the tests, the bench and the multi-GPU driver use;
the C++ host class (include/Word2Vec.h) drives the same C-ABI. All compute runs
in the HIP kernels of libw2v_hip.so.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native as N


def _ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays passed to the C-ABI must be C-contiguous"
    return a.ctypes.data_as(C.c_void_p)


@dataclass
class Config:
    """Mirror of w2v_dev_config (Word2Vec ctor fields, Word2Vec.h:64-66)."""

    word_dim: int = 200
    window: int = 5
    negative: int = 0
    hs: bool = True
    cbow: bool = True
    cbow_mean: bool = False
    iter: int = 1
    init_alpha: float = 0.025
    min_alpha: float = 1e-6
    table_size: int = 100_000_000
    device: int = -1

    def to_c(self) -> N.DevConfig:
        return N.DevConfig(
            int(self.word_dim), int(self.window), int(self.negative), int(bool(self.hs)),
            int(bool(self.cbow)), int(bool(self.cbow_mean)), int(self.iter),
            float(self.init_alpha), float(self.min_alpha), int(self.table_size),
            int(self.device), 0,
        )


class DeviceTrainer:
    """Owns one w2v_dev handle (one GPU)."""

    def __init__(self, cfg: Config):
        self.lib = N.load_dev_lib()
        self.cfg = cfg
        h = C.c_void_p()
        c = cfg.to_c()
        N.check(self.lib, self.lib.w2v_dev_create(C.byref(c), C.byref(h)), "w2v_dev_create")
        self.h = h
        self.V = 0

    # -- lifecycle -----------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.w2v_dev_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        N.check(self.lib, rc, what)

    # -- configuration -------------------------------------------------------
    def set_stream(self, stream_handle: int | None):
        self._chk(self.lib.w2v_dev_set_stream(self.h, C.c_void_p(stream_handle or 0) if stream_handle else None),
                  "w2v_dev_set_stream")

    def set_rng(self, mode: int, seed: int = 0):
        self._chk(self.lib.w2v_dev_set_rng(self.h, mode, seed & ((1 << 64) - 1)), "w2v_dev_set_rng")

    def set_schedule(self, sched: int):
        self._chk(self.lib.w2v_dev_set_schedule(self.h, sched), "w2v_dev_set_schedule")

    # -- uploads -------------------------------------------------------------
    def upload_vocab(self, sample_prob, table_bounds=None, codes=None, points=None, code_offsets=None):
        sp = np.ascontiguousarray(sample_prob, dtype=np.float32)
        tb = None if table_bounds is None else np.ascontiguousarray(table_bounds, dtype=np.int64)
        cd = None if codes is None else np.ascontiguousarray(codes, dtype=np.uint8)
        pt = None if points is None else np.ascontiguousarray(points, dtype=np.int32)
        co = None if code_offsets is None else np.ascontiguousarray(code_offsets, dtype=np.int64)
        self._chk(self.lib.w2v_dev_upload_vocab(self.h, sp.size, _ptr(sp), _ptr(tb), _ptr(cd), _ptr(pt), _ptr(co)),
                  "w2v_dev_upload_vocab")
        self.V = sp.size

    def upload_table(self, table):
        t = np.ascontiguousarray(table, dtype=np.uint32)
        self._chk(self.lib.w2v_dev_upload_table(self.h, _ptr(t), t.size), "w2v_dev_upload_table")

    def upload_model(self, W=None, C_=None, S=None):
        d = self.cfg.word_dim
        arrs = [None if a is None else np.ascontiguousarray(a, dtype=np.float32).reshape(-1, d) for a in (W, C_, S)]
        self._chk(self.lib.w2v_dev_upload_model(self.h, *[_ptr(a) for a in arrs]), "w2v_dev_upload_model")

    def max_diff(self, other) -> dict:
        """w2v_dev_model_max_diff: per matrix (max |self - other|, max |self|)."""
        out = (C.c_float * 6)()
        self._chk(self.lib.w2v_dev_model_max_diff(self.h, other.h, out), "w2v_dev_model_max_diff")
        return {k: (out[i], out[3 + i]) for i, k in enumerate(("W", "C", "S"))}

    def download_model(self):
        d, V = self.cfg.word_dim, self.V
        W = np.empty((V, d), np.float32)
        need_c = self.cfg.negative > 0 or self.cfg.cbow
        Cm = np.empty((V, d), np.float32) if need_c else None
        S = np.empty((max(V - 1, 0), d), np.float32) if self.cfg.hs else None
        self._chk(self.lib.w2v_dev_download_model(self.h, _ptr(W), _ptr(Cm), _ptr(S)), "w2v_dev_download_model")
        return W, Cm, S

    def bind_model(self, dW: int, dC: int | None, dS: int | None, pitch: int):
        """Train on caller-owned device buffers (e.g. torch tensors) of row pitch `pitch` floats."""
        self._chk(self.lib.w2v_dev_bind_model(self.h, C.c_void_p(dW), C.c_void_p(dC) if dC else None,
                                              C.c_void_p(dS) if dS else None, int(pitch)), "w2v_dev_bind_model")

    def row_pitch(self) -> int:
        """The smallest row pitch (floats) bind_model accepts: the kernels' row width."""
        p = C.c_int64()
        self._chk(self.lib.w2v_dev_row_pitch(self.h, C.byref(p)), "w2v_dev_row_pitch")
        return p.value

    def model_layout(self):
        w, c, s, p = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_int64()
        self._chk(self.lib.w2v_dev_model_layout(self.h, C.byref(w), C.byref(c), C.byref(s), C.byref(p)),
                  "w2v_dev_model_layout")
        return w.value, c.value, s.value, p.value

    def upload_corpus(self, ids, sent_offsets, train_words: int):
        i = np.ascontiguousarray(ids, dtype=np.int32)
        o = np.ascontiguousarray(sent_offsets, dtype=np.int64)
        self._chk(self.lib.w2v_dev_upload_corpus(self.h, _ptr(i), i.size, _ptr(o), o.size - 1, int(train_words)),
                  "w2v_dev_upload_corpus")
        self.n_sent = o.size - 1

    def share_corpus(self, src: "DeviceTrainer"):
        """Train on src's resident corpus (same device and vocab; no copy). The C side counts references,
        so src may be closed first; the corpus is freed with the last handle holding it."""
        self._chk(self.lib.w2v_dev_share_corpus(self.h, src.h), "w2v_dev_share_corpus")
        self.n_sent = src.n_sent

    def adopt_corpus(self, ingest):
        """w2v_dev_adopt_corpus: the samples of a mapped GpuIngest (word2vec_amd/ingest.py), device to device."""
        self._chk(self.lib.w2v_dev_adopt_corpus(self.h, ingest.g), "w2v_dev_adopt_corpus")
        ni, ns, tw = C.c_int64(), C.c_int64(), C.c_int64()
        self._chk(self.lib.w2v_ingest_samples_size(ingest.g, C.byref(ni), C.byref(ns), C.byref(tw)),
                  "w2v_ingest_samples_size")
        self.n_sent = ns.value

    def upload_replay(self, stream, offsets):
        s = np.ascontiguousarray(stream, dtype=np.uint32)
        o = np.ascontiguousarray(offsets, dtype=np.int64)
        self._chk(self.lib.w2v_dev_upload_replay(self.h, _ptr(s), s.size, _ptr(o), o.size), "w2v_dev_upload_replay")

    # -- training ------------------------------------------------------------
    def set_progress(self, cw: int):
        self._chk(self.lib.w2v_dev_set_progress(self.h, int(cw)), "w2v_dev_set_progress")

    def set_progress_async(self, cw: int):
        """Set the device word counter, ordered on the handle's stream (no host sync)."""
        self._chk(self.lib.w2v_dev_set_progress_async(self.h, int(cw)), "w2v_dev_set_progress_async")

    def set_train_words(self, train_words: int):
        """Denominator of the alpha schedule (Word2Vec.cpp:362-363,379-380)."""
        self._chk(self.lib.w2v_dev_set_train_words(self.h, int(train_words)), "w2v_dev_set_train_words")

    def get_progress(self) -> int:
        v = C.c_int64()
        self._chk(self.lib.w2v_dev_get_progress(self.h, C.byref(v)), "w2v_dev_get_progress")
        return v.value

    def train_epoch(self, epoch: int, order=None) -> dict:
        st = N.DevStats()
        o = None if order is None else np.ascontiguousarray(order, dtype=np.int64)
        self._chk(self.lib.w2v_dev_train_epoch(self.h, int(epoch), _ptr(o), C.byref(st)), "w2v_dev_train_epoch")
        return st.as_dict()

    def train_epoch_async(self, epoch: int, order_dev_ptr: int | None = None):
        self._chk(self.lib.w2v_dev_train_epoch_async(self.h, int(epoch),
                                                     C.c_void_p(order_dev_ptr) if order_dev_ptr else None),
                  "w2v_dev_train_epoch_async")

    def train_sentences_async(self, epoch: int, order_dev_ptr: int, count: int):
        """Train `count` sentences listed in a device int64 array (a slice of an epoch's order)."""
        self._chk(self.lib.w2v_dev_train_sentences_async(self.h, int(epoch), C.c_void_p(order_dev_ptr), int(count)),
                  "w2v_dev_train_sentences_async")

    def set_order(self, order):
        """Keep an epoch's sentence order on the device (for train_slice_async)."""
        o = np.ascontiguousarray(order, dtype=np.int64)
        self._chk(self.lib.w2v_dev_set_order(self.h, _ptr(o), o.size), "w2v_dev_set_order")

    def train_slice_async(self, epoch: int, first: int, count: int):
        """Train order[first:first + count] of the order set with set_order."""
        self._chk(self.lib.w2v_dev_train_slice_async(self.h, int(epoch), int(first), int(count)),
                  "w2v_dev_train_slice_async")

    def synchronize(self):
        self._chk(self.lib.w2v_dev_synchronize(self.h), "w2v_dev_synchronize")

    def read_stats(self) -> dict:
        st = N.DevStats()
        self._chk(self.lib.w2v_dev_read_stats(self.h, C.byref(st)), "w2v_dev_read_stats")
        return st.as_dict()

    def knobs(self) -> str:
        """Experiment environment variables this handle read at creation ("" if none)."""
        return self.lib.w2v_dev_knobs(self.h).decode()

    def reset_stats(self):
        self._chk(self.lib.w2v_dev_reset_stats(self.h), "w2v_dev_reset_stats")

    def set_hot_rows(self, hot_rows: int):
        """Rows updated with atomics: -2 = auto from the corpus statistics (default), -1 = all,
        0 = none (plain Hogwild RMW), k = the k most frequent."""
        self._chk(self.lib.w2v_dev_set_hot_rows(self.h, int(hot_rows)), "w2v_dev_set_hot_rows")

    def set_hot_auto(self, tau_rows: float = 0.0, tau_nodes: float = 1.0):
        """Thresholds of the automatic hot rows (expected updates in flight of a W / C row, of a Huffman node);
        tau_rows 0 = the library default (1)."""
        self._chk(self.lib.w2v_dev_set_hot_auto(self.h, float(tau_rows), float(tau_nodes)), "w2v_dev_set_hot_auto")

    def policy(self) -> dict:
        """The update policy the last parallel launch used."""
        r, n, p, c = C.c_int64(), C.c_int64(), C.c_int32(), C.c_int32()
        self._chk(self.lib.w2v_dev_policy(self.h, C.byref(r), C.byref(n), C.byref(p), C.byref(c)), "w2v_dev_policy")
        f, cf = C.c_int32(), C.c_int32()
        self._chk(self.lib.w2v_dev_flush_policy(self.h, C.byref(f), C.byref(cf)), "w2v_dev_flush_policy")
        tr, tn = C.c_float(), C.c_float()
        self._chk(self.lib.w2v_dev_hot_tau(self.h, C.byref(tr), C.byref(tn)), "w2v_dev_hot_tau")
        mu = C.c_float()
        self._chk(self.lib.w2v_dev_private_rate_used(self.h, C.byref(mu)), "w2v_dev_private_rate_used")
        wc = C.c_int64()
        self._chk(self.lib.w2v_dev_wave_cap_used(self.h, C.byref(wc)), "w2v_dev_wave_cap_used")
        dp = C.c_int32()
        self._chk(self.lib.w2v_dev_deep_used(self.h, C.byref(dp)), "w2v_dev_deep_used")
        return {"hot_rows": r.value, "hot_nodes": n.value, "private_rows": p.value, "context_rows": c.value,
                "flush_centers": f.value, "context_flush": cf.value, "hot_tau_rows": tr.value,
                "private_rate": round(mu.value, 4), "wave_cap": wc.value, "deep": dp.value}

    def set_private_rows(self, n: int):
        """Hottest output rows privatised per workgroup in LDS: -1 auto (default), 0 off."""
        self._chk(self.lib.w2v_dev_set_private_rows(self.h, int(n)), "w2v_dev_set_private_rows")

    def set_private_rate(self, mu: float):
        """Privatise only rows updated >= mu times per center (0 = no rate limit, -1 = automatic: 0.1 for a
        launch with fewer sentences than the chip holds waves)."""
        self._chk(self.lib.w2v_dev_set_private_rate(self.h, float(mu)), "w2v_dev_set_private_rate")

    def set_private_sync(self, flush_centers: int = 0, average_over: float = 8.0):
        """Workgroup centers between flushes of the private rows (0 = auto) and the
        concurrency their summed deltas are scaled to (0 = plain sum); include/w2v_dev.h."""
        self._chk(self.lib.w2v_dev_set_private_sync(self.h, int(flush_centers), float(average_over)),
                  "w2v_dev_set_private_sync")

    def set_context_private(self, rows: int = -1, flush_centers: int = 0):
        """CBOW: hottest context rows privatised in LDS too (-1 auto, 0 off) and the
        workgroup centers between their flushes (0 = auto); include/w2v_dev.h."""
        self._chk(self.lib.w2v_dev_set_context_private(self.h, int(rows), int(flush_centers)),
                  "w2v_dev_set_context_private")

    def row_update_rates(self, which: int, rows: int) -> np.ndarray:
        """Expected updates per raw token of each row of matrix `which` (0 W, 1 C, 2 synapses1)."""
        out = np.empty(rows, np.float64)
        self._chk(self.lib.w2v_dev_row_update_rates(self.h, int(which), out.ctypes.data_as(C.POINTER(C.c_double)),
                                                    int(rows)), "w2v_dev_row_update_rates")
        return out

    def set_max_waves(self, n: int):
        """Cap on wavefronts in flight (0 = as many as fit)."""
        self._chk(self.lib.w2v_dev_set_max_waves(self.h, int(n)), "w2v_dev_set_max_waves")

    def set_update(self, mode: int):
        """W2V_UPDATE_PER_PAIR (the reference's, default) or W2V_UPDATE_SHARED_NEGATIVES
        (minibatch skip-gram on the matrix cores, BASELINE configs[4]); include/w2v_dev.h."""
        self._chk(self.lib.w2v_dev_set_update(self.h, int(mode)), "w2v_dev_set_update")

    def set_fixed_alpha(self, alpha: float):
        self._chk(self.lib.w2v_dev_set_fixed_alpha(self.h, float(alpha)), "w2v_dev_set_fixed_alpha")

    def apply_rows(self, rows, codes, x, grad, alpha: float, hs_form: bool):
        """Sequential NS/HS updates of distinct host rows on the device; returns (rows, grad)."""
        r = np.array(rows, dtype=np.float32, copy=True).reshape(-1, self.cfg.word_dim)
        c = np.ascontiguousarray(codes, dtype=np.uint8)
        x = np.ascontiguousarray(x, dtype=np.float32)
        g = np.array(grad, dtype=np.float32, copy=True)
        self._chk(self.lib.w2v_dev_apply_rows(self.h, _ptr(r), _ptr(c), c.size, _ptr(x), _ptr(g), float(alpha),
                                              int(bool(hs_form))), "w2v_dev_apply_rows")
        return r, g
