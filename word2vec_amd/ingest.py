"""GPU corpus ingestion (include/w2v_ingest.h): the vocabulary count and the
id mapping of a corpus file on the device, bit-exact with the host readers
(csrc/host/corpus.cpp) — Word2Vec.cpp:132-160 (build_vocab's count in corpus
order) and :212-230 (build_sample), for the line_docs reader
(Word2Vec.cpp:19-30) and the reference CLI's text8 reader (main.cpp:63-92).

    g = GpuIngest("corpus.txt", "lines")
    words = g.count()                 # [(word, count)] in order of first occurrence
    g.map({w: i for i, w in ...})     # vocab index per word (absent: dropped)
    ids, offsets, train_words = g.samples()
    trainer.adopt_corpus(g)           # the samples stay in HBM
"""
from __future__ import annotations

import ctypes as C
import mmap
import os

import numpy as np

from . import _native as N

FORMATS = {"lines": N.W2V_INGEST_LINES, "text8": N.W2V_INGEST_TEXT8}


class GpuIngest:
    def __init__(self, path: str | os.PathLike, format: str = "lines", device: int = -1, chunk_bytes: int = 0,
                 resident_max: int = -1):
        if format not in FORMATS:
            raise ValueError(f'format must be "lines" or "text8", not {format!r}')
        self.lib = N.load_dev_lib()
        self.path = str(path)
        self._f = open(self.path, "rb")
        size = os.fstat(self._f.fileno()).st_size
        self._m = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ) if size > 0 else None
        self.size = size
        g = C.c_void_p()
        N.check(self.lib, self.lib.w2v_ingest_create(int(device), FORMATS[format], int(chunk_bytes), C.byref(g)),
                "w2v_ingest_create")
        self.g = g
        N.check(self.lib, self.lib.w2v_ingest_set_resident(self.g, int(resident_max)), "w2v_ingest_set_resident")
        self.n_words = None

    def _data(self):
        """The mapped file as a uint8 array (no copy) and its address."""
        if self._m is None:
            return None, None
        arr = np.frombuffer(self._m, dtype=np.uint8)
        return arr, arr.ctypes.data_as(C.c_void_p)

    def count(self) -> list[tuple[str, int]]:
        arr, ptr = self._data()
        N.check(self.lib, self.lib.w2v_ingest_count(self.g, ptr, self.size), "w2v_ingest_count")
        nw, raw, ns = C.c_int64(), C.c_int64(), C.c_int64()
        N.check(self.lib, self.lib.w2v_ingest_summary(self.g, C.byref(nw), C.byref(raw), C.byref(ns)),
                "w2v_ingest_summary")
        self.n_words, self.raw_tokens, self.n_sentences = nw.value, raw.value, ns.value
        first = np.empty(self.n_words, np.int64)
        length = np.empty(self.n_words, np.int32)
        cnt = np.empty(self.n_words, np.int64)
        N.check(self.lib, self.lib.w2v_ingest_words(self.g, first.ctypes.data, length.ctypes.data, cnt.ctypes.data),
                "w2v_ingest_words")
        m = self._m
        self.words = [m[int(o):int(o) + int(n)].decode("utf-8", errors="surrogateescape") for o, n in zip(first, length)]
        self.counts = cnt
        del arr
        return list(zip(self.words, (int(c) for c in cnt)))

    def map(self, index: dict) -> None:
        """Pass 2: `index` maps a word to its vocab index (words not in it are dropped)."""
        if self.n_words is None:
            raise RuntimeError("GpuIngest.count() first")
        vi = np.array([index.get(w, -1) for w in self.words], dtype=np.int32)
        arr, ptr = self._data()
        N.check(self.lib, self.lib.w2v_ingest_map(self.g, ptr, self.size, vi.ctypes.data, vi.size), "w2v_ingest_map")
        del arr

    def samples(self):
        """(ids int32, offsets int64, train_words) of pass 2, copied to the host."""
        ni, ns, tw = C.c_int64(), C.c_int64(), C.c_int64()
        N.check(self.lib, self.lib.w2v_ingest_samples_size(self.g, C.byref(ni), C.byref(ns), C.byref(tw)),
                "w2v_ingest_samples_size")
        ids = np.empty(ni.value, np.int32)
        off = np.empty(ns.value + 1, np.int64)
        N.check(self.lib, self.lib.w2v_ingest_download(self.g, ids.ctypes.data, off.ctypes.data), "w2v_ingest_download")
        return ids, off, tw.value

    def close(self):
        if getattr(self, "g", None):
            self.lib.w2v_ingest_destroy(self.g)
            self.g = None
        if getattr(self, "_m", None) is not None:
            self._m.close()
            self._m = None
        if getattr(self, "_f", None) is not None:
            self._f.close()
            self._f = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
