"""ctypes binding of include/w2v_host.h (libword2vec_amd.so): the host-side
vocab products that feed the device (bit-exact restatements of the
reference's make_table / precalc_sampling / create_huffman_tree)."""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

HOST_LIB = Path(__file__).resolve().parent / "lib" / "libword2vec_amd.so"
if os.environ.get("W2V_DEV_LIB"):  # a diagnostic device library: use the host library linked beside it
    HOST_LIB = Path(os.environ["W2V_DEV_LIB"]).resolve().parent / "libword2vec_amd.so"
_lib = None


def load_host_lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not HOST_LIB.exists():
            raise RuntimeError(f"word2vec_amd: host library {HOST_LIB} is missing; run make -C word2vec_amd/csrc")
        L = C.CDLL(str(HOST_LIB), mode=C.RTLD_GLOBAL)
        P, I64, I32, F = C.c_void_p, C.c_int64, C.c_int32, C.c_float
        sig = {
            "w2v_host_version": (C.c_char_p, []),
            "w2v_host_sample_probs": (None, [P, I64, F, P]),
            "w2v_host_table_bounds": (None, [P, I64, I32, P]),
            "w2v_host_table_fill": (None, [P, I64, P, I64]),
            "w2v_host_huffman": (I64, [P, I64, P, P, P, I64]),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype, f.argtypes = r, a
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def sample_probs(counts, subsample: float) -> np.ndarray:
    c = np.ascontiguousarray(counts, np.int64)
    out = np.empty(c.size, np.float32)
    load_host_lib().w2v_host_sample_probs(_p(c), c.size, subsample, _p(out))
    return out


def table_bounds(counts, table_size: int) -> np.ndarray:
    c = np.ascontiguousarray(counts, np.int64)
    out = np.empty(c.size + 1, np.int64)
    load_host_lib().w2v_host_table_bounds(_p(c), c.size, int(table_size), _p(out))
    return out


def table_fill(bounds, table_size: int) -> np.ndarray:
    b = np.ascontiguousarray(bounds, np.int64)
    out = np.empty(int(table_size), np.uint32)
    load_host_lib().w2v_host_table_fill(_p(b), b.size - 1, _p(out), out.size)
    return out


def huffman(counts):
    c = np.ascontiguousarray(counts, np.int64)
    L = load_host_lib()
    off = np.empty(c.size + 1, np.int64)
    n = L.w2v_host_huffman(_p(c), c.size, None, None, _p(off), 0)
    if n < 0:
        raise ValueError("huffman needs at least 2 words")
    codes = np.empty(max(n, 1), np.uint8)
    points = np.empty(max(n, 1), np.int32)
    L.w2v_host_huffman(_p(c), c.size, _p(codes), _p(points), _p(off), n)
    return codes[:n], points[:n], off
