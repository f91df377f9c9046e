"""ctypes binding of the C-ABI in include/w2v_dev.h (libw2v_hip.so).

The library is built in-tree (``word2vec_amd/lib``) by ``__graft_entry__.build()``
or ``make -C word2vec_amd/csrc``. There is no fallback: if the HIP library is
missing, importing the device API raises, so nothing can silently run a CPU
path in its place.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_DIR = Path(__file__).resolve().parent / "lib"
DEV_LIB = LIB_DIR / "libw2v_hip.so"

W2V_OK = 0
W2V_ERR_ARG = 1
W2V_ERR_HIP = 2
W2V_ERR_STATE = 3
W2V_ERR_UNSUPPORTED = 4
W2V_ERR_DIVERGED = 5
W2V_ERR_COMM = 6
W2V_GROUP_ID_BYTES = 128
W2V_GROUP_SUM = 0
W2V_GROUP_AVERAGE = 1
W2V_GROUP_ROW_AVERAGE = 2
W2V_GROUP_ADAPTIVE = 3
W2V_GROUP_SPLIT = 4
W2V_GROUP_SATURATION = 5
W2V_RNG_PHILOX = 0
W2V_RNG_REPLAY = 1
W2V_SCHED_PARALLEL = 0
W2V_SCHED_SEQUENTIAL = 1
W2V_UPDATE_PER_PAIR = 0
W2V_UPDATE_SHARED_NEGATIVES = 1
W2V_HOT_AUTO = -2


class DevConfig(C.Structure):
    _fields_ = [
        ("word_dim", C.c_int32),
        ("window", C.c_int32),
        ("negative", C.c_int32),
        ("hs", C.c_int32),
        ("cbow", C.c_int32),
        ("cbow_mean", C.c_int32),
        ("iter", C.c_int32),
        ("init_alpha", C.c_float),
        ("min_alpha", C.c_float),
        ("table_size", C.c_int64),
        ("device", C.c_int32),
        ("reserved", C.c_int32),
    ]


class DevStats(C.Structure):
    _fields_ = [
        ("words", C.c_int64),
        ("centers", C.c_int64),
        ("contexts", C.c_int64),
        ("targets", C.c_int64),
        ("draws", C.c_int64),
        ("sentences", C.c_int64),
        ("nonfinite", C.c_int64),
    ]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


_P = C.c_void_p
_I32 = C.c_int32
_I64 = C.c_int64
_U64 = C.c_uint64
_F = C.c_float

# name -> (restype, argtypes); mirrors include/w2v_dev.h one for one.
SIGNATURES = {
    "w2v_dev_version": (C.c_char_p, []),
    "w2v_dev_limits": (C.c_int, [C.POINTER(_I32)] * 5),
    "w2v_dev_shared_limits": (C.c_int, [C.POINTER(_I32)] * 3),
    "w2v_dev_last_error": (C.c_char_p, []),
    "w2v_dev_knobs": (C.c_char_p, [_P]),
    "w2v_dev_create": (C.c_int, [C.POINTER(DevConfig), C.POINTER(_P)]),
    "w2v_dev_destroy": (None, [_P]),
    "w2v_dev_set_stream": (C.c_int, [_P, _P]),
    "w2v_dev_set_rng": (C.c_int, [_P, _I32, _U64]),
    "w2v_dev_set_schedule": (C.c_int, [_P, _I32]),
    "w2v_dev_upload_vocab": (C.c_int, [_P, _I64, _P, _P, _P, _P, _P]),
    "w2v_dev_upload_table": (C.c_int, [_P, _P, _I64]),
    "w2v_dev_upload_model": (C.c_int, [_P, _P, _P, _P]),
    "w2v_dev_download_model": (C.c_int, [_P, _P, _P, _P]),
    "w2v_dev_upload_rows": (C.c_int, [_P, _I32, _P, _I64, _P]),
    "w2v_dev_download_rows": (C.c_int, [_P, _I32, _P, _I64, _P]),
    "w2v_dev_bind_model": (C.c_int, [_P, _P, _P, _P, _I64]),
    "w2v_dev_row_pitch": (C.c_int, [_P, C.POINTER(_I64)]),
    "w2v_dev_model_layout": (C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), C.POINTER(_P), C.POINTER(_I64)]),
    "w2v_dev_upload_corpus": (C.c_int, [_P, _P, _I64, _P, _I64, _I64]),
    "w2v_dev_share_corpus": (C.c_int, [_P, _P]),
    "w2v_dev_upload_replay": (C.c_int, [_P, _P, _I64, _P, _I64]),
    "w2v_dev_set_progress": (C.c_int, [_P, _I64]),
    "w2v_dev_get_progress": (C.c_int, [_P, C.POINTER(_I64)]),
    "w2v_dev_set_progress_async": (C.c_int, [_P, _I64]),
    "w2v_dev_set_train_words": (C.c_int, [_P, _I64]),
    "w2v_dev_train_epoch": (C.c_int, [_P, _I32, _P, C.POINTER(DevStats)]),
    "w2v_dev_train_epoch_async": (C.c_int, [_P, _I32, _P]),
    "w2v_dev_train_sentences_async": (C.c_int, [_P, _I32, _P, _I64]),
    "w2v_dev_synchronize": (C.c_int, [_P]),
    "w2v_dev_set_order": (C.c_int, [_P, _P, _I64]),
    "w2v_dev_train_slice_async": (C.c_int, [_P, _I32, _I64, _I64]),
    "w2v_dev_read_stats": (C.c_int, [_P, C.POINTER(DevStats)]),
    "w2v_dev_reset_stats": (C.c_int, [_P]),
    "w2v_dev_set_fixed_alpha": (C.c_int, [_P, _F]),
    "w2v_dev_set_hot_rows": (C.c_int, [_P, _I64]),
    "w2v_dev_set_hot_auto": (C.c_int, [_P, _F, _F]),
    "w2v_dev_policy": (C.c_int, [_P, C.POINTER(_I64), C.POINTER(_I64), C.POINTER(_I32), C.POINTER(_I32)]),
    "w2v_dev_flush_policy": (C.c_int, [_P, C.POINTER(_I32), C.POINTER(_I32)]),
    "w2v_dev_hot_tau": (C.c_int, [_P, C.POINTER(_F), C.POINTER(_F)]),
    "w2v_dev_private_rate_used": (C.c_int, [_P, C.POINTER(_F)]),
    "w2v_dev_wave_cap_used": (C.c_int, [_P, C.POINTER(_I64)]),
    "w2v_dev_deep_used": (C.c_int, [_P, C.POINTER(_I32)]),
    "w2v_dev_set_replica_count": (C.c_int, [_P, _I32]),
    "w2v_dev_model_max_diff": (C.c_int, [_P, _P, C.POINTER(_F)]),
    "w2v_dev_replica_count": (C.c_int, [_P, C.POINTER(_I32)]),
    "w2v_dev_set_private_rows": (C.c_int, [_P, _I32]),
    "w2v_dev_set_private_rate": (C.c_int, [_P, _F]),
    "w2v_dev_set_private_sync": (C.c_int, [_P, _I32, _F]),
    "w2v_dev_set_context_private": (C.c_int, [_P, _I32, _I32]),
    "w2v_dev_set_max_waves": (C.c_int, [_P, _I64]),
    "w2v_dev_set_update": (C.c_int, [_P, _I32]),
    "w2v_dev_apply_rows": (C.c_int, [_P, _P, _P, _I32, _P, _P, _F, _I32]),
    "w2v_group_unique_id": (C.c_int, [_P]),
    "w2v_group_create": (C.c_int, [_P, _I32, _P, _I32, _I32, C.POINTER(_P)]),
    "w2v_group_destroy": (None, [_P]),
    "w2v_group_set_overlap": (C.c_int, [_P, _I32]),
    "w2v_group_set_mode": (C.c_int, [_P, _I32]),
    "w2v_group_set_split": (C.c_int, [_P, _I64, _F]),
    "w2v_group_set_saturation": (C.c_int, [_P, _I64, _F]),
    "w2v_group_row_divisors": (C.c_int, [_P, _I32, C.POINTER(_F), _I64]),
    "w2v_dev_row_update_rates": (C.c_int, [_P, _I32, C.POINTER(C.c_double), _I64]),
    "w2v_group_split_rows": (C.c_int, [_P, C.POINTER(_I64)]),
    "w2v_group_average_async": (C.c_int, [_P]),
    "w2v_group_average_rows_async": (C.c_int, [_P, _I64]),
    "w2v_group_finish": (C.c_int, [_P]),
    "w2v_group_info": (C.c_int, [_P, C.POINTER(_I32), C.POINTER(_I32), C.POINTER(_I32), C.POINTER(_I64)]),
    # include/w2v_ingest.h
    "w2v_ingest_create": (C.c_int, [_I32, _I32, _I64, C.POINTER(_P)]),
    "w2v_ingest_destroy": (None, [_P]),
    "w2v_ingest_set_resident": (C.c_int, [_P, _I64]),
    "w2v_ingest_count": (C.c_int, [_P, _P, _I64]),
    "w2v_ingest_summary": (C.c_int, [_P, C.POINTER(_I64), C.POINTER(_I64), C.POINTER(_I64)]),
    "w2v_ingest_words": (C.c_int, [_P, _P, _P, _P]),
    "w2v_ingest_map": (C.c_int, [_P, _P, _I64, _P, _I64]),
    "w2v_ingest_samples_size": (C.c_int, [_P, C.POINTER(_I64), C.POINTER(_I64), C.POINTER(_I64)]),
    "w2v_ingest_download": (C.c_int, [_P, _P, _P]),
    "w2v_dev_adopt_corpus": (C.c_int, [_P, _P]),
}
W2V_INGEST_LINES = 0
W2V_INGEST_TEXT8 = 1

_lib = None


def load_dev_lib(path: os.PathLike | str | None = None) -> C.CDLL:
    """Load libw2v_hip.so (raises if it was not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else Path(os.environ.get("W2V_DEV_LIB") or DEV_LIB)
    if not p.exists():
        raise RuntimeError(
            f"word2vec_amd: HIP library {p} is missing; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C word2vec_amd/csrc`"
        )
    lib = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


class DevError(RuntimeError):
    def __init__(self, msg: str, code: int = 0):
        super().__init__(msg)
        self.code = code


def check(lib: C.CDLL, rc: int, what: str) -> None:
    if rc != W2V_OK:
        msg = lib.w2v_dev_last_error().decode(errors="replace")
        raise DevError(f"{what} failed (code {rc}): {msg}", rc)
