"""The C-ABI libraries load on a CPU-only host and export exactly what the
public headers declare (no compute calls: there is no GPU here)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "word2vec_amd" / "lib"


def declared(header: Path):
    txt = re.sub(r"/\*.*?\*/", "", header.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(w2v_[a-z0-9_]+)\s*\(", txt)))


@pytest.mark.parametrize("header,lib", [("w2v_dev.h", "libw2v_hip.so"), ("w2v_ingest.h", "libw2v_hip.so"),
                                        ("w2v_host.h", "libword2vec_amd.so")])
def test_library_exports_every_declared_symbol(header, lib):
    names = declared(ROOT / "include" / header)
    assert len(names) >= 4
    so = ctypes.CDLL(str(LIB / lib))
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    from word2vec_amd import _native

    names = sorted(set(declared(ROOT / "include" / "w2v_dev.h")) | set(declared(ROOT / "include" / "w2v_ingest.h")))
    assert sorted(_native.SIGNATURES) == names
    lib = _native.load_dev_lib()
    assert lib.w2v_dev_version().decode().startswith("word2vec_amd")


def test_dev_lib_fails_loudly_when_missing(tmp_path):
    from word2vec_amd import _native

    with pytest.raises(RuntimeError, match="missing"):
        _native.load_dev_lib(tmp_path / "nope.so")


def test_create_rejects_bad_configs_without_gpu():
    """Argument validation runs before any HIP call, so it is testable here."""
    from word2vec_amd import _native as N

    lib = N.load_dev_lib()
    h = ctypes.c_void_p()
    for bad in (dict(word_dim=0), dict(window=40), dict(negative=64), dict(hs=0, negative=0), dict(word_dim=2048)):
        kw = dict(word_dim=100, window=5, negative=5, hs=0, cbow=0, cbow_mean=0, iter=1, init_alpha=0.025,
                  min_alpha=1e-4, table_size=1000, device=0, reserved=0)
        kw.update(bad)
        cfg = N.DevConfig(**kw)
        assert lib.w2v_dev_create(ctypes.byref(cfg), ctypes.byref(h)) != 0
        assert lib.w2v_dev_last_error()


def test_ingest_rejects_bad_arguments_without_gpu():
    from word2vec_amd import _native as N

    lib = N.load_dev_lib()
    g = ctypes.c_void_p()
    assert lib.w2v_ingest_create(0, 7, 0, ctypes.byref(g)) != 0  # bad format
    assert b"format" in lib.w2v_dev_last_error()
    assert lib.w2v_ingest_create(0, 0, -1, ctypes.byref(g)) != 0
    assert lib.w2v_ingest_count(None, None, 0) != 0
    assert lib.w2v_ingest_summary(None, None, None, None) != 0
    assert lib.w2v_dev_adopt_corpus(None, None) != 0
