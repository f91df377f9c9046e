"""The C++ Word2Vec class (include/Word2Vec.h) on the host: vocabulary
products, weight init and file formats are bit-identical to the reference
restatement; the CLI keeps the reference's flags and validation. CPU only."""
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

from tests.corpus import zipf_sentences
from tests.harness import MODES, oracle_run
from word2vec_amd.model import Word2Vec

ROOT = Path(__file__).resolve().parents[1]
CLI = ROOT / "word2vec_amd" / "bin" / "word2vec"


def make_pair(mode, sents, dim=16, seed=77, ts=50_000, min_count=2, subsample=1e-3):
    m = MODES[mode]
    w = Word2Vec(iter=1, window=5, min_count=min_count, table_size=ts, word_dim=dim, negative=m["negative"],
                 subsample_threshold=subsample, init_alpha=0.05, min_alpha=2.5e-6, cbow_mean=True,
                 train_method=m["train_method"], model=m["model"])
    w.seed(seed)
    w.build_vocab(sents)
    o = oracle_run(sents, mode, dim=dim, table_size=ts, min_count=min_count, subsample=subsample, seed=seed,
                   train=False)
    return w, o


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("seed", [1, 2])
def test_vocab_products_match_oracle(mode, seed):
    sents = zipf_sentences(30, 400, 600, seed=seed, ragged=True)
    w, o = make_pair(mode, sents)
    assert w.vocab()[0] == o.vocab()[0]
    np.testing.assert_array_equal(w.vocab()[1], o.vocab()[1])
    np.testing.assert_array_equal(w.sample_probs().view(np.uint32), o.sample_probs().view(np.uint32))
    if MODES[mode]["negative"]:
        np.testing.assert_array_equal(w.table(), o.table())
    if MODES[mode]["train_method"] == "hs":
        for a, b in zip(w.huffman(), o.huffman()):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("mode", list(MODES))
def test_init_weights_bit_identical(mode):
    sents = zipf_sentences(10, 300, 300, seed=3)
    w, o = make_pair(mode, sents)
    w.init_weights()  # oracle_run already drew one init (main.cpp:190); match it
    w.init_weights()  # ... and the re-init train() does (Word2Vec.cpp:358)
    o.init_weights()
    for k in range(3):
        a, b = w.matrix(k), o.matrix(k)
        assert a.shape == b.shape, (k, a.shape, b.shape)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


def _cpp_g(x: float) -> str:
    # std::ostream << float at the default precision 6 == printf("%g")
    return "%g" % float(np.float32(x))


def test_save_word2vec_text_format(tmp_path):
    sents = zipf_sentences(10, 200, 100, seed=5)
    w, _ = make_pair("sg_ns", sents, dim=7)
    w.init_weights()
    W = w.matrix(0)
    W[0, :3] = [1e-5, -0.5, 123456789.0]
    w.set_matrix(0, W)
    f = tmp_path / "v.txt"
    w.save_word2vec(f, which=0)
    lines = f.read_text().split("\n")
    words, _ = w.vocab()
    assert lines[0] == f"{len(words)} 7"
    for i, word in enumerate(words):  # vocab order, word then space-separated %g coefficients
        assert lines[i + 1] == word + " " + " ".join(_cpp_g(v) for v in W[i])
    assert lines[len(words) + 1] == "" and len(lines) == len(words) + 2
    assert lines[1].split()[1:4] == ["1e-05", "-0.5", "1.23457e+08"]


def test_save_load_binary_roundtrip(tmp_path):
    sents = zipf_sentences(10, 200, 100, seed=6)
    w, _ = make_pair("sg_ns", sents, dim=5)
    w.init_weights()
    W = w.matrix(0)
    f = tmp_path / "v.bin"
    w.save_word2vec(f, which=0, binary=True)
    raw = f.read_bytes()
    r, sp, c, nl = struct.unpack_from("<qcqc", raw, 0)
    assert (r, sp, c, nl) == (W.shape[0], b" ", 5, b"\n")
    pos = 18
    words, _ = w.vocab()
    for i, word in enumerate(words):
        assert raw[pos:pos + len(word) + 1] == word.encode() + b" "
        pos += len(word) + 1
        np.testing.assert_array_equal(np.frombuffer(raw, np.float32, 5, pos), W[i])
        pos += 20
        assert raw[pos:pos + 1] == b"\n"
        pos += 1
    assert pos == len(raw)
    w.set_matrix(0, np.zeros_like(W))
    w.load_word2vec(f, binary=True)
    np.testing.assert_array_equal(w.matrix(0), W)


def test_save_load_text_roundtrip(tmp_path):
    sents = zipf_sentences(10, 200, 100, seed=7)
    w, _ = make_pair("sg_ns", sents, dim=6)
    w.init_weights()
    W = w.matrix(0)
    f = tmp_path / "v.txt"
    w.save_word2vec(f)
    w.set_matrix(0, np.zeros_like(W))
    w.load_word2vec(f)
    np.testing.assert_allclose(w.matrix(0), W, rtol=1e-5, atol=1e-9)  # 6 significant digits


def test_save_read_vocab(tmp_path):
    sents = zipf_sentences(10, 200, 100, seed=8)
    w, _ = make_pair("sg_ns", sents)
    f = tmp_path / "vocab.txt"
    w.save_vocab(f)
    words, counts = w.vocab()
    lines = f.read_text().splitlines()
    assert lines == [f"{i} {c} {t}" for i, (t, c) in enumerate(zip(words, counts))]
    w2 = Word2Vec(word_dim=4)
    w2.read_vocab(f)
    assert w2.vocab()[0] == words
    np.testing.assert_array_equal(w2.vocab()[1], counts)


def test_train_without_gpu_fails_loudly():
    """No silent CPU fallback: without a GPU the device path raises."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    sents = zipf_sentences(5, 100, 50, seed=9)
    w, _ = make_pair("sg_ns", sents)
    with pytest.raises(RuntimeError, match="w2v_dev"):
        w.train(sents)


def _cli(*args, cwd=None):
    return subprocess.run([str(CLI), *args], capture_output=True, text=True, cwd=cwd, timeout=60)


def test_cli_help_and_validation(tmp_path):
    r = _cli()
    assert r.returncode == 0 and "-train_method" in r.stdout and "-negative" in r.stdout
    r = _cli("-model", "sg", "-train_method", "ns")  # ns without -negative (main.cpp:164-168)
    assert r.returncode == 1 and "Please set -negative > 0!" in r.stdout
    r = _cli("-train_method", "hs", "-negative", "5")  # (main.cpp:169-173)
    assert r.returncode == 1 and "Do not set -negative under hierarchical softmax!" in r.stdout
    r = _cli("-train_method", "hs", "-model", "sg-align")
    assert r.returncode == 1 and "aligned skip gram" in r.stdout
    r = _cli("-size")  # ArgPos: flag without a value (main.cpp:50-61)
    assert r.returncode == 1 and "Argument missing for -size" in r.stdout


def test_checkpoint_round_trip(tmp_path):
    """save_checkpoint / load_checkpoint: W, C, synapses1, the
    word counter and the generator state come back bit-identical; a vocab
    mismatch is refused. (Continuing training from it runs on the GPU:
    tests/test_gpu_class.py.)"""
    import pytest

    from tests.corpus import zipf_sentences
    from word2vec_amd.model import Word2Vec

    sents = zipf_sentences(30, 100, 300, seed=3)
    a = Word2Vec(iter=1, window=5, min_count=2, table_size=10_000, word_dim=24, negative=5, train_method="ns",
                 model="sg")
    a.seed(5)
    a.build_vocab(sents)
    a.init_weights()
    W, Cm = a.matrix(0), a.matrix(1)
    a.set_matrix(1, Cm + 0.25)
    a.save_checkpoint(tmp_path / "ck.bin")
    b = Word2Vec(iter=1, window=5, min_count=2, table_size=10_000, word_dim=24, negative=5, train_method="ns",
                 model="sg")
    b.build_vocab(sents)
    b.load_checkpoint(tmp_path / "ck.bin")
    np.testing.assert_array_equal(b.matrix(0), W)
    np.testing.assert_array_equal(b.matrix(1), Cm + 0.25)
    c = Word2Vec(iter=1, window=5, min_count=2, table_size=10_000, word_dim=24, negative=5, train_method="ns",
                 model="sg")
    c.build_vocab(sents[:10])
    with pytest.raises(RuntimeError, match="vocabulary"):
        c.load_checkpoint(tmp_path / "ck.bin")


def test_checkpoint_load_rejects_bad_shapes(tmp_path):
    """load_checkpoint checks every matrix against the object's shapes and
    changes nothing when one is wrong (an NS checkpoint into an HS object)."""
    import pytest as _pytest

    from tests.corpus import zipf_sentences
    from word2vec_amd.model import Word2Vec

    sents = zipf_sentences(20, 100, 200, seed=5)
    ns = Word2Vec(iter=1, window=5, min_count=2, table_size=10_000, word_dim=16, negative=5, train_method="ns",
                  model="sg")
    ns.seed(1)
    ns.build_vocab(sents)
    ns.init_weights()
    ns.save_checkpoint(tmp_path / "ns.bin")
    hs = Word2Vec(iter=1, window=5, min_count=2, table_size=10_000, word_dim=16, negative=5, train_method="hs",
                  model="sg")
    hs.seed(1)
    hs.build_vocab(sents)
    hs.init_weights()
    before = hs.matrix(0)
    with _pytest.raises(RuntimeError, match="checkpoint"):
        hs.load_checkpoint(tmp_path / "ns.bin")
    np.testing.assert_array_equal(hs.matrix(0), before)


def test_checkpoint_version1_loads(tmp_path):
    """a round-2 (version 1) checkpoint — magic W2VCKPT1, then V,
    d, vocab hash, current_words, the generator, the matrices; no schedule
    position — still loads (as a whole-schedule checkpoint); an unknown
    version is named as such, not as a foreign file."""
    import struct

    from tests.corpus import zipf_sentences
    from word2vec_amd.model import Word2Vec

    sents = zipf_sentences(20, 100, 200, seed=4)
    kw = dict(iter=1, window=5, min_count=2, table_size=10_000, word_dim=12, negative=5, train_method="ns", model="sg")
    a = Word2Vec(**kw)
    a.seed(2)
    a.build_vocab(sents)
    a.init_weights()
    a.set_matrix(1, a.matrix(1) + 0.5)
    a.save_checkpoint(tmp_path / "v2.bin")
    raw = (tmp_path / "v2.bin").read_bytes()
    assert raw[:8] == b"W2VCKPT2"
    head = raw[8:32]  # V, d, vocab hash
    cw = raw[32:40]
    q = 8 + 24 + 24 + 8  # past magic, V/d/hash, cw/epochs/iter, key
    gl = struct.unpack("<q", raw[q:q + 8])[0]
    gen = raw[q:q + 8 + gl]
    q += 8 + gl
    gl2 = struct.unpack("<q", raw[q:q + 8])[0]
    mats = raw[q + 8 + gl2:]
    (tmp_path / "v1.bin").write_bytes(b"W2VCKPT1" + head + cw + gen + mats)
    b = Word2Vec(**kw)
    b.build_vocab(sents)
    b.load_checkpoint(tmp_path / "v1.bin")
    np.testing.assert_array_equal(b.matrix(0), a.matrix(0))
    np.testing.assert_array_equal(b.matrix(1), a.matrix(1))
    (tmp_path / "v9.bin").write_bytes(b"W2VCKPT9" + raw[8:])
    with pytest.raises(RuntimeError, match="version"):
        b.load_checkpoint(tmp_path / "v9.bin")


def test_replica_mode_rejected_early():
    """replica_mode outside -1 .. W2V_GROUP_ADAPTIVE (e.g. 4 = SPLIT,
    whose per-row divisors the class does not compute) fails in train() before
    any replica is created (check_limits), naming the member."""
    from tests.corpus import zipf_sentences
    from word2vec_amd.model import Word2Vec

    sents = zipf_sentences(5, 50, 100, seed=1)
    for bad in (4, 5, -2):
        w = Word2Vec(iter=1, window=5, min_count=1, table_size=1000, word_dim=16, negative=5, train_method="ns",
                     model="sg", gpu_devices=[0, 0], replica_mode=bad)
        w.build_vocab(sents)
        with pytest.raises(RuntimeError, match="replica_mode"):
            w.train(sents)


def test_hyperparameter_limits_fail_early():
    """The reference accepts any window / negative / word_dim
    (Word2Vec.cpp:254, 285, 335). The per-pair kernels take negatives past 63
    (drawn 64 at a time) and CBOW windows past 127 (walked from the sentence)
    up to 4096 (both walks are quadratic: round 5 stopped the range where its
    cost was measured) and rows up to 2048 floats (w2v_dev_limits); beyond
    that, and for the shared-negatives tiles (window 8, negative 15, rows of
    <= 1024 floats: w2v_dev_shared_limits), the range is enforced before any
    corpus or device work: the class names the member, the CLI the
    reference's flag."""
    import ctypes as C

    from tests.corpus import zipf_sentences
    from word2vec_amd import _native as N
    from word2vec_amd.model import Word2Vec

    lib = N.load_dev_lib()
    v = [C.c_int32() for _ in range(5)]
    assert lib.w2v_dev_limits(*[C.byref(x) for x in v]) == 0
    assert [x.value for x in v] == [2048, 4096, 4096, 8, 15]
    sv = [C.c_int32() for _ in range(3)]
    assert lib.w2v_dev_shared_limits(*[C.byref(x) for x in sv]) == 0
    assert [x.value for x in sv] == [1024, 8, 15]
    sents = zipf_sentences(5, 50, 100, seed=1)
    for kw, what in ((dict(window=4097), "window"), (dict(negative=4097), "negative"),
                     (dict(word_dim=2049), "word_dim")):
        base = dict(iter=1, window=5, min_count=1, table_size=1000, word_dim=16, negative=5, train_method="ns",
                    model="sg")
        base.update(kw)
        w = Word2Vec(**base)
        w.build_vocab(sents)
        with pytest.raises(RuntimeError, match=what):
            w.train(sents)
    w = Word2Vec(iter=1, window=9, min_count=1, table_size=1000, word_dim=16, negative=5, train_method="ns",
                 model="sg", shared_negatives=True)
    w.build_vocab(sents)
    with pytest.raises(RuntimeError, match="shared_negatives"):
        w.train(sents)
    w = Word2Vec(iter=1, window=5, min_count=1, table_size=1000, word_dim=1100, negative=5, train_method="ns",
                 model="sg", shared_negatives=True)
    w.build_vocab(sents)
    with pytest.raises(RuntimeError, match="shared_negatives.*word_dim <= 1024"):
        w.train(sents)
    r = _cli("-window", "4097", "-negative", "5")
    assert r.returncode == 1 and "Please set -window in [0, 4096]" in r.stdout
    r = _cli("-negative", "4097")
    assert r.returncode == 1 and "Please set -negative <= 4096" in r.stdout
    r = _cli("-size", "1100", "-negative", "5", "-shared-negatives", "1")
    assert r.returncode == 1 and "-size <= 1024" in r.stdout
    r = _cli("-size", "3000", "-negative", "5")
    assert r.returncode == 1 and "Please set -size in [1, 2048]" in r.stdout
    r = _cli("-negative", "16", "-shared-negatives", "1")
    assert r.returncode == 1 and "-shared-negatives 1" in r.stdout


def _compile_caller(src_args, out, cwd):
    """g++ with the reference's own build line (main.cpp:2, minus -march and
    the Eigen path) against include/ and the product libraries."""
    lib = ROOT / "word2vec_amd" / "lib"
    cmd = ["g++", "-std=c++11", "-O2", "-fopenmp", *src_args, "-I", str(ROOT / "include"), "-o", str(out),
           "-L", str(lib), "-lword2vec_amd", "-lw2v_hip", f"-Wl,-rpath,{lib}"]
    return subprocess.run(cmd, capture_output=True, text=True, cwd=cwd, timeout=300)


def test_reference_shaped_caller_compiles(tmp_path):
    """a caller written against the reference's API and
    environment (tests/callers/ref_caller.cpp: Eigen::initParallel,
    omp_set_num_threads, unqualified std names) compiles and links against
    include/Word2Vec.h and the product libraries unmodified (it runs on the
    GPU in tests/test_gpu_class.py)."""
    r = _compile_caller([str(ROOT / "tests" / "callers" / "ref_caller.cpp")], tmp_path / "ref_caller", tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]


def test_reference_caller_compiles(tmp_path):
    """The reference's own main.cpp (read from /root/reference as text, fed to
    the compiler on stdin so its directory's Word2Vec.h is not found) compiles
    and links against include/ unmodified: the drop-in header provides the
    environment it relies on. Container only: the GPU box has
    no /root/reference."""
    src = Path("/root/reference/main.cpp")
    if not src.exists():
        pytest.skip("reference not present (GPU box)")
    lib = ROOT / "word2vec_amd" / "lib"
    cmd = ["g++", "-std=c++11", "-O2", "-fopenmp", "-x", "c++", "-", "-I", str(ROOT / "include"), "-o",
           str(tmp_path / "ref_main"), "-L", str(lib), "-lword2vec_amd", "-lw2v_hip", f"-Wl,-rpath,{lib}"]
    r = subprocess.run(cmd, input=src.read_text(encoding="utf-8-sig"), capture_output=True, text=True,
                       cwd=tmp_path, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
