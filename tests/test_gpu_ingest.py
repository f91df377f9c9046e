"""GPU corpus ingestion (include/w2v_ingest.h) against the
host readers (csrc/host/corpus.cpp), which tests/test_corpus_file.py pins to
the reference's string path (build_vocab(line_docs(path)), Word2Vec.cpp:19-30,
132-169; the CLI's text8 reader, main.cpp:63-92; build_sample, :212-230).
Bit-exact: vocabulary order and counts, token ids, sentence offsets,
train_words — over chunk sizes that cut the file into many pieces, empty
lines, tabs / CR / leading whitespace, an unterminated last line, bytes
>= 0x80, an empty file, and the device-to-device hand-over to a training
handle (w2v_dev_adopt_corpus)."""
import numpy as np
import pytest

from tests.test_corpus_file import _write_corpus

pytestmark = pytest.mark.gpu


def _model(gpu_ingest, chunk=0, min_count=3):
    from word2vec_amd.model import Word2Vec

    return Word2Vec(iter=1, window=5, min_count=min_count, table_size=10_000, word_dim=16, negative=5,
                    subsample_threshold=1e-3, train_method="ns", model="sg", verbose=False,
                    gpu_ingest=gpu_ingest, ingest_chunk_bytes=chunk)


def make_trainer_for(counts):
    """An SG-NS training handle for a vocab with these counts (table_size 10000)."""
    from word2vec_amd.device import Config, DeviceTrainer

    cfg = Config(word_dim=32, window=5, negative=5, hs=False, cbow=False, cbow_mean=True, iter=1, init_alpha=0.025,
                 min_alpha=1e-4, table_size=10_000)
    d = DeviceTrainer(cfg)
    p = counts.astype(np.float64) ** 0.75
    bounds = np.concatenate([[0], np.floor(np.cumsum(p) / p.sum() * 10_000)]).astype(np.int64)
    bounds[-1] = 10_000
    d.upload_vocab(np.ones(counts.size, np.float32), bounds)
    rng = np.random.default_rng(0)
    d.upload_model((rng.random((counts.size, 32), np.float32) - 0.5) / 32, np.zeros((counts.size, 32), np.float32))
    return d


def _host_samples(path, index):
    """build_sample over line_docs (Word2Vec.cpp:19-30, 212-230) on the file's bytes."""
    raw = path.read_bytes()
    lines = raw.split(b"\n")
    if lines and lines[-1] == b"":
        lines = lines[:-1]
    ids, off = [], [0]
    for ln in lines:
        ids.extend(index[t.decode()] for t in ln.split() if t.decode() in index)
        off.append(len(ids))
    return np.array(ids, np.int32), np.array(off, np.int64), sum(len(ln.split()) for ln in lines)


def _both(path, fmt, chunk=0, min_count=3):
    host, gpu = _model(False, min_count=min_count), _model(True, chunk, min_count=min_count)
    host.build_vocab_file(path, fmt, 4)
    gpu.build_vocab_file(path, fmt, 4)
    hw, hc = host.vocab()
    gw, gc = gpu.vocab()
    assert gw == hw
    np.testing.assert_array_equal(gc, hc)
    hs = host.file_samples(path, fmt, 4)
    gs = gpu.file_samples(path, fmt, 4)
    assert gs[2] == hs[2]                       # train_words
    np.testing.assert_array_equal(gs[1], hs[1])  # sentence offsets
    np.testing.assert_array_equal(gs[0], hs[0])  # ids
    return hs


@pytest.mark.parametrize("fmt", ["lines", "text8"])
@pytest.mark.parametrize("trailing_newline", [True, False])
@pytest.mark.parametrize("chunk", [0, 4096, 65_536])
def test_gpu_ingest_matches_host_reader(tmp_path, fmt, trailing_newline, chunk):
    path = tmp_path / "corpus.txt"
    _write_corpus(path, 20_000, seed=7, trailing_newline=trailing_newline)
    ids, off, tw = _both(path, fmt, chunk)
    assert ids.size > 100_000 and off.size > 10


def test_gpu_ingest_odd_bytes_and_blank_runs(tmp_path):
    """Non-ASCII bytes are word bytes (only the C-locale space set splits),
    runs of blank lines are empty sentences, \\v and \\f split tokens."""
    rng = np.random.default_rng(3)
    words = [b"caf\xc3\xa9", b"\xff\xfe", b"na\xefve", b"a", b"bb", b"ccc", b"\x01ctl", b"x" * 300]
    parts = []
    for i in range(30_000):
        k = int(rng.integers(0, 12))
        toks = [words[int(j)] for j in rng.integers(0, len(words), k)]
        seps = [b" ", b"\t", b"\v", b"\f", b"\r", b"  "]
        line = b""
        for t in toks:
            line += t + seps[int(rng.integers(0, len(seps)))]
        parts.append(line)
        if i % 50 == 0:
            parts.extend([b"", b"   ", b"\t"])
    path = tmp_path / "odd.txt"
    path.write_bytes(b"\n".join(parts))
    for fmt in ("lines", "text8"):
        for chunk in (0, 4096):
            _both(path, fmt, chunk, min_count=1)


def test_gpu_ingest_empty_and_whitespace_only(tmp_path):
    for name, data in (("empty.txt", b""), ("ws.txt", b" \n\n\t \n"), ("one.txt", b"word")):
        p = tmp_path / name
        p.write_bytes(data)
        for fmt in ("lines", "text8"):
            _both(p, fmt, min_count=1)


@pytest.mark.parametrize("resident", [-1, 0])
def test_gpu_ingest_python_wrapper_and_adopt(tmp_path, resident):
    """GpuIngest.count() returns the words in order of first occurrence with
    their counts (what the host merge yields); adopt_corpus hands the samples
    to a training handle, which then trains the same words as after
    upload_corpus of the same samples."""
    import torch

    from word2vec_amd.ingest import GpuIngest

    path = tmp_path / "corpus.txt"
    text = _write_corpus(path, 8_000, seed=5)
    first = {}
    for t in text.split():
        first[t] = first.get(t, 0) + 1
    g = GpuIngest(path, "lines", device=0, chunk_bytes=8192, resident_max=resident)
    words = g.count()
    assert [w for w, _ in words] == list(first)        # dict order = first occurrence
    assert [c for _, c in words] == list(first.values())
    vocab = sorted((w for w, c in words if c >= 3), key=lambda w: -first[w])
    index = {w: i for i, w in enumerate(vocab)}
    g.map(index)
    ids, off, tw = g.samples()
    assert tw == len(text.split())
    host_ids, host_off, host_tw = _host_samples(path, index)
    np.testing.assert_array_equal(off, host_off)
    np.testing.assert_array_equal(ids, host_ids)
    assert tw == host_tw

    counts = np.array([first[w] for w in vocab], np.int64)
    ta, tb = make_trainer_for(counts), make_trainer_for(counts)
    ta.adopt_corpus(g)
    tb.upload_corpus(ids, off, tw)
    sa, sb = ta.train_epoch(0), tb.train_epoch(0)
    assert sa["words"] == sb["words"] and sa["sentences"] == sb["sentences"]
    assert ta.policy() == tb.policy()   # the same corpus statistics (token histogram)
    torch.cuda.synchronize()
    g.close()
