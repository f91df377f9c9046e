"""Streaming corpus ingestion (Word2Vec::build_vocab_file / file_samples,
word2vec_amd/csrc/host/corpus.cpp) against the string path the reference
takes: build_vocab(line_docs(path)) (Word2Vec.cpp:19-30, 132-169) and the
reference CLI's text8 reader (main.cpp:63-92) + build_sample (:212-230).
Host only (no GPU): vocabulary order and counts must be identical, and so
must the token ids, sentence offsets and train_words."""
import numpy as np
import pytest

from tests.corpus import zipf_ids
from word2vec_amd.model import Word2Vec


def _model(min_count=3):
    return Word2Vec(iter=1, window=5, min_count=min_count, table_size=10_000, word_dim=16, negative=5,
                    subsample_threshold=1e-3, train_method="ns", model="sg", verbose=False)


def _write_corpus(path, n_lines, seed, trailing_newline=True):
    rng = np.random.default_rng(seed)
    ids = zipf_ids(n_lines * 40, 5000, seed=seed)
    lines, k = [], 0
    for i in range(n_lines):
        n = int(rng.integers(0, 80))
        toks = [f"w{r}" for r in ids[k:k + n]]
        k += n
        if i % 97 == 5:
            toks = []                     # an empty sentence
        sep = "\t" if i % 13 == 0 else " "
        line = sep.join(toks)
        if i % 17 == 3:
            line = "  " + line + " \r"   # leading / trailing whitespace, CR
        lines.append(line)
    text = "\n".join(lines) + ("\n" if trailing_newline else "")
    path.write_text(text)
    return text


def line_docs(text):
    """Word2Vec.cpp:19-30 (getline, then whitespace tokens)."""
    parts = text.split("\n")
    if parts and parts[-1] == "":
        parts = parts[:-1]
    return [p.split() for p in parts]


def text8_docs(text):
    """main.cpp:63-92: whitespace tokens in 1000-token sentences."""
    toks = text.split()
    return [toks[i:i + 1000] for i in range(0, len(toks), 1000)]


def _expected_samples(sents, words):
    index = {w: i for i, w in enumerate(words)}
    ids, off = [], [0]
    for s in sents:
        ids.extend(index[t] for t in s if t in index)
        off.append(len(ids))
    return np.array(ids, np.int32), np.array(off, np.int64), sum(len(s) for s in sents)


@pytest.mark.parametrize("fmt", ["lines", "text8"])
@pytest.mark.parametrize("threads", [1, 4])
@pytest.mark.parametrize("trailing_newline", [True, False])
def test_file_vocab_and_samples_match_string_path(tmp_path, fmt, threads, trailing_newline):
    path = tmp_path / "corpus.txt"
    text = _write_corpus(path, 60_000 if threads > 1 else 3_000, seed=7, trailing_newline=trailing_newline)
    sents = line_docs(text) if fmt == "lines" else text8_docs(text)

    ref = _model()
    ref.build_vocab(sents)
    ref_words, ref_counts = ref.vocab()

    m = _model()
    m.build_vocab_file(path, fmt, threads)
    words, counts = m.vocab()
    assert words == ref_words
    np.testing.assert_array_equal(counts, ref_counts)

    ids, off, tw = m.file_samples(path, fmt, threads)
    eids, eoff, etw = _expected_samples(sents, words)
    assert tw == etw
    np.testing.assert_array_equal(off, eoff)
    np.testing.assert_array_equal(ids, eids)


def test_file_threads_do_not_change_anything(tmp_path):
    path = tmp_path / "corpus.txt"
    _write_corpus(path, 80_000, seed=11)
    out = []
    for threads in (1, 3, 8):
        m = _model()
        m.build_vocab_file(path, "lines", threads)
        out.append((m.vocab()[0], *m.file_samples(path, "lines", threads)))
    for o in out[1:]:
        assert o[0] == out[0][0]
        np.testing.assert_array_equal(o[1], out[0][1])
        np.testing.assert_array_equal(o[2], out[0][2])
        assert o[3] == out[0][3]


def test_empty_and_missing_files(tmp_path):
    empty = tmp_path / "empty.txt"
    empty.write_text("")
    m = _model()
    m.build_vocab_file(empty, "lines", 2)
    assert m.vocab()[0] == []
    ids, off, tw = m.file_samples(empty, "text8", 2)
    assert ids.size == 0 and off.tolist() == [0] and tw == 0
    with pytest.raises(RuntimeError, match="cannot open"):
        m.build_vocab_file(tmp_path / "nope.txt")
    with pytest.raises(RuntimeError, match="format"):
        m.build_vocab_file(empty, "csv")
