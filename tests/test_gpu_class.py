"""The C++ Word2Vec class end to end on the GPU against the oracle: train()
in replay mode (the reference's own mt19937 draws), the per-call methods
train_sentence_*, negative_sampling, hierarchical_softmax, and the CLI."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

from tests.corpus import zipf_sentences
from tests.harness import MODES, check_parity, oracle_run
from word2vec_amd.model import Word2Vec

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _pair(mode, sents, dim=32, iters=2, seed=5, replay=True, ts=50_000):
    m = MODES[mode]
    w = Word2Vec(iter=iters, window=5, min_count=2, table_size=ts, word_dim=dim, negative=m["negative"],
                 subsample_threshold=1e-3, init_alpha=0.05, min_alpha=2.5e-6, cbow_mean=True,
                 train_method=m["train_method"], model=m["model"], replay_rng=replay)
    w.seed(seed)
    w.build_vocab(sents)
    w.init_weights()
    return w


@pytest.mark.parametrize("mode", list(MODES))
def test_class_train_replay_matches_oracle(mode):
    sents = zipf_sentences(10, 150, 300, seed=12, ragged=True)
    w = _pair(mode, sents)
    w.train(sents)
    o = oracle_run(sents, mode, dim=32, iters=2, table_size=50_000, seed=5)
    got, want, init = [], [], []
    for k in range(3):
        if o.matrix(k).size == 0:
            continue
        assert w.matrix(k).shape == o.matrix(k).shape
        got.append(w.matrix(k))
        want.append(o.matrix(k))
        init.append(o.matrix(k, True))
    check_parity(got, want, init, 2e-5, 2e-3, tag=f"class train {mode}")


@pytest.mark.parametrize("mode", list(MODES))
def test_class_train_sentence_matches_oracle(mode):
    sents = zipf_sentences(6, 120, 200, seed=13)
    w = _pair(mode, sents, iters=1)
    o = oracle_run(sents, mode, dim=32, iters=1, table_size=50_000, seed=5, train=False)
    o.build_sample()
    ids, off = o.samples()
    cbow = MODES[mode]["model"] == "cbow"
    init = [o.matrix(k) for k in range(3)]
    for s in range(3):
        sent = ids[off[s]:off[s + 1]]
        w.train_sentence(sent, 0.03, cbow)
        o.train_sentence(sent, 0.03, cbow)
    ks = [k for k in range(3) if o.matrix(k).size]
    check_parity([w.matrix(k) for k in ks], [o.matrix(k) for k in ks], [init[k] for k in ks], 1e-5, 2e-3,
                 tag=f"class train_sentence {mode}")


def test_class_negative_sampling_and_hs_match_oracle():
    sents = zipf_sentences(6, 200, 150, seed=14)
    for mode in ("sg_ns", "sg_hs"):
        w = _pair(mode, sents, iters=1)
        o = oracle_run(sents, mode, dim=32, iters=1, table_size=50_000, seed=5, train=False)
        rng = np.random.default_rng(1)
        # give the output matrices content so the updates are non-trivial
        k_out = 1 if mode == "sg_ns" else 2
        M = rng.standard_normal(o.matrix(k_out).shape).astype(np.float32) * 0.1
        w.set_matrix(k_out, M)
        o.set_matrix(k_out, M)
        for word in (0, 3, 17):
            x = rng.standard_normal(32).astype(np.float32) * 0.1
            g0 = rng.standard_normal(32).astype(np.float32) * 0.01
            if mode == "sg_ns":
                gw = w.negative_sampling(word, x, g0, 1, 0.025)
                go = o.negative_sampling(word, x, g0, 1, 0.025)
            else:
                gw = w.hierarchical_softmax(word, x, g0, 0.025)
                go = o.hierarchical_softmax(word, x, g0, 0.025)
            check_parity([gw], [go], [g0], 1e-5, 2e-3, tag=f"{mode} grad word {word}")
        check_parity([w.matrix(k_out)], [o.matrix(k_out)], [M], 1e-5, 2e-3, tag=f"{mode} rows")


@pytest.mark.parametrize("mode", list(MODES))
def test_class_train_parallel_philox(mode):
    sents = zipf_sentences(300, 500, 3000, seed=15, ragged=True)
    w = _pair(mode, sents, dim=100, replay=False, ts=1_000_000)
    before = [w.matrix(k).copy() for k in range(3)]
    w.train(sents)
    for k in range(3):
        m = w.matrix(k)
        assert np.isfinite(m).all()
    moved = [np.abs(w.matrix(k) - before[k]).max() for k in range(3) if before[k].size]
    assert max(moved) > 0


def test_cli_end_to_end(tmp_path):
    sents = zipf_sentences(50, 1000, 2000, seed=16)
    corpus = tmp_path / "corpus.txt"
    corpus.write_text(" ".join(" ".join(s) for s in sents))
    out = tmp_path / "vec.txt"
    vocab = tmp_path / "vocab.txt"
    r = subprocess.run([str(ROOT / "word2vec_amd" / "bin" / "word2vec"), "-train", str(corpus), "-output", str(out),
                        "-size", "64", "-negative", "5", "-iter", "2", "-save-vocab", str(vocab)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = out.read_text().splitlines()
    V, d = map(int, lines[0].split())
    assert d == 64 and len(lines) == V + 1 == len(vocab.read_text().splitlines()) + 1
    vals = np.array([float(x) for x in lines[1].split()[1:]])
    assert vals.size == 64 and np.isfinite(vals).all()


def test_cli_gpu_ingest_identical(tmp_path):
    """The CLI with -gpu-ingest 1 (vocab count and id mapping on the GPU)
    writes the same vocab file and the same words in the same order as with the
    host readers (the CLI seeds its generator from std::random_device, as the
    reference does, so the vectors themselves differ from run to run)."""
    sents = zipf_sentences(30, 1000, 2000, seed=18)
    corpus = tmp_path / "corpus.txt"
    corpus.write_text(" ".join(" ".join(s) for s in sents))
    outs = []
    for gi in ("0", "1"):
        out, vocab = tmp_path / f"vec{gi}.txt", tmp_path / f"vocab{gi}.txt"
        r = subprocess.run([str(ROOT / "word2vec_amd" / "bin" / "word2vec"), "-train", str(corpus), "-output", str(out),
                            "-size", "32", "-negative", "5", "-iter", "1", "-replay", "1", "-save-vocab", str(vocab),
                            "-gpu-ingest", gi], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        outs.append((vocab.read_text(), out.read_text()))
    assert outs[0][0] == outs[1][0]
    w0 = [l.split()[0] for l in outs[0][1].splitlines()[1:]]
    w1 = [l.split()[0] for l in outs[1][1].splitlines()[1:]]
    assert w0 == w1 and outs[0][1].splitlines()[0] == outs[1][1].splitlines()[0]


@pytest.mark.parametrize("gpu_ingest", [False, True])
@pytest.mark.parametrize("mode", ["sg_ns", "cbow_hs"])
def test_class_train_file_equals_train(tmp_path, mode, gpu_ingest):
    """train_file (mapped corpus, threaded tokenisation) trains exactly what
    train(line_docs(path)) does: replay mode is deterministic, so the matrices
    must be identical."""
    sents = zipf_sentences(20, 150, 300, seed=17, ragged=True)
    path = tmp_path / "c.txt"
    path.write_text("\n".join(" ".join(s) for s in sents) + "\n")
    a = _pair(mode, sents, iters=1)
    a.train(sents)
    m = MODES[mode]
    b = Word2Vec(iter=1, window=5, min_count=2, table_size=50_000, word_dim=32, negative=m["negative"],
                 subsample_threshold=1e-3, init_alpha=0.05, min_alpha=2.5e-6, cbow_mean=True,
                 train_method=m["train_method"], model=m["model"], replay_rng=True, gpu_ingest=gpu_ingest)
    b.seed(5)
    b.build_vocab_file(path, "lines", 2)
    b.init_weights()
    b.train_file(path, "lines", 2)
    assert a.vocab()[0] == b.vocab()[0]
    for k in range(3):
        np.testing.assert_array_equal(a.matrix(k), b.matrix(k))


def test_checkpoint_resume_continues(tmp_path):
    """A checkpoint written after epoch 1 of an iter-2 schedule (checkpoint_path)
    resumes THAT schedule: a new object that loads it and trains runs only epoch
    2, with the saved word counter (alpha continues from where it was), key and
    shuffle stream, and ends bit-identical to the uninterrupted run (one
    wavefront, so the schedule is deterministic). A checkpoint of the whole
    schedule starts a new one on the loaded weights (counter from 0, alpha from
    init_alpha, as every train() of the reference, Word2Vec.cpp:359): the
    weights move by a full epoch's amount, not by min_alpha's."""
    sents = zipf_sentences(40, 150, 300, seed=17)
    kw = dict(iter=2, window=5, min_count=2, table_size=50_000, word_dim=32, negative=5, subsample_threshold=1e-3,
              init_alpha=0.025, min_alpha=2.5e-6, cbow_mean=True, train_method="ns", model="sg", max_waves=1)
    a = Word2Vec(**kw, checkpoint_path=str(tmp_path / "ck.%d"))
    a.seed(3)
    a.build_vocab(sents)
    a.init_weights()
    W0 = a.matrix(0)
    a.train(sents)
    assert a.epochs_done == 2
    words_2 = a.current_words
    W2 = a.matrix(0)
    assert (tmp_path / "ck.1").exists() and (tmp_path / "ck.2").exists()
    # mid-schedule: continue
    b = Word2Vec(**kw)
    b.build_vocab(sents)
    b.load_checkpoint(tmp_path / "ck.1")
    W1 = b.matrix(0)
    assert 0 < b.current_words < words_2 and b.epochs_done == 1
    b.train(sents)
    assert b.epochs_done == 2 and b.current_words == words_2
    np.testing.assert_array_equal(b.matrix(0), W2)
    np.testing.assert_array_equal(b.matrix(1), a.matrix(1))
    # whole schedule: a new schedule on the loaded weights
    c = Word2Vec(**kw)
    c.build_vocab(sents)
    c.load_checkpoint(tmp_path / "ck.2")
    np.testing.assert_array_equal(c.matrix(0), W2)
    c.train(sents)
    assert c.current_words == words_2  # counted from 0 again
    step_new = np.abs(c.matrix(0) - W2).mean()
    step_first = np.abs(W1 - W0).mean()
    assert np.isfinite(c.matrix(0)).all()
    assert step_new > 0.25 * step_first, (step_new, step_first)


@pytest.mark.parametrize("model,method", [("sg", "ns"), ("cbow", "hs")])
def test_reference_shaped_caller_trains(tmp_path, model, method):
    """tests/callers/ref_caller.cpp — the reference CLI's
    call sequence and environment, written against the reference API only —
    built here against include/Word2Vec.h and run on the GPU: it writes the
    reference's vocab file (index count text) and vector file ("rows cols"
    header, one word and its d values per line, W or C by mode as
    main.cpp:196-201) for the corpus's vocabulary, with finite trained values."""
    from tests.test_class_host import _compile_caller

    exe = tmp_path / "ref_caller"
    r = _compile_caller([str(Path(__file__).parent / "callers" / "ref_caller.cpp")], exe, tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    sents = zipf_sentences(40, 150, 400, seed=61, ragged=True)
    corpus = tmp_path / "corpus.txt"
    corpus.write_text("\n".join(" ".join(s) for s in sents) + "\n")
    r = subprocess.run([str(exe), str(corpus), str(tmp_path / "vec.txt"), str(tmp_path / "vocab.txt"), model, method],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    w = Word2Vec(iter=1, window=5, min_count=2, table_size=100000, word_dim=32, negative=5 if method == "ns" else 0,
                 subsample_threshold=1e-3, init_alpha=0.05, min_alpha=2.5e-6, cbow_mean=True, train_method=method,
                 model=model)
    w.build_vocab(sents)
    words, counts = w.vocab()
    assert (tmp_path / "vocab.txt").read_text().splitlines() == [f"{i} {c} {t}" for i, (t, c) in
                                                                 enumerate(zip(words, counts))]
    lines = (tmp_path / "vec.txt").read_text().splitlines()
    assert lines[0] == f"{len(words)} 32"
    assert [ln.split()[0] for ln in lines[1:]] == words
    vals = np.array([[float(x) for x in ln.split()[1:]] for ln in lines[1:]])
    assert vals.shape == (len(words), 32) and np.isfinite(vals).all() and np.abs(vals).max() > 0
