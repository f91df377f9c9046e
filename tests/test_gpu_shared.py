"""GPU parity of the shared-negatives minibatch skip-gram (BASELINE configs[4],
W2V_UPDATE_SHARED_NEGATIVES) against its sequential CPU restatement
(oracle/w2v_oracle.cpp:sgsn_sentence), through the C-ABI.

Both sides draw from the same Philox streams, so every subsampling decision,
window shrink and shared negative is identical; the difference left is fp32
summation order (MFMA 16x16x4 chains + a 4-wave partial sum vs the oracle's
sequential sums). Tolerance: the north star's 1e-5 relative for a single
deterministic update (one sentence); 1e-4 over a multi-sentence epoch, where
rounding differences compound through repeated rows.
"""
import numpy as np
import pytest

from oracle import Oracle
from tests.corpus import zipf_sentences
from tests.harness import check_parity, device_from_oracle
from word2vec_amd import _native as N
from word2vec_amd.device import Config

pytestmark = pytest.mark.gpu

KEY = 0x0DDC_0FFE_E0DD_F00D


def _setup(sents, dim, window=5, negative=15, table_size=100_000, subsample=1e-3, alpha=0.05):
    o = Oracle(iter=1, window=window, min_count=2, table_size=table_size, word_dim=dim, negative=negative,
               subsample_threshold=subsample, init_alpha=alpha, min_alpha=2.5e-6, cbow_mean=True,
               train_method="ns", model="sg")
    o.load_sentences(sents)
    o.seed(1234)
    o.build_vocab()
    o.init_weights()
    o.build_sample()
    # C starts at zero in the reference (init_weights); give it small random rows
    # so the first update exercises every GEMM term (L != 0, dW != 0).
    rng = np.random.default_rng(5)
    o.set_matrix(1, ((rng.random((o.V, dim)) - 0.5) / dim).astype(np.float32))
    o.set_shared_negatives(True)
    cfg = Config(word_dim=dim, window=window, negative=negative, hs=False, cbow=False, cbow_mean=True, iter=1,
                 init_alpha=alpha, min_alpha=2.5e-6, table_size=table_size)
    d = device_from_oracle(o, cfg, initial=False)
    d.set_update(N.W2V_UPDATE_SHARED_NEGATIVES)
    d.set_rng(N.W2V_RNG_PHILOX, KEY)
    d.set_schedule(N.W2V_SCHED_SEQUENTIAL)
    d.set_progress(0)
    return o, d


def _compare(o, d, order, tol, elem_tol, tag):
    init = [o.matrix(0), o.matrix(1)]
    o.train_philox(0, 1, order, KEY, 0)
    st = d.train_epoch(0, order)
    assert st["words"] == o.current_words
    W, Cm, _ = d.download_model()
    for k in (0, 1):
        assert np.abs(o.matrix(k) - init[k]).max() > 0, k
    check_parity([W, Cm], [o.matrix(0), o.matrix(1)], init, tol, elem_tol, tag=tag)
    return st


@pytest.mark.parametrize("dim", [64, 300, 512])
def test_shared_single_sentence(dim):
    sents = zipf_sentences(1, 160, 80, seed=21)
    o, d = _setup(sents, dim)
    st = _compare(o, d, np.arange(1), 1e-5, 5e-3, f"shared single d{dim}")
    assert st["centers"] > 0 and st["targets"] > st["centers"]
    d.close()


@pytest.mark.parametrize("window,negative", [(5, 15), (8, 15), (3, 5), (1, 1)])
def test_shared_epoch(window, negative):
    sents = zipf_sentences(12, 200, 300, seed=23, ragged=True)
    o, d = _setup(sents, 128, window=window, negative=negative)
    n = o.samples()[1].size - 1
    _compare(o, d, np.random.default_rng(1).permutation(n), 1e-4, 5e-3, f"shared epoch w{window} neg{negative}")
    d.close()


def test_shared_parallel_runs_and_counts():
    sents = zipf_sentences(300, 300, 3000, seed=25, ragged=True)
    o, d = _setup(sents, 512, table_size=1_000_000, subsample=1e-4)
    d.set_schedule(N.W2V_SCHED_PARALLEL)
    st = d.train_epoch(0, None)
    ids, off = o.samples()
    assert st["words"] == ids.size
    assert st["sentences"] == off.size - 1
    assert st["draws"] == 15 * st["centers"]  # every center with a context draws 15
    W, Cm, _ = d.download_model()
    assert np.isfinite(W).all() and np.isfinite(Cm).all()
    d.close()


def test_shared_rejects_unsupported():
    from word2vec_amd.device import DeviceTrainer

    for kw in (dict(hs=True, negative=0), dict(cbow=True), dict(negative=16), dict(window=9)):
        base = dict(word_dim=64, window=5, negative=5, hs=False, cbow=False, iter=1, table_size=10_000)
        base.update(kw)
        d = DeviceTrainer(Config(**base))
        with pytest.raises(N.DevError, match="shared negatives"):
            d.set_update(N.W2V_UPDATE_SHARED_NEGATIVES)
        d.close()
