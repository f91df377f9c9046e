"""Pin the oracle's shared-negatives minibatch skip-gram (w2v_oracle.cpp:
sgsn_sentence, BASELINE configs[4]) against an independent numpy restatement
(float64 GEMMs, Python Philox from tests/refpy.py) on a few sentences. The
formulation has no reference counterpart (it is pWord2Vec's: windows over the
tokens subsampling keeps), so this restatement plus the reference's own pieces
it keeps (subsampling draw, window shrink, NS sigmoid and label arithmetic,
Word2Vec.cpp:251-271, 319-353) is what pins it."""
import numpy as np
import pytest

from oracle import Oracle
from tests import refpy
from tests.corpus import zipf_sentences

KEY = (0x9ABCDEF0, 0x12345678)


def numpy_sgsn(W, C, keep, table, ids, off, order, window, K, alpha, ts):
    W = W.astype(np.float64)
    C = C.astype(np.float64)
    for s in order:
        sent = ids[off[s]:off[s + 1]]
        kept = []  # (id, position, window shrink) of the tokens subsampling keeps
        for i, c in enumerate(sent):
            t0, t1, _, _ = refpy.philox4x32_10((i, int(s), 0xFFFFFFFF, 0), KEY)
            if keep[c] < refpy.canonical_float(t0):
                continue
            kept.append((int(c), i, (t1 * max(window, 1)) >> 32))
        n = len(kept)
        for t, (c, i, rw) in enumerate(kept):
            lo, hi = max(0, t - window + rw), min(n, t + window + 1 - rw)
            ins, mult = [], []
            for j in range(lo, hi):
                if j == t:
                    continue
                if kept[j][0] in ins:
                    mult[ins.index(kept[j][0])] += 1
                else:
                    ins.append(kept[j][0])
                    mult.append(1)
            if not ins:
                continue
            outs, lab = [int(c)], [1.0]
            for k in range(K):
                o0, o1, _, _ = refpy.philox4x32_10((i, int(s), k, 0), KEY)
                w = int(table[((o1 << 32 | o0) * ts) >> 64])
                if w not in outs:
                    outs.append(w)
                    lab.append(0.0)
            Wi, Co = W[ins], C[outs]
            L = Wi @ Co.T
            E = np.array(mult, np.float64)[:, None] * (np.array(lab)[None, :] - 1 / (1 + np.exp(-L))) * alpha
            W[ins] += E @ Co  # ins are unique, so fancy-index += is exact
            C[outs] += E.T @ Wi
    return W, C


@pytest.mark.parametrize("window,K,dim", [(5, 15, 16), (8, 15, 24), (2, 3, 8)])
def test_oracle_shared_negatives_matches_numpy(window, K, dim):
    sents = zipf_sentences(6, 120, 60, seed=31, ragged=True)
    ts, alpha = 20_000, 0.05
    o = Oracle(iter=1, window=window, min_count=1, table_size=ts, word_dim=dim, negative=K,
               subsample_threshold=1e-2, init_alpha=alpha, min_alpha=1e-4, train_method="ns", model="sg")
    o.load_sentences(sents)
    o.seed(3)
    o.build_vocab()
    o.init_weights()
    o.build_sample()
    rng = np.random.default_rng(2)
    o.set_matrix(1, ((rng.random((o.V, dim)) - 0.5) / dim).astype(np.float32))
    o.set_shared_negatives(True)
    W0, C0 = o.matrix(0), o.matrix(1)
    ids, off = o.samples()
    order = np.arange(off.size - 1)[::-1].copy()  # <= 10 sentences: alpha stays init_alpha
    o.train_philox(0, 1, order, KEY[0] | (KEY[1] << 32), 0)
    Wn, Cn = numpy_sgsn(W0, C0, o.sample_probs(), o.table(), ids, off, order, window, K, alpha, ts)
    for got, want, init in ((o.matrix(0), Wn, W0), (o.matrix(1), Cn, C0)):
        dw = want - init
        assert np.abs(dw).max() > 0
        err = np.abs((got - init) - dw).max() / np.abs(dw).max()
        print(f"rel err {err:.2e}")
        assert err < 1e-5
