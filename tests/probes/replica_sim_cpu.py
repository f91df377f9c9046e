"""CPU simulation of data-parallel replica exchange with the sequential oracle per
replica (test infrastructure: the oracle is the checker). For DESIGN.md §6 and
profiles/r02_replica_sim_cpu.log.
usage: python tests/probes/replica_sim_cpu.py <corpus> <mode> <R> <rounds> <sum|avg|rowavg|capS> [warm_fraction]"""
import sys; sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parents[2]))
import numpy as np
from tests import paired
from word2vec_amd.evaluate import analogy_accuracy, similarity_score
name, mode, R, rounds, how = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
warm = float(sys.argv[6]) if len(sys.argv) > 6 else 0.0
import os
_lr = float(os.environ.get("W2V_SIM_LR_SCALE", "1"))
if _lr != 1.0:  # linear learning-rate scaling with R (large-batch SGD's rule), for the avg exchange
    _params = paired.params
    paired.params = lambda *a, **k: dict(_params(*a, **k), init_alpha=_params(*a, **k)["init_alpha"] * _lr)
sents, qs, pairs = paired.corpus(name)
o, orders, key, p = paired.setup(name, mode, 1, sents)
ids, off = o.samples()
n = off.size - 1
order = orders[:n]
words, _ = o.vocab()
mats = [0, 1] if mode.endswith("ns") or mode.startswith("cbow") else [0]
if mode.endswith("hs"): mats = mats + [2]
P = {k: o.matrix(k).copy() for k in mats}
glob = 0
tw = o.train_words
if warm > 0:  # replica 0 alone trains the first `warm` fraction, then the rest is sharded
    nw = int(n * warm)
    wl = order[:nw]
    sub_ids = np.concatenate([ids[off[s]:off[s + 1]] for s in wl])
    sub_off = np.concatenate([[0], np.cumsum([off[s + 1] - off[s] for s in wl])])
    for k in mats: o.set_matrix(k, P[k])
    o.set_samples(sub_ids, sub_off, tw)
    o.train_philox(0, 1, np.arange(len(wl)), key + 999, 0)
    for k in mats: P[k] = o.matrix(k).copy()
    glob = int(sub_off[-1])
    order = order[nw:]
    n = len(order)
shards = [order[n * i // R:n * (i + 1) // R] for i in range(R)]
if how.startswith("sat"):  # sat<beta>: smooth saturation-corrected sum (w2v_group SATURATION)
    from word2vec_amd import host as _host
    _, cnt = o.vocab()
    f = cnt / cnt.sum()
    keep = np.minimum(1.0, _host.sample_probs(cnt, 1e-4).astype(np.float64))
    fk = f * keep
    qk = fk.sum()
    u_tab = cnt ** 0.75 / (cnt ** 0.75).sum()
    rate = {0: fk, 1: qk * 6.0 * (f + 5 * u_tab)}  # SG-NS per raw token (window 5: win1 = 6 on average... )
    beta0 = float(how[4:] if how.startswith("satd") else how[3:])
    tok_round = tw / R / rounds

    def divisors(beta):
        out = {}
        for k in mats:
            u = rate[k] * tok_round
            a = -np.expm1(u * np.log1p(-beta))
            b = -np.expm1(R * u * np.log1p(-beta))
            out[k] = np.where(b > 0, R * a / np.maximum(b, 1e-300), 1.0)
        return out
    WCS = divisors(beta0)
for r in range(rounds):
    D = {k: np.zeros_like(P[k]) for k in mats}
    touched = {k: np.zeros(P[k].shape[0]) for k in mats}
    sq = {k: np.zeros(P[k].shape[0]) for k in mats}
    for i in range(R):
        sh = shards[i]
        sl = sh[len(sh) * r // rounds: len(sh) * (r + 1) // rounds]
        if len(sl) == 0:
            continue
        # corpus = the slice's sentences (ids relabelled 0..m-1)
        sub_ids = np.concatenate([ids[off[s]:off[s + 1]] for s in sl])
        sub_off = np.concatenate([[0], np.cumsum([off[s + 1] - off[s] for s in sl])])
        for k in mats: o.set_matrix(k, P[k])
        o.set_samples(sub_ids, sub_off, max(1, tw // R))
        o.train_philox(0, 1, np.arange(len(sl)), key + 1000 * i + r, glob // R)
        for k in mats:
            d = o.matrix(k) - P[k]
            D[k] += d
            touched[k] += (np.abs(d).max(1) > 0)
            sq[k] += (d.astype(np.float64) ** 2).sum(1)
    if how.startswith("satd"):  # beta follows the learning rate (linear decay, as alpha)
        WCS = divisors(max(beta0 * (1.0 - glob / tw), beta0 * 1e-4))
    for k in mats:
        if how == "sum": P[k] = P[k] + D[k]
        elif how == "avg": P[k] = P[k] + D[k] / R
        elif how.startswith("sat"): P[k] = P[k] + D[k] / WCS[k][:, None].astype(np.float32)
        elif how == "adapt":  # w2v_group ADAPTIVE: c = max(1, |sum D|^2 / sum |D|^2) per row
            coh = (D[k].astype(np.float64) ** 2).sum(1) / np.maximum(sq[k], 1e-30)
            P[k] = P[k] + D[k] / np.maximum(1.0, coh)[:, None].astype(np.float32)
        elif how.startswith("cap"):  # scale 1 / max(1, c / S) with S = int(how[3:])
            S = float(how[3:])
            P[k] = P[k] + D[k] / np.maximum(1, touched[k] / S)[:, None]
        else: P[k] = P[k] + D[k] / np.maximum(1, touched[k])[:, None]
    glob += sum(int(off[s + 1] - off[s]) for sh in shards for s in sh[len(sh) * r // rounds: len(sh) * (r + 1) // rounds])
E = P[1 if mode == "cbow_hs" else 0]
print(name, mode, R, rounds, how + (f"_lr{_lr:g}" if _lr != 1.0 else ""), warm, round(analogy_accuracy(words, E, qs)["accuracy"], 2), round(similarity_score(words, E, pairs)["spearman"], 2), flush=True)
