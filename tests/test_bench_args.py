"""bench.py's argument handling (CPU only): a BASELINE preset (--config) sets
defaults, and flags given explicitly win over it (DESIGN.md §4.1's per-mode
table runs `--config c3 --mode cbow_hs`)."""
import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _parse(argv, monkeypatch):
    spec = importlib.util.spec_from_file_location("bench_under_test", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
    return mod.parse()


def test_preset_sets_defaults(monkeypatch):
    a = _parse(["--config", "c1"], monkeypatch)
    assert (a.mode, a.dim, a.negative, a.vocab, a.tokens) == ("sg_ns", 100, 5, 350_000, 17_000_000)


def test_explicit_flags_override_preset(monkeypatch):
    a = _parse(["--config", "c3", "--mode", "cbow_hs", "--dim", "200"], monkeypatch)
    assert (a.mode, a.dim, a.vocab, a.tokens) == ("cbow_hs", 200, 1_000_000, 50_000_000)


def test_no_preset_is_the_headline(monkeypatch):
    a = _parse([], monkeypatch)
    assert (a.mode, a.dim, a.negative, a.gpus) == ("sg_ns", 300, 5, 1)


def test_replica_auto_matches_the_class(monkeypatch):
    """bench.py --gpus N exchanges like Word2Vec::replica_mode auto on
    configs[3]'s 10 B / N-token shards (Word2Vec.cpp run_epochs_replicas)."""
    spec = importlib.util.spec_from_file_location("bench_under_test", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert [mod.auto_replica_mode(n) for n in (2, 4, 8)] == ["average", "average", "adaptive"]
    assert mod.auto_replica_mode(2, 200_000_000) == "sum"  # short shards: the sum for two
    assert mod.auto_replica_mode(3, 200_000_000) == "adaptive"
    assert mod.config3_sync_words(8) == 10_000_000_000 // 8 // 128  # the adaptive divisor's cadence
    assert mod.config3_sync_words(4, "average") == 10_000_000_000 // 4 // 64
    hdr = (ROOT / "include" / "Word2Vec.h").read_text()
    assert "kAutoReplicaRounds = 64;" in hdr and "kAutoAverageWords = 4000000;" in hdr
    assert "kAutoAdaptiveRounds = 128;" in hdr
    assert "kAutoAverageReplicas = 4;" in hdr
