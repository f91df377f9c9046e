"""The host side of the boundary under AddressSanitizer + UndefinedBehaviorSanitizer
(the reference is racy and UB-prone by design; the rebuild's
host code is checked): word2vec_amd/csrc/check/host_selftest.cpp builds the
vocabulary, Huffman paths, unigram table, sampling, weights, corpus readers
and vector / vocab files, and drives the C bridge's argument checks, with no
device call (make -C word2vec_amd/csrc asan)."""
import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
BIN = ROOT / "word2vec_amd" / "bin" / "host_selftest_asan"


def test_host_code_clean_under_asan_ubsan(tmp_path):
    subprocess.run(["make", "-s", "-C", str(ROOT / "word2vec_amd" / "csrc"), "asan"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(BIN), str(tmp_path)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failure(s)" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
