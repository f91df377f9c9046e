"""Debug: one replayed sentence (sg_ns, d200) on the library named by
W2V_DEV_LIB; saves the trained W / C to OUT.npz with the oracle's."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from tests.corpus import zipf_sentences  # noqa: E402
from tests.test_gpu_parity import _run_replay  # noqa: E402

sents = zipf_sentences(1, 48, 400, seed=3)
got, want, init = _run_replay("sg_ns", sents, dim=200, window=5, iters=1, table_size=10_000, min_count=1)
np.savez(sys.argv[1], W=got[0], C=got[1], Wo=want[0], Co=want[1], W0=init[0], C0=init[1])
