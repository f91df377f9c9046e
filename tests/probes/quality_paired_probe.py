"""GPU probe for the paired quality gates (tests/paired.py): per corpus /
mode / seed, the GPU scores at one wavefront and at full concurrency next to
the oracle's paired golden, with wall times. Run on the GPU box:
python tests/probes/quality_paired_probe.py [corpus] [modes,...] [seeds,...] [max_waves,...] [policy;policy;...]
where a policy is "k=v,k=v" over tests/paired.train_gpu_paired's policy keys
(hot_rows, private_rows, flush_centers, private_average, context_rows,
context_flush); "-" = the default policy."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from tests import paired  # noqa: E402
from word2vec_amd.evaluate import analogy_accuracy, similarity_score  # noqa: E402


def parse_policy(p):
    if p in ("", "-"):
        return {}
    out = {}
    for kv in p.split(","):
        k, v = kv.split("=")
        out[k] = float(v) if k in ("private_average", "hot_tau_rows", "hot_tau_nodes", "private_rate") else int(v)
    return out


def main(name="text8_like", modes="sg_ns,cbow_hs", seeds="1", waves="1,0", policies="-"):
    gold = json.loads((ROOT / "tests" / "golden" / "quality_paired_oracle.json").read_text())
    sents, qs, pairs = paired.corpus(name)
    for mode in modes.split(","):
        for seed in [int(s) for s in seeds.split(",")]:
            ref = [r for r in gold[name][mode] if r["seed"] == seed][0]
            for mw, pol in [(int(w), p) for w in waves.split(",") for p in policies.split(";")]:
                t = time.time()
                words, E = paired.train_gpu_paired(name, mode, seed, sents, max_waves=mw, policy=parse_policy(pol))
                dt = time.time() - t
                a = analogy_accuracy(words, E, qs)["accuracy"]
                s = similarity_score(words, E, pairs)["spearman"]
                print(json.dumps({"corpus": name, "mode": mode, "seed": seed, "max_waves": mw, "policy": pol,
                                  "secs": round(dt, 1),
                                  "analogy": round(a, 2), "similarity": round(s, 2),
                                  "d_analogy": round(a - ref["analogy"], 2),
                                  "d_similarity": round(s - ref["similarity"], 2)}), flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
