# Signed paired deltas (GPU - oracle golden, same init / keys / orders) for
# every gated mode, one wave and full concurrency, default policy.
set -o pipefail
timeout -k 10 300 python -u tests/probes/quality_paired_probe.py planted sg_ns,sg_hs,cbow_ns,cbow_hs 1,2,3 1,0 - || exit 1
timeout -k 10 300 python -u tests/probes/quality_paired_probe.py text8_like sg_ns,cbow_hs 1,2,3 0 - || exit 1
timeout -k 10 300 python -u tests/probes/quality_paired_probe.py text8_small sg_ns,cbow_hs 1 1,0 - || exit 1
