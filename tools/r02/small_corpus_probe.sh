# Full-concurrency quality vs the wave cap on the paired corpora (text8_small
# is 2,000 sentences: fewer than the chip's resident waves).
set -o pipefail
timeout -k 10 300 python -u tests/probes/quality_paired_probe.py text8_small sg_ns,cbow_hs 1 0,2048,1024,512,256 - || exit 1
timeout -k 10 300 python -u tests/probes/quality_paired_probe.py planted sg_ns,cbow_hs 1,2 0,1024,512,256 - || exit 1
timeout -k 10 300 python -u tests/probes/quality_paired_probe.py text8_like sg_ns,cbow_hs 1 0,2048,1024 - || exit 1
