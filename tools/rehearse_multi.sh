# Rehearse bench.py's N > 1 path on a one-GPU box: N ranks (torchrun, gloo
# control plane) all on cuda:0 (W2V_BENCH_SHARE_GPU=1). RCCL refuses two ranks
# on one GPU, so each rank runs the native exchange on a ONE-rank group (rank 0
# makes one group id per rank and broadcasts them, as it broadcasts the real
# group's id; every round's delta kernel, ncclAllReduce and fold run) and the
# replicas are combined across the processes by a gloo mean on top
# (replicas.make_averager / RehearsalAverager). Checks the multi-rank code
# path (sharding, rounds at the configs[3] cadence, the group calls, barriers,
# max-over-ranks time; stderr logs the native group's exchange count); the
# numbers are not bench lines.
#   bash tools/rehearse_multi.sh [N] [extra bench args]
N=${1:-2}; shift
W2V_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N --steps 2 --warmup 1 --cpu-seconds 0 "$@"
