# rocprofv3 stats + FETCH/WRITE passes for every preset (tag $1), then the N=2
# bench path rehearsed on the one GPU (2 ranks on cuda:0, gloo; not a bench line).
# usage (GPU box): bash tools/gpu_profile_rehearsal.sh <tag>
set -o pipefail
TAG=${1:-r01m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
bash "$R/tools/profile_all.sh" $TAG || exit 1
cd "$R"
W2V_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --tokens 10000000 > gpurun_out/rehearsal_n2.json 2> gpurun_out/rehearsal_n2.err || { tail -20 gpurun_out/rehearsal_n2.err; exit 1; }
cat gpurun_out/rehearsal_n2.json
