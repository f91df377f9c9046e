# Build a timing-only experiment variant of the device library under
# word2vec_amd/lib/<tag>/ (run here, on the CPU; the .so travels with gpurun):
#   tools/r02/exp_variant.sh <tag> "<extra hipcc flags>" [NV list, default "4 5"]
# Only the per-pair kernels of the listed row widths are recompiled with the
# flags; every other object is the product build's. Use with W2V_DEV_LIB.
set -euo pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
tag=$1; flags=$2; nvs=${3:-"4 5"}
C=$R/word2vec_amd/csrc; L=$R/word2vec_amd/lib; D=$L/$tag
DEV=${DEVDIR:-$C/device}  # DEVDIR: another copy of csrc/device (e.g. an earlier commit's, for A/B runs)
mkdir -p "$D/obj"
cp "$L"/obj/w2v_*.o "$D/obj/"
pids=()
for n in $nvs; do  # a row width, or "shared" for the shared-negatives kernel
  if [ "$n" = shared ]; then src=w2v_shared.hip; obj=w2v_shared.o; def=; else src=w2v_inst.hip; obj=w2v_inst_nv$n.o; def="-DW2V_NV=$n -mllvm -amdgpu-atomic-optimizer-strategy=None"; fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall $flags \
    -I"$R/include" -I"$DEV" -I"$C/host" $def -c -o "$D/obj/$obj" "$DEV/$src" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$D/libw2v_hip.so" "$D"/obj/*.o -L/opt/rocm/lib -lrccl \
  -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
g++ -std=c++11 -O2 -fPIC -ffp-contract=off -Wall -pthread -I"$R/include" -I"$C/device" -I"$C/host" -shared \
  -o "$D/libword2vec_amd.so" "$C"/host/vocab_products.cpp "$C"/host/Word2Vec.cpp "$C"/host/model_c_api.cpp \
  "$C"/host/corpus.cpp -L"$D" -lw2v_hip -Wl,-rpath,'$ORIGIN'
rm -rf "$D/obj"
echo "built $D"
