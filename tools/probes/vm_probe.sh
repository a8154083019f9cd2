set -o pipefail
# (record of a round-3 probe: the libburgers_hip_vm3*.so variants were built with tools/probes/build_variant.sh and a -DBURG_DONE_VM=3 knob since removed -- store waits were 0.1 % of the loop)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/vm
for lib in libburgers_hip_prof.so libburgers_hip_vm3prof.so; do for shp in "4096 4096" "8192 2048"; do
 echo "== $lib $shp" >> gpurun_out/vm/why.txt
 BURG_LIB=finitedifference_amd/$lib BURG_STREAM_DEBUG=8 timeout -k 10 120 python tools/probes/why_probe.py $shp >> gpurun_out/vm/why.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids gpurun_out/vm/why.txt | grep -v "^\[stream\] launch" | tail -40
TAG=vm LIBS="libburgers_hip.so libburgers_hip_vm3.so" bash tools/probes/ab_slab.sh
