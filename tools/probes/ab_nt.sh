set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_nt}
mkdir -p $O
for rep in 1 2; do
for lib in libburgers_hip.so libburgers_hip_nt1.so libburgers_hip_nt3.so libburgers_hip_nt2.so; do
  BURG_LIB=finitedifference_amd/$lib timeout -k 10 200 python tools/probes/ab4096.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail -5 $O/ab.txt; exit 1; }
done
done
cat $O/ab.txt
