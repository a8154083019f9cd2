# A/B of narrow-kernel build variants at 1024^2 (tools/probes/ab1024.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_n}
mkdir -p $O
rm -f $O/ab.txt
for rep in 1 2; do
for lib in $LIBS; do
  BURG_LIB=finitedifference_amd/$lib timeout -k 10 200 python tools/probes/ab1024.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail -5 $O/ab.txt; exit 1; }
done
done
cat $O/ab.txt
