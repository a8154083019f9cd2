set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_u}
mkdir -p $O
rm -f $O/ab.txt
BURG_LIB=finitedifference_amd/libburgers_hip_u16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regime.py -x -q --timeout 200 --timeout-method thread -k "pipe and not 4096 or sweep or slow_path or chunked or slab_halo" > $O/pytest_u8.log 2>&1 || { tail -30 $O/pytest_u8.log; exit 1; }
tail -2 $O/pytest_u8.log
for rep in 1 2; do
for lib in libburgers_hip.so libburgers_hip_u16.so libburgers_hip_u16k32.so; do
  BURG_LIB=finitedifference_amd/$lib timeout -k 10 200 python tools/probes/ab1024.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail -5 $O/ab.txt; exit 1; }
done
done
cat $O/ab.txt
