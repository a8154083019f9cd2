# A/B of narrow-kernel builds at 1024^2 (tools/probes/ab1024.py); the pipe /
# sweep / slow-path / slab GPU tests first, on the in-tree library
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_u}
mkdir -p $O
rm -f $O/ab.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regime.py -x -q --timeout 200 --timeout-method thread -k "pipe and not 4096 or sweep or slow_path or chunked or slab_halo" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for lib in $LIBS; do
  BURG_LIB=finitedifference_amd/$lib timeout -k 10 200 python tools/probes/ab1024.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail -5 $O/ab.txt; exit 1; }
done
done
cat $O/ab.txt
