# A/B of library builds at 1024^2 (sweep + one trajectory) and 4096^2; the
# pipe parity tests on TESTLIB first (if given)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_both}
mkdir -p $O
rm -f $O/ab.txt
if [ -n "$TESTLIB" ]; then
  BURG_LIB=finitedifference_amd/$TESTLIB timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regime.py -x -q --timeout 200 --timeout-method thread -k "pipe or sweep or slow_path or chunked or slab or 4096" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for rep in 1 2; do
for lib in $LIBS; do
  BURG_LIB=finitedifference_amd/$lib timeout -k 10 200 python tools/probes/ab1024.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail -5 $O/ab.txt; exit 1; }
  BURG_LIB=finitedifference_amd/$lib AB_REPS=3 timeout -k 10 200 python tools/probes/ab4096.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail -5 $O/ab.txt; exit 1; }
done
done
cat $O/ab.txt
