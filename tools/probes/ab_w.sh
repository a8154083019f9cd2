# A/B of wide-kernel build variants at 4096^2 (tools/probes/ab4096.py) + the
# wide parity tests on the variant
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_w}
mkdir -p $O
rm -f $O/ab.txt
if [ -n "$TESTLIB" ]; then
BURG_LIB=finitedifference_amd/$TESTLIB timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regime.py -x -q --timeout 300 --timeout-method thread -k "wide or 4096 or chunked or slow_path or steady" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
fi
for rep in 1 2; do
for lib in $LIBS; do
  BURG_LIB=finitedifference_amd/$lib timeout -k 10 200 python tools/probes/ab4096.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail -5 $O/ab.txt; exit 1; }
done
done
cat $O/ab.txt
