# A/B of library builds (LIBS, in finitedifference_amd/) at 1024^2 (sweep +
# one trajectory) and 4096^2, after the WHOLE -m gpu suite on TESTLIB
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_full}
mkdir -p $O
rm -f $O/ab.txt
if [ -n "$TESTLIB" ]; then
  BURG_LIB=finitedifference_amd/$TESTLIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for rep in 1 2; do
for lib in $LIBS; do
  BURG_LIB=finitedifference_amd/$lib timeout -k 10 200 python tools/probes/ab1024.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail -5 $O/ab.txt; exit 1; }
  BURG_LIB=finitedifference_amd/$lib AB_REPS=3 timeout -k 10 200 python tools/probes/ab4096.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail -5 $O/ab.txt; exit 1; }
done
done
cat $O/ab.txt
