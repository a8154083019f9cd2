# chunked-run snapshot parity probe (tools/probes/chunk_probe.py) over wide and
# narrow tilings; then the bench-regime test file
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-chunkp}
mkdir -p $O
rm -f $O/out.txt
for a in "700 200 256 11 4 1" "2048 512 256 40 15 1" "2100 64 1024 12 5 1" "1000 130 128 13 3 1" "1024 1024 16 40 7 1" "4096 4096 256 500 0 100 0"; do
  timeout -k 10 200 python tools/probes/chunk_probe.py $a >> $O/out.txt 2>&1 || { echo FAIL $a; tail -5 $O/out.txt; exit 1; }
done
grep -v amdgpu.ids $O/out.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_regime.py -x -v --timeout 300 --timeout-method thread > $O/pytest_regime.log 2>&1 || { tail -40 $O/pytest_regime.log; exit 1; }
tail -25 $O/pytest_regime.log
