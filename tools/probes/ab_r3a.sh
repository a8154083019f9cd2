# A/B of the mailbox granule stride (16 B packed vs 128 B, round 2) + the
# chain probe + the pipe parity tests on the packed build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_r3a}
mkdir -p $O
timeout -k 10 120 tools/probes/chain_probe > $O/chain.txt 2>&1 || { cat $O/chain.txt; exit 1; }
cat $O/chain.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "pipe or slab or sweep or fine750" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for lib in finitedifference_amd/libburgers_hip.so finitedifference_amd/libburgers_hip_g128.so; do
  BURG_LIB=$lib timeout -k 10 200 python tools/probes/ab_bench.py >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
done
done
cat $O/ab.txt
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/b4_FETCH_SIZE -o run -- python3 bench.py --steps 3 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check > /dev/null 2> $O/fetch.err || { tail -5 $O/fetch.err; exit 1; }
echo ABOK
