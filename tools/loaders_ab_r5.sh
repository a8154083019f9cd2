# two loader waves per wide workgroup (BURG_LOADERS=2) vs one: parity subset, then rates
set -o pipefail
O=gpurun_out/loaders_ab; mkdir -p $O
V=finitedifference_amd/libburgers_hip_loaders2.so
BURG_LIB=$V timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_regime.py tests/test_gpu_retained.py \
  -k "planted_bitwise or large_h or 4096_bench or chunked or capped or rank_shape or workgroup_order or snap_every or retained" \
  > $O/pytest_loaders2.log 2>&1 || { tail -30 $O/pytest_loaders2.log; exit 1; }
for r in 1 2; do for v in base l2; do
  if [ $v = l2 ]; then L=$V; else L=finitedifference_amd/libburgers_hip.so; fi
  BURG_LIB=$L BURG_STREAM_DEBUG=8 timeout -k 10 120 python tools/probes/traj_rate.py 16384 2048 10 3 >> $O/rates.jsonl 2>> $O/err_$v.log || exit 1
  BURG_LIB=$L BURG_STREAM_DEBUG=8 timeout -k 10 120 python tools/probes/traj_rate.py 4096 4096 1 3 >> $O/rates.jsonl 2>> $O/err_$v.log || exit 1
done; done
