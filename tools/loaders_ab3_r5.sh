# four loader waves (one per compute wave) vs two (default)
set -o pipefail
O=gpurun_out/loaders_ab3; mkdir -p $O
V=finitedifference_amd/libburgers_hip_loaders4.so
BURG_LIB=$V timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_regime.py -k "planted_bitwise or 4096_bench or capped or rank_shape" \
  > $O/pytest_loaders4.log 2>&1 || { tail -30 $O/pytest_loaders4.log; exit 1; }
for r in 1 2; do for v in base l4; do
  if [ $v = l4 ]; then L=$V; else L=finitedifference_amd/libburgers_hip.so; fi
  for shp in "16384 2048 10" "4096 4096 1" "8192 8192 1" "8192 2048 1"; do
    set -- $shp
    BURG_LIB=$L BURG_STREAM_DEBUG=8 timeout -k 10 150 python tools/probes/traj_rate.py $1 $2 $3 3 >> $O/rates.jsonl 2>> $O/err_$v.log || exit 1
  done
done; done
