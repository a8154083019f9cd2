# burg_run_npy writer pool A/B (run_fom.main's timed region at 1024^2 x 500)
set -o pipefail
O=gpurun_out/npy_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "npy" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
for cfg in "1 0" "4 0" "8 0" "4 1" "1 1"; do
  set -- $cfg
  BURG_NPY_WRITERS=$1 BURG_NPY_FSYNC=$2 timeout -k 10 120 python tools/probes/npy_rate.py 3 >> $O/rates.jsonl 2>> $O/err.log || exit 1
done
