set -o pipefail
O=gpurun_out/sbs; mkdir -p $O
timeout -k 10 120 python tools/probes/sweep_rate.py 3 >> $O/rates.jsonl 2>> $O/err.log || exit 1
BURG_SWEEP_BATCH=2 timeout -k 10 120 python tools/probes/sweep_rate.py 3 >> $O/rates.jsonl 2>> $O/err.log || exit 1
BURG_SWEEP_BATCH=3 timeout -k 10 120 python tools/probes/sweep_rate.py 3 >> $O/rates.jsonl 2>> $O/err.log || exit 1
