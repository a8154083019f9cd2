set -o pipefail
O=gpurun_out/swf; mkdir -p $O
timeout -k 10 120 python tools/probes/sweep_rate.py 2 >> $O/rates.jsonl 2>> $O/err.log || exit 1
BURG_PAIR=0 timeout -k 10 120 python tools/probes/sweep_rate.py 2 >> $O/rates.jsonl 2>> $O/err.log || exit 1
