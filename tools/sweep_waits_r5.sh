set -o pipefail
O=gpurun_out/swaits; mkdir -p $O
BURG_STREAM_DEBUG=8 timeout -k 10 120 python tools/probes/sweep_rate.py 2 >> $O/rates.jsonl 2>> $O/err_pair.log || exit 1
BURG_PAIR=0 BURG_STREAM_DEBUG=8 timeout -k 10 120 python tools/probes/sweep_rate.py 2 >> $O/rates.jsonl 2>> $O/err_one.log || exit 1
BURG_STREAM_DEBUG=8 timeout -k 10 120 python tools/probes/traj_rate.py 1024 1024 1 2 >> $O/rates.jsonl 2>> $O/err_traj.log || exit 1
