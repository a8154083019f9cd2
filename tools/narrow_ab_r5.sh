# narrow-kernel hand-off knobs: comm look-ahead (BURG_KLA) and mailbox depth (BURG_PIPE_R)
set -o pipefail
O=gpurun_out/narrow_ab; mkdir -p $O
for r in 1 2; do for v in base kla32 kla8 r16; do
  if [ $v = base ]; then L=finitedifference_amd/libburgers_hip.so; else L=finitedifference_amd/libburgers_hip_$v.so; fi
  BURG_LIB=$L BURG_STREAM_DEBUG=8 timeout -k 10 120 python tools/probes/sweep_rate.py 3 >> $O/rates.jsonl 2>> $O/err_$v.log || exit 1
  BURG_LIB=$L BURG_STREAM_DEBUG=8 timeout -k 10 120 python tools/probes/traj_rate.py 1024 1024 1 3 >> $O/rates.jsonl 2>> $O/err_$v.log || exit 1
done; done
