set -o pipefail
O=gpurun_out/w512ab; mkdir -p $O
for v in base u8 base u8; do
  if [ $v = u8 ]; then L=finitedifference_amd/libburgers_hip_w512u8.so; else L=finitedifference_amd/libburgers_hip.so; fi
  BURG_LIB=$L BURG_STREAM_DEBUG=8 timeout -k 10 120 python tools/probes/traj_rate.py 16384 2048 10 3 >> $O/rates.jsonl 2>> $O/err_$v.log || exit 1
done
for v in base u8; do
  if [ $v = u8 ]; then L=finitedifference_amd/libburgers_hip_w512u8.so; else L=finitedifference_amd/libburgers_hip.so; fi
  BURG_LIB=$L timeout -k 10 120 python tools/probes/traj_rate.py 4096 4096 1 3 >> $O/rates.jsonl 2>> $O/err_$v.log || exit 1
done
