# comm-wave priority on the fixed build: 0 (default) / 1 / 2
set -o pipefail
O=gpurun_out/commprio2; mkdir -p $O
for r in 1 2; do for v in base cp1 cp2; do
  if [ $v = base ]; then L=finitedifference_amd/libburgers_hip.so; else L=finitedifference_amd/libburgers_hip_$v.so; fi
  BURG_LIB=$L timeout -k 10 150 python tools/probes/traj_rate.py 4096 4096 1 3 >> $O/rates.jsonl 2>> $O/err.log || exit 1
  BURG_LIB=$L timeout -k 10 150 python tools/probes/traj_rate.py 16384 2048 10 3 >> $O/rates.jsonl 2>> $O/err.log || exit 1
  BURG_LIB=$L timeout -k 10 150 python tools/probes/sweep_rate.py 3 >> $O/rates.jsonl 2>> $O/err.log || exit 1
  BURG_LIB=$L timeout -k 10 150 python tools/probes/traj_rate.py 1024 1024 1 3 >> $O/rates.jsonl 2>> $O/err.log || exit 1
done; done
