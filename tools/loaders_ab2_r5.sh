# two loader waves (default since round 5) vs one (BURG_LOADERS=1 build) on the other wide widths
set -o pipefail
O=gpurun_out/loaders_ab2; mkdir -p $O
V=finitedifference_amd/libburgers_hip_loaders1.so
for r in 1 2; do for v in base l1; do
  if [ $v = l1 ]; then L=$V; else L=finitedifference_amd/libburgers_hip.so; fi
  for shp in "8192 8192 1 0" "8192 2048 1 0" "4096 2048 1 0" "2048 2048 1 64" "2048 1024 1 32" "16384 2048 1 0"; do
    set -- $shp
    TRAJ_W=$4 BURG_LIB=$L timeout -k 10 150 python tools/probes/traj_rate.py $1 $2 $3 2 >> $O/rates.jsonl 2>> $O/err_$v.log || exit 1
  done
done; done
