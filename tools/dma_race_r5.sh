# LDS-DMA publish race: the comm wave at priority 2 (cp2*) exposes it; cp2 has
# the loader's read-back before filled[] (the fix), cp2norb has not (control).
# Then the read-back's cost at default priority (base vs norb).
set -o pipefail
O=gpurun_out/dmarace; mkdir -p $O
for cfg in "cp2 1024 128 128 4" "cp2 1024 256 256 4" "cp2 2048 256 256 4" "cp2 4096 512 256 3" "cp2 4096 512 512 3" \
           "cp2norb 1024 128 128 4" "cp2norb 2048 256 256 4"; do
  set -- $cfg
  BURG_LIB=finitedifference_amd/libburgers_hip_$1.so timeout -k 10 200 python tools/probes/race_probe.py $2 $3 $4 $5 | sed "s/^/{\"lib\": \"$1\", \"r\": /; s/\$/}/" >> $O/race.jsonl 2>> $O/err.log || exit 1
done
BURG_LIB=finitedifference_amd/libburgers_hip_cp2.so timeout -k 10 150 python tools/probes/traj_rate.py 4096 4096 1 2 >> $O/rates.jsonl 2>> $O/err.log || exit 1
BURG_LIB=finitedifference_amd/libburgers_hip_cp2.so timeout -k 10 150 python tools/probes/traj_rate.py 16384 2048 10 2 >> $O/rates.jsonl 2>> $O/err.log || exit 1
for r in 1 2; do for v in base norb; do
  if [ $v = base ]; then L=finitedifference_amd/libburgers_hip.so; else L=finitedifference_amd/libburgers_hip_$v.so; fi
  for shp in "4096 4096 1" "16384 2048 10" "8192 8192 1"; do
    set -- $shp
    BURG_LIB=$L timeout -k 10 150 python tools/probes/traj_rate.py $1 $2 $3 3 >> $O/rates.jsonl 2>> $O/err.log || exit 1
  done
done; done
