set -o pipefail
O=gpurun_out/race4; mkdir -p $O
for cfg in "cp2vgpr 4096 64 256 6" "cp2vgpr 1024 128 128 4" "cp2vgpr 2048 256 256 4" "cp2vgpr 4096 512 256 3" \
           "cp1 4096 64 256 6" "cp1 1024 128 128 4" "cp1 2048 256 256 4" "base 4096 64 256 6" "base 1024 128 128 4"; do
  set -- $cfg
  if [ $1 = base ]; then L=finitedifference_amd/libburgers_hip.so; else L=finitedifference_amd/libburgers_hip_$1.so; fi
  BURG_LIB=$L timeout -k 10 200 python tools/probes/race_probe.py $2 $3 $4 $5 | sed "s/^/{\"lib\": \"$1\", \"r\": /; s/\$/}/" >> $O/race.jsonl 2>> $O/err.log || exit 1
done
