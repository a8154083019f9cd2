set -o pipefail
O=gpurun_out/race3; mkdir -p $O
for cfg in "cp2drain 4096 64 256 6" "cp2drain 1024 128 128 4" "cp2drain 2048 256 256 4" "cp2 4096 64 256 6" "cp2 4096 64 256 6"; do
  set -- $cfg
  BURG_LIB=finitedifference_amd/libburgers_hip_$1.so timeout -k 10 200 python tools/probes/race_probe.py $2 $3 $4 $5 | sed "s/^/{\"lib\": \"$1\", \"r\": /; s/\$/}/" >> $O/race.jsonl 2>> $O/err.log || exit 1
done
