# comm-priority-2 race: which hand-off kind (W/E via comm only, S/N only)
set -o pipefail
O=gpurun_out/race2; mkdir -p $O
for cfg in "cp2 2048 64 256 6" "cp2 4096 64 256 6" "cp2 1024 512 256 4" "cp2 1024 1024 256 3" "cp2 1024 256 256 4" "cp2 1024 128 256 6"; do
  set -- $cfg
  BURG_LIB=finitedifference_amd/libburgers_hip_$1.so timeout -k 10 200 python tools/probes/race_probe.py $2 $3 $4 $5 | sed "s/^/{\"lib\": \"$1\", \"r\": /; s/\$/}/" >> $O/race.jsonl 2>> $O/err.log || exit 1
done
