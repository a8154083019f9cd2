set -o pipefail
O=gpurun_out/race8; mkdir -p $O
RACE_SAVE=$O/r4096x64.npz BURG_LIB=finitedifference_amd/libburgers_hip_cp2.so timeout -k 10 200 python tools/probes/race_probe.py 4096 64 256 6 >> $O/race.jsonl 2>> $O/err.log || exit 1
RACE_SAVE=$O/r1024x128.npz BURG_LIB=finitedifference_amd/libburgers_hip_cp2.so timeout -k 10 200 python tools/probes/race_probe.py 1024 128 128 4 >> $O/race.jsonl 2>> $O/err.log || exit 1
