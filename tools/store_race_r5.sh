# Store-data race: with the comm wave at priority 2
# the old build (cp2old) corrupts stored states; the fixed build (cp2) must not.
# Wide and narrow (one-cell and paired) shapes, bitwise against the oracle.
set -o pipefail
O=gpurun_out/storerace; mkdir -p $O
run() {  # lib pair nx ny W T
  BURG_PAIR=$2 BURG_LIB=finitedifference_amd/libburgers_hip_$1.so timeout -k 10 200 python tools/probes/race_probe.py $3 $4 $5 $6 | sed "s/^/{\"lib\": \"$1\", \"pair\": \"$2\", \"r\": /; s/\$/}/" >> $O/race.jsonl 2>> $O/err.log
}
for lib in cp2 cp2old; do
  run $lib 0 4096 64 256 6 || exit 1
  run $lib 0 2048 256 256 4 || exit 1
  run $lib 0 4096 512 512 3 || exit 1
  run $lib 0 1024 256 16 6 || exit 1
  run $lib 1 1024 256 16 6 || exit 1
  run $lib 0 2048 512 16 4 || exit 1
  run $lib 1 2048 512 16 4 || exit 1
done
# the fixed default build's rates (compare: profiles/r05/ab/loaders, narrow/)
for shp in "4096 4096 1" "16384 2048 10" "8192 8192 1" "1024 1024 1"; do
  set -- $shp
  timeout -k 10 150 python tools/probes/traj_rate.py $1 $2 $3 3 >> $O/rates.jsonl 2>> $O/err.log || exit 1
done
timeout -k 10 150 python tools/probes/sweep_rate.py 3 >> $O/rates.jsonl 2>> $O/err.log || exit 1
