# Diagnose the NaN seen with the comm wave at priority 2 (a timing-dependent
# race): which builds / shapes produce non-finite or different states.
# Each run is its own process under a time limit; a failing run is recorded
# and the script goes on only if it failed cleanly (library error, rc 1).
set -o pipefail
O=gpurun_out/cp2diag; mkdir -p $O
run() {  # tag lib nx ny
  BURG_LIB=finitedifference_amd/libburgers_hip_$2.so timeout -k 10 150 python tools/probes/traj_rate.py $3 $4 1 2 > $O/$1.json 2> $O/$1.err
  rc=$?
  echo "$1 rc=$rc $(tail -c 300 $O/$1.json)" >> $O/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc $rc"; exit 2; fi
  return 0
}
run cp2_4096 cp2 4096 4096
run cp2l1_4096 cp2l1 4096 4096
run cp2_8192x2048 cp2 8192 2048
run cp2_16384x2048 cp2 16384 2048
run cp2_2048x512 cp2 2048 512
run cp2l1_8192x2048 cp2l1 8192 2048
