cd $GRAFT_REPO_ROOT
X="--steps 5 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e"
for v in maxilp def maxilp def; do
  if [ $v = def ]; then export BURG_LIB=$GRAFT_REPO_ROOT/finitedifference_amd/libburgers_hip_def.so; else unset BURG_LIB; fi
  a=$(timeout -k 10 120 python bench.py $X --nx 1024 --dt 0.05 --sweep 9 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['roofline']['avg_launch_ms'])")
  b=$(timeout -k 10 120 python bench.py $X 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['roofline']['avg_launch_ms'])")
  echo "$v sweep1024: $a  traj4096: $b"
done
