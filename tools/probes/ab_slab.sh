# A/B of library builds (LIBS) on the per-GPU slab shape of the N = 2 / 4
# bench (8192 x 2048 rows, one rank) and the 4096^2 N = 1 trajectory
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_slab}
mkdir -p $O
rm -f $O/ab.txt
X="--no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check --steps 4 --warmup 1"
for rep in 1 2; do
for lib in $LIBS; do
  BURG_LIB=finitedifference_amd/$lib timeout -k 10 200 python bench.py --nx 8192 --rows-per-gpu 2048 $X > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
  python -c "import json; d=json.load(open('$O/s.json')); print('$lib 8192x2048', d['value'], d['ms_per_step'], d['engine']['blocked_diagonals'])" >> $O/ab.txt
  BURG_LIB=finitedifference_amd/$lib AB_REPS=3 timeout -k 10 200 python tools/probes/ab4096.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail -5 $O/ab.txt; exit 1; }
done
done
cat $O/ab.txt
