# Workgroup order A/B (BURG_WG_MAP unset = the planner's choice, 0 row-major,
# 1 column-major) on the per-GPU slab shapes of the N = 2/4 and N = 8 bench,
# 4096^2 and the 1024^2 narrow kernels (sweep + one trajectory)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_order}
mkdir -p $O
rm -f $O/ab.txt
X="--no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check --steps 4 --warmup 1"
for rep in 1 2; do
for m in ${MAPS:-auto 0 1}; do
  if [ $m = auto ]; then unset BURG_WG_MAP; else export BURG_WG_MAP=$m; fi
  for nx in 8192 16384; do
    timeout -k 10 200 python bench.py --nx $nx --rows-per-gpu 2048 $X > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
    python -c "import json; d=json.load(open('$O/s.json')); print('map $m ${nx}x2048', d['value'], d['ms_per_step'], d['engine']['blocked_diagonals'])" >> $O/ab.txt
  done
  AB_REPS=3 timeout -k 10 200 python tools/probes/ab4096.py 2>&1 | grep -v amdgpu.ids | sed "s/^/map $m /" >> $O/ab.txt || exit 1
  timeout -k 10 200 python tools/probes/ab1024.py 2>&1 | grep -v amdgpu.ids | sed "s/^/map $m /" >> $O/ab.txt || exit 1
done
done
cat $O/ab.txt
