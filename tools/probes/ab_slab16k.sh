# A/B of library builds (LIBS) on the N = 8 per-GPU slab (16384 x 2048, W = 512)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab_slab16k}
mkdir -p $O
rm -f $O/ab.txt
X="--no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check --steps 3 --warmup 1"
for rep in 1 2; do
for lib in $LIBS; do
  BURG_LIB=finitedifference_amd/$lib timeout -k 10 200 python bench.py --nx 16384 --rows-per-gpu 2048 $X > $O/s.json 2> $O/s.err || { tail -5 $O/s.err; exit 1; }
  python -c "import json; d=json.load(open('$O/s.json')); print('$lib 16384x2048', d['value'], d['ms_per_step'], d['engine']['blocked_diagonals'])" >> $O/ab.txt
done
done
cat $O/ab.txt
