set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_final4
mkdir -p $O
cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_stats.json 2> $O/stats.err || { tail -5 $O/stats.err; exit 1; }
echo STATSOK
