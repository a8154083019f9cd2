#!/bin/bash
# Round-3 profiles (under gpurun): rocprofv3 kernel stats of the driver's
# bench command, and the HBM (FETCH_SIZE / WRITE_SIZE) and clock
# (GRBM_GUI_ACTIVE) passes -- one counter per run -- of the 4096^2
# trajectory (b4), the 1024^2 9-mu sweep (b1), one 1024^2 trajectory (bs)
# and the LSPG Gram probe (bl).  tools/pmc_to_json.py folds them into
# profiles/pmc_traffic.json.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-prof_r3}
mkdir -p $O
cd $R
if [ -z "$NO_STATS" ]; then
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_stats.json 2> $O/stats.err || { tail -5 $O/stats.err; exit 1; }
echo stats ok
fi
B4="bench.py --steps 3 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check"
B1="bench.py --nx 1024 --dt 0.05 --sweep 9 --steps 3 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check"
BS="bench.py --nx 1024 --dt 0.05 --steps 3 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check"
BL="tools/lspg_probe.py 1024 95 3"
# per-GPU slabs of the N = 2/4 and N = 8 lines, one rank (s8, s16)
S8="bench.py --nx 8192 --rows-per-gpu 2048 --steps 3 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check"
S16="bench.py --nx 16384 --rows-per-gpu 2048 --steps 2 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check"
for name in ${NAMES:-b4 b1 bs bl}; do
  if [ "$name" = pod ]; then
    # where the 250^2 rsvd POD's device time goes (kernel stats only)
    POD_PROBE_RSVD_ONLY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pod_stats -o run -- python3 tools/pod_probe.py > $O/pod_probe.json 2> $O/pod_stats.err || { tail -5 $O/pod_stats.err; exit 1; }
    echo "pod stats ok"
    continue
  fi
  case $name in b4) CMD=$B4;; b1) CMD=$B1;; bs) CMD=$BS;; bl) CMD=$BL;; s8) CMD=$S8;; s16) CMD=$S16;; esac
  if [ "$name" = s8 ] || [ "$name" = s16 ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${name}_stats -o run -- python3 $CMD > $O/${name}_bench.json 2> $O/${name}_stats.err || { tail -5 $O/${name}_stats.err; exit 1; }
    echo "$name stats ok"
  fi
  for ctr in FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $O/${name}_$ctr -o run -- python3 $CMD > /dev/null 2> $O/${name}_$ctr.err || { tail -5 $O/${name}_$ctr.err; exit 1; }
    echo "$name $ctr ok"
  done
done
echo PROFOK
