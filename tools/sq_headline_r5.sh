#!/bin/bash
# SQ counters of the 4096^2 headline kernel (final build): where the compute
# waves' cycles go (one pass, 8 SQ counters)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sq_headline
mkdir -p $O
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check > $O/bench.json 2> $O/sq.err || { tail -5 $O/sq.err; exit 1; }
echo SQOK
