#!/bin/bash
# Round-6 profiles of the final build: rocprofv3 kernel stats of the default
# bench command, and the FETCH_SIZE / WRITE_SIZE / GRBM_GUI_ACTIVE passes
# (one counter per run) of the 4096^2 trajectory (b4), the 1024^2 9-mu sweep
# (b1) and one 1024^2 trajectory (bs) -- tools/prof_r3.sh; then the SQ pass
# of the single 1024^2 trajectory (issue vs wait).
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-prof_r6} NAMES="b4 b1 bs" bash tools/prof_r3.sh || exit 1
O=gpurun_out/${TAG:-prof_r6}
BS="bench.py --nx 1024 --dt 0.05 --steps 3 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e --no-residual-check"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU --output-format csv -d $O/bs_SQ -o run -- python3 $BS > /dev/null 2> $O/bs_sq.err || { tail -5 $O/bs_sq.err; exit 1; }
echo "bs SQ ok"
