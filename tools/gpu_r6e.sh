#!/bin/bash
# Round-6 final-build evidence: rocprofv3 stats + PMC passes (tools/prof_r6.sh),
# smoke, the default bench line, the N = 8 per-GPU slab line and the N = 2
# rehearsal (tools/gpu_r6.sh without the suite)
set -o pipefail
export TMPDIR=/tmp
TAG=prof_r6 bash tools/prof_r6.sh || exit 1
echo PROF_OK
SKIP_SUITE=1 TAG=r6e bash tools/gpu_r6.sh || exit 1
O=gpurun_out/r6e
timeout -k 10 300 python bench.py --nx 16384 --rows-per-gpu 2048 --snap-every 10 --steps 3 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e > $O/slab_16384x2048.json 2> $O/slab.err || { tail -20 $O/slab.err; exit 1; }
echo SLAB_OK
