#!/bin/bash
# A/B of the store wave (BURG_STORE_WAVE=1, libburgers_hip_sw.so) for the
# one-cell W = 16 kernels: the narrow bitwise tests on
# the variant, then interleaved timing of one 1024^2 x 500 trajectory
# (bench.single_1024) and of the 9-mu sweep on the one-cell kernel
# (BURG_PAIR=0), base vs sw, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_sw}; mkdir -p $O
BURG_LIB=$PWD/finitedifference_amd/libburgers_hip_sw.so timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "pipe_1024 or pipe_bitwise_sequential or sweep_each or retained or slab_halo_two or sweep_1024 or run_fom_main or direct_npy" > $O/pytest_sw.log 2>&1 || { tail -30 $O/pytest_sw.log; exit 1; }
tail -1 $O/pytest_sw.log
for r in 1 2 3; do for v in base sw; do
  L=$PWD/finitedifference_amd/libburgers_hip.so; [ $v = sw ] && L=$PWD/finitedifference_amd/libburgers_hip_sw.so
  BURG_LIB=$L timeout -k 10 300 python3 -c "
import json, bench
s = bench.single_1024(bench.os.path.join(bench.ROOT, 'profiles', 'pmc_traffic.json'), bench.os.path.join(bench.ROOT, 'profiles', 'r05', 'pipe_isa.json'))
print(json.dumps({'v': '$v', 'r': $r, 'single_ms': s['avg_launch_ms'], 'single_value': s['value'], 'ramp_ms': s['ramp_ms']}))
" >> $O/ab.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
  BURG_PAIR=0 BURG_LIB=$L timeout -k 10 300 python3 -c "
import json, bench
c = bench.config2_1024(None)
print(json.dumps({'v': '$v', 'r': $r, 'sweep_onecell_ms': c['avg_launch_ms'], 'sweep_onecell_value': c['value']}))
" >> $O/ab.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done; done
cat $O/ab.jsonl
echo ABOK
