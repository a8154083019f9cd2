#!/bin/bash
# 4096^2 A/B of two one-knob variants: ring stores
# non-temporal (BURG_RING_AUX=18: sc1 + nt) and the loader without the
# defensive read-back of its DMA'd rows (BURG_DMA_READBACK=0); the 4096^2
# bitwise tests on each first; 3 interleaved rounds; then an N = 4 rehearsal
# (four slab ranks sharing the GPU: the middle ranks read and write a halo)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab_aux}; mkdir -p $O
for v in rnt nrb; do
  BURG_LIB=$PWD/finitedifference_amd/libburgers_hip_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "4096 or wide_bitwise or slab_wide_tile" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
B4="bench.py --steps 5 --warmup 1 --no-1024 --no-rom --no-cpu-baseline --stencil-nx 0 --no-e2e"
for r in 1 2 3; do for v in base rnt nrb; do
  L=$PWD/finitedifference_amd/libburgers_hip.so; [ $v != base ] && L=$PWD/finitedifference_amd/libburgers_hip_$v.so
  BURG_LIB=$L timeout -k 10 200 python3 $B4 > $O/${v}_r$r.json 2> $O/${v}_r$r.err || { tail -5 $O/${v}_r$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${v}_r$r.json')); print('$v r$r', d['value'], d['roofline']['avg_launch_ms'], d['residual_check']['ok'])"
done; done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29703 bench.py --gpus 4 --rehearse-one-gpu --nx 2048 --rows-per-gpu 256 --stream-w 128 --steps 5 --warmup 1 2> $O/n4.err | grep '^{' > $O/bench_rehearse_n4.json || { tail -5 $O/n4.err; exit 1; }
echo REHEARSE4_OK
