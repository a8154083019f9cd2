#!/bin/bash
# A library variant for A/B runs: pipe.hip and pipe_narrow.hip rebuilt with
# extra defines, linked with the other objects of the default build.
#   tools/probes/build_variant.sh NAME "-DBURG_X=1 ..."  ->  finitedifference_amd/libburgers_hip_NAME.so
set -e
cd "$(dirname "$0")/../../finitedifference_amd/csrc"
make -s
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result -Wno-bitwise-instead-of-logical"
$H -mllvm -amdgpu-sched-strategy=max-ilp $2 -c pipe.hip -o build/pipe_$1.o
# (the narrow unit too, with the same defines)
$H -mllvm -amdgpu-sched-strategy=max-ilp $2 -c pipe_narrow.hip -o build/pipenarrow_$1.o
OBJS=$(ls build/*.o | grep -v -e 'build/pipe.o' -e 'build/pipe_narrow.o' -e '_prof.o' -e 'build/pipe_.*\.o' -e 'build/pipenarrow_.*\.o')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../libburgers_hip_$1.so build/pipe_$1.o build/pipenarrow_$1.o $(echo $OBJS | tr ' ' '\n' | sort -u) \
  -L/opt/rocm/lib -lrocsolver -lrocblas -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo built ../libburgers_hip_$1.so
