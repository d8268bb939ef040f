#!/bin/bash
# Build variant librsl copies with rsl_doa_toep.hip compiled under extra -D flags (build container; the GPU box only
# loads them through RSL_LIBRARY).   tools/doa_libvar.sh NAME "-DFOO=0 -DBAR=1"  ->  radar-slam_amd/lib/librsl_NAME.so
set -e
cd "$(dirname "$0")/../radar-slam_amd/csrc"
make -j8 >/dev/null
mkdir -p /tmp/rsl_var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-value \
  -Wno-pass-failed -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form=1 $2 -c rsl_doa_toep.hip -o /tmp/rsl_var/toep_$1.o
objs=$(ls ../build/*.o | grep -v rsl_doa_toep.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../lib/librsl_$1.so $objs /tmp/rsl_var/toep_$1.o
echo built ../lib/librsl_$1.so
