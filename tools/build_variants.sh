#!/bin/bash
# build librbe variants into abvariants/ : name:flags pairs
set -e
cd "$(dirname "$0")/.."
mkdir -p abvariants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=6 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -Xarch_device -fno-honor-nans -Xarch_device -mno-amdgpu-ieee -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form $flags \
    -o abvariants/lib_$name.so rbe550_final_project_amd/csrc/rp_lib.hip -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &
done
wait
ls abvariants
