#!/bin/bash
# build the library of a git revision into build/variants/lib_NAME.so (A/B across
# source versions): tools/build_rev.sh REV NAME [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2; shift 2
tmp=$(mktemp -d /tmp/rbe_rev_XXXX)
git archive "$rev" rbe550_final_project_amd/csrc include | tar -x -C "$tmp"
mkdir -p build/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=6 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -Xarch_device -fno-honor-nans -Xarch_device -mno-amdgpu-ieee -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form "$@" \
  -o build/variants/lib_$name.so "$tmp/rbe550_final_project_amd/csrc/rp_lib.hip" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$tmp"
echo build/variants/lib_$name.so
