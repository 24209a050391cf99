#!/bin/bash
# builds the standalone A/B harnesses (diagnostic tools) with the library's flags
cd "$(dirname "$0")/../.."
F="--offload-arch=gfx950 -mcode-object-version=6 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -Xarch_device -fno-honor-nans -Xarch_device -mno-amdgpu-ieee -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form"
for t in "$@"; do
  case $t in
    val_stats) /opt/rocm/bin/hipcc $F -DRP_PAIR_STATS -o tools/lab/val_stats tools/val_lab.hip -ldl || exit 1 ;;
    *) /opt/rocm/bin/hipcc $F -o tools/lab/$t tools/$t.hip -ldl || exit 1 ;;
  esac
done
