# nearest-node threshold seeds per range: 8 (in-tree) vs 32 / 128 (abvariants/lib_s32,
# lib_s128): C5 covered-well plans (tools/well_ab.py, NN time; same plans), two
# interleaved rounds; exact-path counts (tools/nn_count.py, -DRP_NN_COUNT builds)
set -o pipefail
rm -f gpurun_out/ab_seeds.log
for r in 1 2; do
  for lib in rbe550_final_project_amd/librbe_mi355x.so abvariants/lib_s32.so abvariants/lib_s128.so; do
    echo "== $lib" >> gpurun_out/ab_seeds.log
    RBE_LIB_PATH=$lib timeout -k 10 300 python tools/well_ab.py dense=RBE_EDGE_PACKED:0 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_seeds.log || exit 1
  done
done
for lib in abvariants/lib_c8.so abvariants/lib_c128.so; do
  echo "== $lib" >> gpurun_out/ab_seeds.log
  timeout -k 10 300 python tools/nn_count.py $lib 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_seeds.log || exit 1
done
