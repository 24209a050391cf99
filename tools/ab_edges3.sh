# loop-free k_edges at 5 waves/SIMD (in-tree) vs 4 (abvariants/lib_ew4.so): C5
# covered-well plans (all large edge launches through k_edges, and the default),
# C4 configured-batch plans, goal3 RRT plans; two interleaved rounds
set -o pipefail
rm -f gpurun_out/ab_e3.log
for r in 1 2; do
  for lib in rbe550_final_project_amd/librbe_mi355x.so abvariants/lib_ew4.so; do
    echo "== $lib" >> gpurun_out/ab_e3.log
    RBE_LIB_PATH=$lib timeout -k 10 300 python tools/well_ab.py dense=RBE_EDGE_PACKED:0 auto=RBE_NN_MFMA:4 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_e3.log || exit 1
    timeout -k 10 120 python tools/plan_bench.py $lib goal4_pentagon_10box 262144 full 2>&1 | grep -v amdgpu.ids | tail -1 >> gpurun_out/ab_e3.log || exit 1
    timeout -k 10 120 python tools/plan_bench.py $lib goal3_tallest_10box 4096 2>&1 | grep -v amdgpu.ids | tail -1 >> gpurun_out/ab_e3.log || exit 1
  done
done
