# edge endpoints loaded beside valid / gfail (abvariants/lib_spec.so, -DRP_EDGE_SPEC=1)
# vs in-tree: C5 covered-well plan edge time, goal3 RRT plans, edge_bench (goal3,
# clutter64); two interleaved rounds
set -o pipefail
rm -f gpurun_out/ab_spec.log
for r in 1 2; do
  for lib in rbe550_final_project_amd/librbe_mi355x.so abvariants/lib_spec.so; do
    echo "== $lib" >> gpurun_out/ab_spec.log
    RBE_LIB_PATH=$lib timeout -k 10 300 python tools/well_ab.py dense=RBE_EDGE_PACKED:0 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_spec.log || exit 1
    timeout -k 10 120 python tools/plan_bench.py $lib goal3_tallest_10box 4096 2>&1 | grep -v amdgpu.ids | tail -1 >> gpurun_out/ab_spec.log || exit 1
    for sc in goal3 clutter64; do
      timeout -k 10 120 python tools/edge_bench.py $lib --scene $sc 2>&1 | grep -v amdgpu.ids | tail -3 >> gpurun_out/ab_spec.log || exit 1
    done
  done
done
