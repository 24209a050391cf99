# edge launches: lane-group kernels up to RBE_ML_EDGE_MAX items (default 65,536) vs
# the one-lane wave-compacted k_edges above; C5 covered-well plans (product
# schedule and whole iterations), C3 / C4 RRT plans; two rounds (the bound is read
# once per process)
set -o pipefail
rm -f gpurun_out/ab_mledge.log
for r in 1 2; do
  for m in 65536 16384 4096; do
    echo "== RBE_ML_EDGE_MAX=$m" >> gpurun_out/ab_mledge.log
    RBE_ML_EDGE_MAX=$m timeout -k 10 300 python tools/well_ab.py sched=RBE_NN_MFMA:4 whole=RBE_PLAN_CHUNK:-1 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_mledge.log || exit 1
    RBE_ML_EDGE_MAX=$m timeout -k 10 120 python tools/plan_bench.py goal3_tallest_10box 4096 2>&1 | grep -v amdgpu.ids | tail -1 >> gpurun_out/ab_mledge.log || exit 1
    RBE_ML_EDGE_MAX=$m timeout -k 10 120 python tools/plan_bench.py goal4_pentagon_10box 262144 full 2>&1 | grep -v amdgpu.ids | tail -1 >> gpurun_out/ab_mledge.log || exit 1
  done
done
