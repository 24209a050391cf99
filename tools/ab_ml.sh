# lane-group kernels A/B: abvariants/lib_head.so (HEAD) vs the in-tree library;
# plans of goal3 / goal1 (RRT forced and straight first), two interleaved rounds
set -o pipefail
rm -f gpurun_out/ab_ml.log
for r in 1 2; do
  for lib in abvariants/lib_head.so rbe550_final_project_amd/librbe_mi355x.so; do
    for m in "" sf; do
      for wl in goal3_tallest_10box goal1_scattered_6box; do
        timeout -k 10 120 python tools/plan_bench.py $lib $wl 4096 $m 2>&1 | grep -v amdgpu.ids | tail -1 >> gpurun_out/ab_ml.log || exit 1
      done
    done
  done
done
