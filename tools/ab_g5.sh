# grid-scene (clutter) k_validity / k_edges at 5 waves per SIMD (abvariants/lib_g5.so:
# -DRP_EDGE_WAVES=5 -DRP_VALIDITY_WAVES_GRID=5; 96 VGPRs, 6 spilled in the BF
# instantiations) vs 4 (in-tree, no spills): C5 covered-well plans, edge_bench
# --host clutter64 (loop-free k_edges and k_validity on the same 4.2 M states),
# bench.py clutter64 config; two interleaved rounds
set -o pipefail
rm -f gpurun_out/ab_g5.log
for r in 1 2; do
  for lib in rbe550_final_project_amd/librbe_mi355x.so abvariants/lib_g5.so; do
    echo "== $lib" >> gpurun_out/ab_g5.log
    RBE_LIB_PATH=$lib timeout -k 10 300 python tools/well_ab.py dense=RBE_EDGE_PACKED:0 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_g5.log || exit 1
    d=gpurun_out/g5_${r}_$(basename $lib .so)
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o kt -- python tools/edge_bench.py $lib --scene clutter64 --host --reps 20 > $d.log 2>&1 || exit 1
    grep -h "k_edges\|k_validity" $d/kt_kernel_stats.csv | awk -F'",' '{print substr($1,2,40), $2}' >> gpurun_out/ab_g5.log
  done
done
