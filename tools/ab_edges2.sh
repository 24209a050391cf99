# edge kernel A/B: the in-tree library vs abvariants/lib_ew5.so (5 waves/SIMD)
set -o pipefail
for v in main ew5; do
  lib=rbe550_final_project_amd/librbe_mi355x.so; [ $v = ew5 ] && lib=abvariants/lib_ew5.so
  for sc in clutter64 goal3; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/eab_${v}_$sc -o kt -- python tools/edge_bench.py $lib --scene $sc > gpurun_out/eab_${v}_$sc.log 2>&1 || exit 1
  done
  RBE_LIB_PATH=$lib timeout -k 10 300 python tools/well_ab.py dense=RBE_EDGE_PACKED:0 auto=RBE_NN_MFMA:4 > gpurun_out/wab_$v.log 2>&1 || exit 1
done
for v in main ew5; do for sc in clutter64 goal3; do echo "$v $sc: $(grep -h 'k_edges\|k_validity' gpurun_out/eab_${v}_$sc/*kernel_stats.csv | awk -F'",' '{split($1,a,"("); print a[1], $2}' | tr '\n' ';') $(grep -h 'verdicts' gpurun_out/eab_${v}_$sc.log | cut -c1-60)"; done; cat gpurun_out/wab_$v.log; done > gpurun_out/ab_summary2.txt
