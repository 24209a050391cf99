set -o pipefail
for v in base ew5; do
  for sc in clutter64 goal3; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/eab_${v}_$sc -o kt -- python tools/edge_bench.py abvariants/lib_$v.so --scene $sc > gpurun_out/eab_${v}_$sc.log 2>&1 || exit 1
  done
  RBE_LIB_PATH=abvariants/lib_$v.so timeout -k 10 300 python tools/well_ab.py dense=RBE_EDGE_PACKED:0,RBE_PLAN_CHUNK:-1 auto=RBE_PLAN_CHUNK:-1 dense_s=RBE_EDGE_PACKED:0 auto_s=RBE_NN_MFMA:4 > gpurun_out/wab_$v.log 2>&1 || exit 1
done
for v in base ew5; do for sc in clutter64 goal3; do echo "$v $sc: $(grep -h 'k_edges\|k_validity\|k_edge_prep' gpurun_out/eab_${v}_$sc/*kernel_stats.csv | awk -F'",' '{split($1,a,"("); print a[1], $2}' | tr '\n' ';')"; done; cat gpurun_out/wab_$v.log; done > gpurun_out/ab_summary.txt
