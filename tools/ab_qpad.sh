# k_validity A/B: in-tree (15 / 11-float queue items) vs abvariants/lib_qpad.so
# (16 / 12 floats: 128-bit LDS accesses); bench.py's validity leg, three rounds
set -o pipefail
rm -f gpurun_out/ab_qpad.log
for r in 1 2 3; do
  for lib in rbe550_final_project_amd/librbe_mi355x.so abvariants/lib_qpad.so; do
    for n in 16777216 4194304; do
      RBE_LIB_PATH=$lib timeout -k 10 120 python bench.py --states $n --steps 30 --no-plan --no-cpu --no-configs 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', $n, round(d['value']/1e9,2), d['roofline']['frac'], d['roofline']['kernel_ms'])" >> gpurun_out/ab_qpad.log || exit 1
    done
  done
done
for lib in rbe550_final_project_amd/librbe_mi355x.so abvariants/lib_qpad.so; do
  timeout -k 10 120 python tools/split_ab.py $lib 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_qpad.log || exit 1
done
