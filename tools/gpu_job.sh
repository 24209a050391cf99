#!/bin/bash
# GPU job runner for gpurun: each GPU step under its own timeout; stop at the
# first fault / abort / timeout (exit 124, 134, 137, 139). Test failures (exit 1)
# do not stop later steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  case $rc in 0|1|5) return 0 ;; *) echo "STOP after $name (rc=$rc)"; exit $rc ;; esac
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread ;;
    testsnx) step pytest_gpu 1000 python -u -m pytest tests -m gpu -v --maxfail 20 --timeout 300 --timeout-method thread ;;
    newtests) step pytest_new 900 python -u -m pytest tests/test_gpu_devices.py tests/test_gpu_async.py -m gpu -v --maxfail 20 --timeout 300 --timeout-method thread ;;
    cpuprobe) step cpuprobe_default 120 python tools/cpu_probe.py && RBE_WAIT_SPIN_US=200 step cpuprobe_spin200 120 python tools/cpu_probe.py && RBE_WAIT_SPIN_US=15 RBE_WAIT_SLEEP_FRAC=0.2 step cpuprobe_spin15 120 python tools/cpu_probe.py && step cpuprobe_b64k 120 python tools/cpu_probe.py --batch 65536 && grep -h wall_s gpurun_out/cpuprobe_*.log ;;
    nnlab) step nnlab 300 tools/lab/nn_lab 131072 300000 7 && cat gpurun_out/nnlab.log ;;
    vallab) step vallab 300 tools/lab/val_lab 16777216 20 goal3 && step vallab0 300 tools/lab/val_lab 16777216 20 goal3 0 && step vallab_t 300 tools/lab/val_lab 16777216 10 toppled && step vallab_p 300 tools/lab/val_lab 4194304 10 pentagon && step vallab2 300 tools/lab/val_lab 16777216 20 goal3 && grep -h "G/s" gpurun_out/vallab*.log ;;
    gtests) step pytest_gpu_cfg 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_group.py -m gpu -x -v --timeout 300 --timeout-method thread && step pytest_gpu_procs 600 python -u -m pytest tests/test_gpu_group_procs.py -m gpu -x -v --timeout 170 --timeout-method thread ;;
    alltests) step pytest_all 1200 python -m pytest tests -q -x ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    benchq) step bench 300 python bench.py --steps 20 --no-cpu ;;
    ab) step ab 600 python tools/variant_bench.py abvariants/*.so && step ab_clutter 600 python tools/variant_bench.py --scene clutter64 abvariants/*.so && step ab_small 600 python tools/variant_bench.py --states 65536 --iters 50 abvariants/*.so ;;
    ptrace) step ptrace 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/ptrace -o pt -- python tools/plan_trace.py && step plantime 300 python tools/plan_trace.py ;;
    gridab) step gridab 600 python tools/grid_ab.py ;;
    ptrace4) step ptrace4 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ptrace4 -o pt -- python tools/plan_trace.py goal4_pentagon_10box 262144 full && python tools/trace_summary.py gpurun_out/ptrace4/pt_kernel_trace.csv > gpurun_out/ptrace4_summary.txt && step ptrace5 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ptrace5 -o pt -- python tools/plan_trace.py clutter64 131072 full && python tools/trace_summary.py gpurun_out/ptrace5/pt_kernel_trace.csv > gpurun_out/ptrace5_summary.txt ;;
    ptraceab) for v in abvariants/*.so; do n=$(basename $v .so); step ptab_$n 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ptab_$n -o pt -- python tools/plan_trace.py $v && python tools/trace_summary.py gpurun_out/ptab_$n/pt_kernel_trace.csv > gpurun_out/ptab_${n}_summary.txt; done ;;
    tstamps) RBE_LIB_PATH=abvariants/lib_stamps.so step tstamps 300 python tools/tstamp_probe.py ;;
    mllanes) for g in 1 8 16 32; do RBE_ML_LANES=$g step mllanes_$g 300 python tools/variant_bench.py abvariants/lib_new.so --scene goal1_5box --states 65536 --iters 50 && RBE_ML_LANES=$g step mllanes3_$g 300 python tools/variant_bench.py abvariants/lib_new.so --scene goal3 --states 65536 --iters 50 && RBE_ML_LANES=$g step mllanes16k_$g 300 python tools/variant_bench.py abvariants/lib_new.so --scene goal3 --states 16384 --iters 50; done ;;
    acceptab) for r in 1 2; do for v in 0 1; do RBE_ACCEPT_SMALL=$v step acceptab_${v}_$r 300 python tools/plan_bench.py goal3_tallest_10box 4096; done; done && RBE_ACCEPT_SMALL=1 step ptab_small 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ptab_small -o pt -- python tools/plan_trace.py && python tools/trace_summary.py gpurun_out/ptab_small/pt_kernel_trace.csv > gpurun_out/ptab_small_summary.txt ;;
    frontab) for r in 1 2; do for v in 0 8 16; do RBE_ML_LANES_FRONT=$v step frontab_${v}_$r 300 python tools/plan_bench.py goal3_tallest_10box 4096; done; done ;;
    rates) step rates 600 python tools/scene_rates.py ;;
    stamps) step stamps 300 python tools/stamp_probe.py abvariants/lib_stamps.so ;;
    sweep) step sweep 600 python tools/plan_sweep.py goal3_tallest_10box 4096 32 64 128 256 512 && step sweep4 600 python tools/plan_sweep.py goal4_pentagon_10box 4096 32 64 128 256 512 ;;
    planab) for v in abvariants/*.so; do step planab_$(basename $v .so) 300 python tools/plan_bench.py $v goal4_pentagon_10box 262144 full; done ;;
    planab3) for v in abvariants/*.so; do step planab3_$(basename $v .so) 300 python tools/plan_bench.py $v goal3_tallest_10box 4096; done ;;
    bench2) step bench2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --no-cpu --backend gloo ;;
    lat) step lat 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lat -o lt -- python tools/latency_probe.py && python tools/latency_probe.py --summarize gpurun_out/lat/lt_kernel_trace.csv > gpurun_out/lat_summary.txt ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o kt -- python bench.py --steps 20 --no-cpu --no-plan --no-configs ;;
    pmc) step pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmc_sq -o sq -- python bench.py --steps 3 --warmup 1 --no-cpu --no-plan --no-configs && step pmc_sq2 600 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq2 -o sq2 -- python bench.py --steps 3 --warmup 1 --no-cpu --no-plan --no-configs && step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python bench.py --steps 3 --warmup 1 --no-cpu --no-plan --no-configs && step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python bench.py --steps 3 --warmup 1 --no-cpu --no-plan --no-configs ;;
    pmcsum) python tools/pmc_summary.py gpurun_out/pmc_sq gpurun_out/pmc_sq2 --json gpurun_out/validity_pmc_sq.json > gpurun_out/validity_pmc_sq.txt && python tools/make_pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write 16777216 gpurun_out/pmc_validity.json > /dev/null && echo pmcsum ok ;;
    c5prof) step c5prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof -o kt -- python tools/c5_profile.py ;;
    nnpmc) step nnpmc_a 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --output-format csv -d gpurun_out/nnpmc_a -o a -- python tools/c5_profile.py pmc && step nnpmc_b 300 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/nnpmc_b -o b -- python tools/c5_profile.py pmc && python tools/pmc_summary.py gpurun_out/nnpmc_a gpurun_out/nnpmc_b --kernel k_nn_mfma --json gpurun_out/nn_pmc.json > gpurun_out/nn_pmc.txt ;;
    c5stats) step c5stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5stats -o kt -- python tools/c5_profile.py ;;
    nntest) step pytest_nn 600 python -u -m pytest tests/test_gpu_nn.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    wellab) step wellab 600 python tools/well_ab.py ;;
    wellprof) step wellprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wellprof -o kt -- python tools/well_ab.py mfma=RBE_NN_MFMA:4,RBE_PLAN_CHUNK:-1 part=RBE_NN_MFMA:0,RBE_PLAN_CHUNK:-1 ;;
    satq) RBE_LIB_PATH=abvariants/lib_q59.so step satq59 300 python -u -m pytest tests/test_gpu_edge_cases.py -k saturated -m gpu -v --timeout 120 --timeout-method thread ;;
    sceneab) for r in 1 2; do step sab_head_$r 300 python tools/plan_bench.py abvariants/lib_head.so goal3_tallest_10box 4096 && for v in 1 0; do RBE_SCENE_COPY=$v step sab_new_${v}_$r 300 python tools/plan_bench.py rbe550_final_project_amd/librbe_mi355x.so goal3_tallest_10box 4096; done; done; cat gpurun_out/sab_*.log | grep median ;;
    nnab) for v in abvariants/lib_head.so rbe550_final_project_amd/librbe_mi355x.so; do n=$(basename $v .so); step nnab_$n 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nnab_$n -o kt -- python tools/nn_bench.py $v --check --tree walk && step nnabu_$n 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nnabu_$n -o kt -- python tools/nn_bench.py $v --check --tree uniform; done; for d in gpurun_out/nnab*_*/; do echo $d; grep -h "k_nn_mfma\|k_nn_part" $d/*kernel_stats.csv | cut -c1-200; done ;;
    counters) rocprofv3 -L > gpurun_out/counters.txt 2>&1; grep -i "mfma\|SQ_INSTS_VALU\b\|VALU_MFMA" gpurun_out/counters.txt | head -40 ;;
    edgepmc) step epmc_a 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --output-format csv -d gpurun_out/epmc_a -o a -- python tools/c5_profile.py pmc && step epmc_b 300 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/epmc_b -o b -- python tools/c5_profile.py pmc && python tools/pmc_summary.py gpurun_out/epmc_a gpurun_out/epmc_b --kernel k_edges --exclude packed --json gpurun_out/edges_pmc.json > gpurun_out/edges_pmc.txt && python tools/pmc_summary.py gpurun_out/epmc_a gpurun_out/epmc_b --kernel k_edges_packed --json gpurun_out/edges_packed_pmc.json > gpurun_out/edges_packed_pmc.txt && python tools/pmc_summary.py gpurun_out/epmc_a gpurun_out/epmc_b --kernel k_nn_mfma --json gpurun_out/nn_pmc.json > gpurun_out/nn_pmc.txt && cat gpurun_out/edges_pmc.txt gpurun_out/edges_packed_pmc.txt gpurun_out/nn_pmc.txt ;;
    edgepad) for pad in 0 20 60; do for sc in goal3 clutter64; do RBE_EDGE_KMAX_PAD=$pad step ep_${sc}_$pad 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ep_${sc}_$pad -o kt -- python tools/edge_bench.py --scene $sc --host && grep -h "k_edges\|k_validity" gpurun_out/ep_${sc}_$pad/*kernel_stats.csv | awk -F'",' '{print "pad '$pad' '$sc'", substr($1,2,40), $2}'; done; done ;;
    edgebench) for sc in clutter64 goal3; do step eb_$sc 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/eb_$sc -o kt -- python tools/edge_bench.py --scene $sc && grep -h "k_edges\|k_validity\|k_edge_prep" gpurun_out/eb_$sc/*kernel_stats.csv | cut -c1-160; done ;;
    edgeab) for v in abvariants/lib_head.so abvariants/lib_ew5.so rbe550_final_project_amd/librbe_mi355x.so; do n=$(basename $v .so); for sc in clutter64 goal3; do step eab_${n}_$sc 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/eab_${n}_$sc -o kt -- python tools/edge_bench.py $v --scene $sc && grep -h "k_edges" gpurun_out/eab_${n}_$sc/*kernel_stats.csv | awk -F'",' '{print "'$n' '$sc'", substr($1,1,30), $2}'; done; done ;;
    nnpmc2) step nnp_a 300 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/nnp_a -o a -- python tools/nn_bench.py --reps 2 && step nnp_b 300 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/nnp_b -o b -- python tools/nn_bench.py --reps 2 && python tools/pmc_summary.py gpurun_out/nnp_a gpurun_out/nnp_b --kernel k_nn_mfma --json gpurun_out/nn_pmc_bench.json > gpurun_out/nn_pmc_bench.txt && cat gpurun_out/nn_pmc_bench.txt ;;
    vsize) for n in 4194304 16777216 4194304 16777216; do step vsize_$n 300 python bench.py --states $n --steps 30 --no-plan --no-cpu --no-configs && grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/vsize_$n.log | head -3 | tr '\n' ' '; echo; done ;;
    nnrange) for r in 0 65536 32768 16384 8192; do RBE_NN_RANGE_MAX=$([ $r = 0 ] && echo "" || echo $r) step nnrange_$r 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nnrange_$r -o kt -- python tools/nn_bench.py && grep -h "k_nn_mfma\|k_nn_reduce" gpurun_out/nnrange_$r/*kernel_stats.csv | awk -F'",' '{print "range '$r'", substr($1,1,30), $2}'; done ;;
    nncount) step nncount 300 python tools/nn_count.py abvariants/lib_nncount.so 4 8 && cat gpurun_out/nncount.log ;;
    nnrb) for m in 4 8 2; do step nnrb_$m 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nnrb_$m -o kt -- python tools/nn_bench.py --mode $m && grep -h "k_nn_mfma" gpurun_out/nnrb_$m/*kernel_stats.csv | awk -F'",' '{print "mode '$m'", substr($1,1,30), $2}'; done ;;
    chunks) step chunks 600 python tools/chunk_sweep.py -1 16 64 256 ;;
    ptests) step pytest_plan 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
    procs) step pytest_procs 900 python -u -m pytest tests/test_gpu_group_procs.py -m gpu -x -v --timeout 400 --timeout-method thread ;;
    small) step small 300 python tools/small_launch.py && step smallprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/smallprof -o kt -- python tools/small_launch.py "" ;;
    vpmc) for v in abvariants/*.so; do n=$(basename $v .so); step vpmc_$n 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/vpmc_$n -o v -- python tools/variant_bench.py $v --rounds 1 --iters 3 && python tools/pmc_summary.py gpurun_out/vpmc_$n > gpurun_out/vpmc_$n.txt; done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== done"
