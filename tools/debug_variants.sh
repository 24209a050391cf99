export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_rrt -o t -- python tools/plan_trace.py goal3_tallest_10box 4096 > gpurun_out/tl_rrt.log 2>&1 || exit 1
python tools/timeline.py gpurun_out/tl_rrt/t_kernel_trace.csv 40 > gpurun_out/tl_rrt.txt
