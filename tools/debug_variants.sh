timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_cfg.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_cfg.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/c5_profile.py > gpurun_out/c5prof.log 2>&1; echo "c5 rc=$?"; cat gpurun_out/c5prof.log
timeout -k 10 200 python -u tools/c5_profile.py grouped > gpurun_out/c5prof_g.log 2>&1; echo "c5g rc=$?"; cat gpurun_out/c5prof_g.log
