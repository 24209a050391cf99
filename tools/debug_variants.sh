TUNE_PLANS=0 timeout -k 10 300 python -u tools/ml_tune.py > gpurun_out/ml_tune.log 2>&1; echo "tune rc=$?"; cat gpurun_out/ml_tune.log
