for w in goal3_tallest_10box goal1_scattered_6box goal4_pentagon_10box; do
SWEEP_STRAIGHT=0 timeout -k 10 120 python -u tools/plan_sweep.py $w 4096 16 32 64 128 256 512 > gpurun_out/sw_$w.log 2>&1; echo "== $w"; cat gpurun_out/sw_$w.log
done
