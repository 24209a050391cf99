for i in 1 2 3; do
DBG_TORCH=1 timeout -k 5 60 python -u tools/debug_seq.py group_then_single > gpurun_out/d$i.log 2>&1 || { echo "d$i FAILED"; exit 1; }; echo "d$i ok"
done
timeout -k 5 120 python -u tools/c5_profile.py > gpurun_out/c5prof.log 2>&1 || { echo c5prof failed; exit 1; }
timeout -k 5 120 python -u tools/c5_profile.py grouped > gpurun_out/c5prof_g.log 2>&1 || { echo c5prof_g failed; exit 1; }
bash tools/gpu_job.sh gtests
