for i in 1 2 3; do
DBG_TORCH=1 RBE_DEBUG_SYNC=1 timeout -k 5 60 python -u tools/debug_seq.py group_then_single > gpurun_out/d$i.log 2>&1; echo "d$i rc=$?"
done
true
