PROBE_VALIDITY=1 PROBE_CTX_STREAM=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tools/share_probe.py > gpurun_out/share.log 2>&1; echo "rc=$?"; grep "world\|after" gpurun_out/share.log
PROBE_TORCH_GPU=1 timeout -k 10 200 python -c "
import os, sys, time, json; sys.path.insert(0, '.')
import torch
from rbe550_final_project_amd.native import Context
torch.cuda.set_device(0); s1 = torch.cuda.Stream(); s2 = torch.cuda.Stream()
x = torch.ones(10, device='cuda')
with torch.cuda.stream(s1): y = x * 2
with torch.cuda.stream(s2): z = x * 3
torch.cuda.synchronize(); print('ok')
" > gpurun_out/q.log 2>&1; echo "q rc=$?"
