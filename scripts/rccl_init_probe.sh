#!/bin/bash
cd $GRAFT_REPO_ROOT
for envs in "" "RCCL_MSCCL_ENABLE=0" "NCCL_NET_PLUGIN=none NCCL_IB_DISABLE=1" "RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0 NCCL_IB_DISABLE=1 NCCL_NET_PLUGIN=none"; do
  env $envs timeout -k 10 120 python3 -c "
import time, torch
import spacedrive_amd as sd
from spacedrive_amd import dedup
ctx = sd.default_context(0); torch.cuda.synchronize()
t0 = time.perf_counter(); c = dedup.make_comm(ctx); t1 = time.perf_counter()
print('env [$envs]: comm init %.2f s' % (t1 - t0))
c.close()
" 2>&1 | grep "comm init" || exit 1
done
