#!/usr/bin/env python3
"""Where a rank's RCCL communicator init time goes (1 rank, this GPU).

Prints one JSON line: seconds for torch.cuda init, init_process_group (eager,
device_id), first all-reduce; run with NCCL_DEBUG=INFO
NCCL_DEBUG_TIMESTAMP_LEVELS=ALL to get RCCL's own timestamped init log on stderr.
"""
import json
import time

t0 = time.time()
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

t_imp = time.time()
torch.cuda.set_device(0)
torch.cuda.init()
x = torch.ones(1, device="cuda")
torch.cuda.synchronize()
t_dev = time.time()
dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=torch.device("cuda", 0))
t_pg = time.time()
dist.all_reduce(x)
torch.cuda.synchronize()
t_ar = time.time()
dist.destroy_process_group()
print(json.dumps({"import_s": round(t_imp - t0, 3), "hip_init_s": round(t_dev - t_imp, 3),
                  "pg_init_s": round(t_pg - t_dev, 3), "first_allreduce_s": round(t_ar - t_pg, 3)}), flush=True)
