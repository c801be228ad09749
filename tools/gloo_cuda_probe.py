"""gloo all_reduce on HIP tensors: ordering after compute kernels, and slice views (storage offset != 0)."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    for dt in (torch.float32, torch.bfloat16):
        buf = torch.zeros(1 << 20, device="cuda", dtype=dt)
        a = torch.randn(4096, 4096, device="cuda")
        for _ in range(3):
            a = a @ a.t() / 4096
        buf.add_(float(rank + 1) + 0 * a[0, 0].to(dt))
        dist.all_reduce(buf, async_op=True).wait()
        torch.cuda.synchronize()
        print(f"rank {rank} {dt} whole: got {buf[0].item()} expected {sum(range(1, world + 1))}", flush=True)
        big = torch.zeros(4 << 20, device="cuda", dtype=dt)
        big[1 << 20:2 << 20] = rank + 1
        w = dist.all_reduce(big[1 << 20:2 << 20], async_op=True)
        w.wait()
        torch.cuda.synchronize()
        print(f"rank {rank} {dt} view: slice {big[(1 << 20) + 5].item()} (expect {sum(range(1, world + 1))}), "
              f"head {big[5].item()} (expect 0)", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.start_processes(worker, args=(2, int(sys.argv[1]) if len(sys.argv) > 1 else 29611), nprocs=2,
                       start_method="spawn")
