"""Probe: can two ranks share one GPU under RCCL (nccl backend)?  Prints the outcome."""
import os, sys, datetime
import torch, torch.distributed as dist
r = int(os.environ["RANK"]); w = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=r, world_size=w, timeout=datetime.timedelta(seconds=60),
                        device_id=torch.device("cuda", 0))
t = torch.full((1 << 20,), float(r + 1), device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
print("rank", r, "allreduce ok", float(t[0]), flush=True)
dist.destroy_process_group()
