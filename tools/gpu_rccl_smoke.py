"""RCCL smoke on ONE GPU (world 1): the member-only gang communicator
(parallel/gang.py::GangPG over ProcessGroupNCCL) rendezvous + all_reduce /
reduce / broadcast on device tensors, and the store-based control plane."""
import os

import torch
import torch.distributed as dist

from tiresias_amd.parallel.gang import GangPG

dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29533", rank=0, world_size=1)
torch.cuda.set_device(0)
pg = GangPG((0,), 0, "nccl")
t = torch.arange(1 << 20, device="cuda", dtype=torch.float32)
pg.all_reduce(t).wait()
pg.reduce(t, 0).wait()
pg.broadcast(t, 0).wait()
torch.cuda.synchronize()
assert torch.equal(t, torch.arange(1 << 20, device="cuda", dtype=torch.float32))
print("GangPG nccl world-1 OK")
dist.destroy_process_group()
