"""RCCL smoke on ONE GPU (world 1): the member-only gang communicator
(parallel/gang.py::GangPG over ProcessGroupNCCL) rendezvous + all_reduce /
reduce / broadcast on device tensors, and its lifecycle on real RCCL:
eager warm-up (comm creation outside any timed region), generation-keyed
re-creation through the PGCache, the watchdog configuration, and abort()
(what the control plane's watcher calls on a communicator containing a dead
rank) leaving the process alive with ``failed()`` reporting it."""
import os
import time

import torch
import torch.distributed as dist

from tiresias_amd.parallel import gang
from tiresias_amd.parallel.gang import GangPG, PGCache, configure_nccl_env

configure_nccl_env()
assert os.environ["TORCH_NCCL_ASYNC_ERROR_HANDLING"] == "2"
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

cache = PGCache()
t0 = time.perf_counter()
a = cache.acquire((0,), 0, "nccl", pin=True)
a.warm(torch.device("cuda", 0))
print(f"create+warm {1e3 * (time.perf_counter() - t0):.1f} ms, gen {a.gen}")
assert not a.failed()
t0 = time.perf_counter()
a.abort()
print(f"abort {1e3 * (time.perf_counter() - t0):.1f} ms, failed={a.failed()}")
assert a.failed()
cache.purge([a.key])
b = cache.acquire((0,), 0, "nccl")
assert b is not a and b.gen == 1
b.warm(torch.device("cuda", 0))
x = torch.ones(1 << 16, device="cuda")
b.all_reduce(x).wait()
torch.cuda.synchronize()
assert float(x[0]) == 1.0 and not b.failed()
cache.release(b)
assert len(cache) == 0
print("PGCache abort / re-create (gen 1) / shutdown OK")
dist.destroy_process_group()
