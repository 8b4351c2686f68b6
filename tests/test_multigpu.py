"""Multi-rank GPU gates for the gang machinery.

* ``test_rccl_world1_lifecycle``: RCCL on ONE GPU -- the member-only gang
  communicator (GangPG over ProcessGroupNCCL) all_reduce / reduce /
  broadcast, generation-keyed re-creation through the PGCache, abort()
  leaving the process alive with ``failed()`` set.
* ``test_shared_gpu_*``: TWO processes on the one GPU of the box (gloo gangs,
  the ``TAM_SHARED_GPU=1`` rehearsal): the spread transport's D2H ordering
  (HierComm with vnode_size 1 all-reducing a bucket a GEMM kernel is STILL
  writing when start() is called) against FlatComm and an fp32 sum, and
  sharded data parallelism on device tensors against the all-reduce path.
* ``test_rccl_multi_*`` (``multigpu``): self-spawned world 2..8 over RCCL,
  skipped below 2 devices -- FlatComm / HierComm equivalence, GangPG.abort
  with a hung peer (the survivor lives, failed() is true), a bitwise P2P
  state move, sharded DDP, and a 2-GPU mini replay with gangs.
"""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, world, *args, timeout=180):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    ps = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    deadline = time.time() + timeout
    for p in ps:
        p.join(max(1.0, deadline - time.time()))
    for p in ps:
        if p.is_alive():
            p.kill()
            p.join(10)
    res = {}
    while not q.empty():
        r, v = q.get()
        res[r] = v
    return [p.exitcode for p in ps], res


def _init(rank, world, port, backend):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    from tiresias_amd.parallel.gang import configure_nccl_env

    configure_nccl_env()
    dist.init_process_group(backend, rank=rank, world_size=world)


# ------------------------------------------------------------------ world 1, RCCL
def _world1(rank, world, port, q):
    from tiresias_amd.parallel.gang import GangPG, PGCache

    _init(rank, world, port, "nccl")
    torch.cuda.set_device(0)
    out = {}
    pg = GangPG((0,), 0, "nccl")
    t = torch.arange(1 << 20, device="cuda", dtype=torch.float32)
    pg.all_reduce(t).wait()
    pg.reduce(t, 0).wait()
    pg.broadcast(t, 0).wait()
    torch.cuda.synchronize()
    out["ops"] = torch.equal(t, torch.arange(1 << 20, device="cuda", dtype=torch.float32))
    cache = PGCache()
    a = cache.acquire((0,), 0, "nccl", pin=True)
    a.warm(torch.device("cuda", 0))
    out["fresh_ok"] = not a.failed()
    a.abort()
    out["aborted_failed"] = a.failed()
    cache.purge([a.key])
    b = cache.acquire((0,), 0, "nccl")
    out["gen"] = b.gen
    b.warm(torch.device("cuda", 0))
    x = torch.ones(1 << 16, device="cuda")
    b.all_reduce(x).wait()
    torch.cuda.synchronize()
    out["recreated_ok"] = float(x[0]) == 1.0 and not b.failed()
    cache.release(b)
    out["cache_empty"] = len(cache) == 0
    q.put((rank, out))
    dist.destroy_process_group()


def test_rccl_world1_lifecycle(gpu):
    codes, res = _run(_world1, 1)
    assert codes == [0], codes
    o = res[0]
    assert o == {"ops": True, "fresh_ok": True, "aborted_failed": True, "gen": 1, "recreated_ok": True,
                 "cache_empty": True}, o


# ------------------------------------------------------------------ 2 ranks on one GPU (gloo gangs)
def _shared_race(rank, world, port, q):
    from tiresias_amd.ops import _lib
    from tiresias_amd.parallel import gang as G

    _init(rank, world, port, "gloo")
    torch.cuda.set_device(0)
    _lib.load(required=True)
    T = torch.ops.tam
    dev = torch.device("cuda", 0)
    n, k = 4096, 2048
    gens = [torch.Generator(device="cpu").manual_seed(100 + r) for r in range(world)]
    ops = [(torch.randn(n, k, generator=g).to(torch.bfloat16), torch.randn(256, k, generator=g).to(torch.bfloat16))
           for g in gens]
    # the fp32 sum every rank should end with, from every rank's inputs
    want = sum(a.float() @ b.float().t() for a, b in ops)
    out = {}
    for kind in ("hier", "flat"):
        comm = G.create_gang_comm((0, 1), rank, vnode_size=1 if kind == "hier" else 0, backend="gloo",
                                  device=dev, nic_gbps=50.0)
        a, b = (x.to(dev) for x in ops[rank])
        errs = []
        for it in range(4):
            bucket = torch.full((n, 256), float("nan"), device=dev)
            # the GEMM writing the bucket is still queued / running when
            # start() is called (no host sync): the transport must order its
            # D2H after it (parallel/gang.py HierComm._exchange)
            T.gemm(a, True, b, True, bucket, 0, None, False, None, 1.0, False)
            h = comm.start(bucket.view(-1))
            comm.finish([h])
            torch.cuda.synchronize()
            errs.append(float((bucket.cpu() - want).abs().max() / want.abs().max()))
        out[kind] = max(errs)
        comm.close()
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_shared_gpu_spread_transport_orders_d2h(gpu):
    """Round-2 advisor finding (HierComm D2H of a half-written bucket):
    two ranks on cuda:0, gloo gangs; the spread transport (vnode_size 1:
    every rank its own virtual node, leaders exchange through pinned host
    memory) and the flat one both give the fp32 sum of the two ranks'
    freshly computed buckets."""
    codes, res = _run(_shared_race, 2)
    assert codes == [0, 0], codes
    for r in (0, 1):
        assert res[r]["hier"] < 1e-2 and res[r]["flat"] < 1e-2, res


def _shared_shard(rank, world, port, q, wire):
    from tiresias_amd.executor.trainer import Trainer
    from tiresias_amd.parallel import gang as G

    _init(rank, world, port, "gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = G.create_gang_comm(tuple(range(world)), rank, backend="gloo", device=dev)
    ref = Trainer("transformer_tiny", dev, seed=7, data_seed=100 + rank, group=comm, bucket_mb=0.05)
    sh = Trainer("transformer_tiny", dev, seed=7, data_seed=100 + rank, group=comm, bucket_mb=0.05,
                 ddp_shard=True, ddp_wire=wire)
    for _ in range(3):
        ref.step()
        sh.step()
    torch.cuda.synchronize()
    e_sh = float((sh.arena.shadow.float() - ref.arena.shadow.float()).norm() / ref.arena.shadow.float().norm())
    sh.consolidate()
    torch.cuda.synchronize()
    e_m = float((sh.arena.master - ref.arena.master).norm() / ref.arena.master.norm())
    q.put((rank, {"shadow": e_sh, "master": e_m, "ratio": sh.ddp.wire_bytes / ref.ddp.wire_bytes,
                  "sum": float(sh.arena.master.double().sum())}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_shared_gpu_sharded_ddp_matches(gpu, wire):
    """Sharded data parallelism on device tensors (HIP optimizer kernels over
    the member's slices, reduce-scatter / all-gather over gloo, two ranks on
    cuda:0) matches the all-reduce path; after consolidate() both members
    hold the same full state."""
    codes, res = _run(_shared_shard, 2, wire)
    assert codes == [0, 0], codes
    tol = 3e-3 if wire == "fp32" else 3e-2
    assert res[0]["sum"] == res[1]["sum"]
    for r in (0, 1):
        assert res[r]["shadow"] < tol and res[r]["master"] < tol, res
        assert res[r]["ratio"] < (0.6 if wire == "bf16" else 0.85), res


def _shared_ipc_move(rank, world, port, q):
    from tiresias_amd.executor.cluster_runtime import Worker
    from tiresias_amd.executor.control import StorePlane

    os.environ["TAM_SHARED_GPU"] = "1"
    _init(rank, world, port, "gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    w = Worker(rank, world, dev, dist.group.WORLD, gang_backend="gloo", monitor_period=0)
    w.plane = StorePlane(rank, world, hb_period=0.5, hb_timeout=10.0)
    g = torch.Generator(device=dev).manual_seed(5)
    state = {"master": torch.randn(1 << 20, device=dev, generator=g),
             "opt0": torch.randn(3 << 18, device=dev, generator=g)}
    bufs = {k: (v.clone() if rank == 0 else torch.zeros_like(v)) for k, v in state.items()}
    act = {"op": "start", "job": "J", "ranks": (1,), "old": (0,), "donors": {1: 0}}
    ops = [("send" if rank == 0 else "recv", b, 1 - rank, k) for k, b in sorted(bufs.items())]
    t0 = time.perf_counter()
    ok = w._do_moves_ipc({"J": (ops, act)}, 0)
    dt = time.perf_counter() - t0
    torch.cuda.synchronize()
    q.put((rank, {"ok": ok["J"], "s": dt, "same": all(torch.equal(bufs[k], state[k]) for k in state)}))
    dist.barrier()
    w.plane.close()
    dist.destroy_process_group()


def test_shared_gpu_ipc_state_move(gpu):
    """One-GPU multi-rank rehearsal: a job's state moves between two ranks
    on cuda:0 device to device through HIP IPC handles published in the
    control store (no gloo host staging): bitwise equal on the receiver."""
    codes, res = _run(_shared_ipc_move, 2)
    assert codes == [0, 0], codes
    assert res[0]["ok"] and res[1]["ok"], res
    assert res[1]["same"], res


# ------------------------------------------------------------------ >= 2 GPUs, RCCL
def _ndev():
    try:
        return torch.cuda.device_count()
    except Exception:
        return 0


multigpu = pytest.mark.skipif(_ndev() < 2, reason="needs >= 2 GPUs (the 8-GPU node)")


def _rccl_multi(rank, world, port, q):
    from tiresias_amd.parallel import gang as G

    _init(rank, world, port, "nccl")
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    out = {}
    ranks = tuple(range(world))
    x = torch.randn(1 << 20, device=dev, generator=torch.Generator(device=dev).manual_seed(rank))
    want = sum(torch.randn(1 << 20, device=dev, generator=torch.Generator(device=dev).manual_seed(r))
               for r in ranks)
    flat = G.create_gang_comm(ranks, rank, backend="nccl", device=dev)
    y = x.clone()
    flat.finish([flat.start(y)])
    out["flat"] = float((y - want).abs().max())
    if world >= 4:
        hier = G.create_gang_comm(ranks, rank, vnode_size=world // 2, backend="nccl", device=dev)
        z = x.clone()
        hier.finish([hier.start(z)])
        out["hier_vs_flat"] = float((z - y).abs().max())
    # bitwise state move rank 0 -> 1 over a 2-rank pair communicator
    pair = G.GangPG((0, 1), rank, "nccl") if rank < 2 else None
    if pair is not None:
        st = torch.randn(1 << 18, device=dev, generator=torch.Generator(device=dev).manual_seed(77))
        buf = st.clone() if rank == 0 else torch.zeros_like(st)
        if rank == 0:
            pair.pg.send([buf], 1, 0).wait()
        else:
            pair.pg.recv([buf], 0, 0).wait()
        torch.cuda.synchronize()
        out["p2p_bitwise"] = bool(torch.equal(buf, st))
    # abort with a hung peer: ranks 0 / 1 share a gang, rank 1 never joins
    # the collective; rank 0's abort() returns and failed() is true
    if rank < 2:
        g = G.GangPG((0, 1), rank, "nccl", timeout_s=5.0, gen=9)
        g.warm(dev)
        if rank == 0:
            t = torch.ones(1 << 16, device=dev)
            g.all_reduce(t)
            time.sleep(2.0)
            g.abort()
            out["abort_failed"] = g.failed()
        else:
            time.sleep(4.0)
            g.abort()                 # the plan's abort action reaches the peer too
        # the survivor is usable: both members build a FRESH communicator
        # (next generation, fresh store keys) and all-reduce through it
        g2 = G.GangPG((0, 1), rank, "nccl", timeout_s=30.0, gen=10)
        t2 = torch.full((1 << 12,), float(rank + 1), device=dev)
        g2.all_reduce(t2).wait()
        torch.cuda.synchronize()
        out["rebuilt_sum"] = float(t2[0])
        out["rebuilt_failed"] = g2.failed()
    q.put((rank, out))
    os._exit(0)


@multigpu
@pytest.mark.multigpu
def test_rccl_multi_gangs(gpu):
    world = min(8, _ndev())
    codes, res = _run(_rccl_multi, world, timeout=240)
    assert all(c == 0 for c in codes), codes
    for r in range(world):
        assert res[r]["flat"] < 1e-3, res[r]
        if "hier_vs_flat" in res[r]:
            assert res[r]["hier_vs_flat"] < 1e-3, res[r]
    assert res[1]["p2p_bitwise"] and res[0]["abort_failed"]
    for r in (0, 1):
        assert res[r]["rebuilt_sum"] == 3.0 and not res[r]["rebuilt_failed"], res[r]


def _rccl_shard(rank, world, port, q):
    from tiresias_amd.executor.trainer import Trainer
    from tiresias_amd.parallel import gang as G

    _init(rank, world, port, "nccl")
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    comm = G.create_gang_comm(tuple(range(world)), rank, backend="nccl", device=dev)
    ref = Trainer("transformer_tiny", dev, seed=7, data_seed=100 + rank, group=comm, bucket_mb=0.05)
    sh = Trainer("transformer_tiny", dev, seed=7, data_seed=100 + rank, group=comm, bucket_mb=0.05,
                 ddp_shard=True, ddp_wire="bf16")
    for _ in range(3):
        ref.step()
        sh.step()
    sh.consolidate()
    torch.cuda.synchronize()
    q.put((rank, float((sh.arena.master - ref.arena.master).norm() / ref.arena.master.norm())))
    os._exit(0)


@multigpu
@pytest.mark.multigpu
def test_rccl_multi_sharded_ddp(gpu):
    world = min(8, _ndev())
    codes, res = _run(_rccl_shard, world, timeout=240)
    assert all(c == 0 for c in codes), codes
    assert all(v < 3e-2 for v in res.values()), res


@multigpu
@pytest.mark.multigpu
def test_rccl_multi_mini_replay(gpu, tmp_path):
    """2-GPU bench replay with gangs over RCCL (the driver's launch shape)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--jobs-per-gpu", "8", "--work-s", "1.0", "--no-nopool-replay"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    d = json.loads(line[-1])
    assert d["n_gpus"] == 2 and d["finished_jobs"] == 16 and not d["gang_errors"]
