"""Run the LIVE cluster on this node's GPUs: the scheduler (rank 0) drives
real DDP training jobs on the hand-written HIP kernels, one process per GPU.

Jobs come from a trace file (either reference schema; durations are mapped to
iterations with the measured per-iteration time, compressed by
``--time_scale``) and/or online submissions through ``--spool`` (see
``cli/submit.py``). Outputs: ``<log_path>/{job,cluster,gpu_live}.csv``,
``decisions.jsonl``, ``summary.json``.

``--backend fake`` runs the same controller against an in-process virtual-time
model of the ranks (``executor/fake.py``): no GPUs, no processes.

Launch (one rank per GPU)::

    python -m torch.distributed.run --standalone --nproc-per-node 8 \\
        -m tiresias_amd.cli.run_cluster --schedule dlas-gpu --scheme tiresias \\
        --trace_file trace.csv --time_scale 0.001 --log_path live1
    # serve submissions until `submit --shutdown`:
    python -m torch.distributed.run --standalone --nproc-per-node 8 \\
        -m tiresias_amd.cli.run_cluster --spool /tmp/tam --log_path live2
"""
from __future__ import annotations

import json
import os
import sys
import time
from datetime import timedelta

import torch
import torch.distributed as dist

from ..config import FLAGS, SimConfig, define_flags
from ..config import flags as fl
from ..executor.cluster_runtime import NOMINAL_ITER_S, ReplayJob, Worker, run_replay
from ..executor.spool import Spool
from ..models import MODELS


def _extra_flags():
    if "spool" in FLAGS:
        return
    fl.DEFINE_string("spool", "", "spool directory for online job submission (cli/submit.py)")
    fl.DEFINE_float("time_scale", 1.0, "multiply trace durations (seconds) by this before mapping "
                    "them to iterations (e.g. 0.001 replays a 1000 s job as ~1 s of training)")
    fl.DEFINE_float("quantum", 0.25, "scheduling round length (s)")
    fl.DEFINE_string("default_model", "resnet50", "model for trace rows without a known model")
    fl.DEFINE_boolean("graph", True, "hipGraph-capture 1-GPU jobs' fwd+bwd")
    fl.DEFINE_integer("max_jobs", 0, "read at most this many trace rows")
    fl.DEFINE_string("trace_units", "seconds", "live-schema trace: seconds or ticks")


def _trace_jobs(cfg: SimConfig, world: int):
    from ..trace import readers

    d = FLAGS.as_dict()
    path = d.get("trace_file")
    if not path:
        return []
    if readers.detect_schema(path) == "live":
        specs = readers.read_live_trace(path, time_div=1.0, minutes_scale=60.0, max_jobs=d["max_jobs"])
    else:
        specs = readers.read_tiresias_trace(path, time_unit=cfg.time_unit, duration_scale=cfg.duration_scale,
                                            max_jobs=d["max_jobs"])
    ts = d["time_scale"]
    jobs = []
    for s in specs:
        if s.num_gpu > world:
            continue
        m = s.model if s.model in MODELS else d["default_model"]
        it_s = NOMINAL_ITER_S.get(m, 0.03) * (1.0 if s.num_gpu == 1 else 1.08)
        iters = max(1, int(round(s.duration * ts / it_s)))
        spec = type(s)(**{**s.__dict__, "submit_time": s.submit_time * ts,
                          "duration": s.duration * ts, "model": m, "iterations": iters})
        jobs.append(ReplayJob(spec=spec, model=m, iterations=iters))
    return jobs


def _main_fake(cfg: SimConfig, d: dict):
    """``--backend fake``: the live controller against an in-process
    virtual-time model of ``num_gpu_p_node`` ranks (executor/fake.py)."""
    from ..executor.fake import run_fake

    world = cfg.cluster.num_gpu_p_node
    cfg.cluster = type(cfg.cluster)(**{**cfg.cluster.__dict__, "num_switch": 1, "num_node_p_switch": 1})
    jobs = _trace_jobs(cfg, world)
    if not jobs:
        raise SystemExit("--backend fake needs --trace_file")
    log_path = cfg.log_path or ("fake-" + time.strftime("%Y%m%d-%H-%M-%S", time.localtime()))
    out = log_path if os.path.isabs(log_path) else os.path.join("log", log_path)
    s = run_fake(cfg, jobs, world, quantum=d["quantum"], out_dir=out)
    print(json.dumps(s, default=str))
    return s


def main(argv=None):
    define_flags()
    _extra_flags()
    FLAGS.parse(sys.argv[1:] if argv is None else argv)
    cfg = SimConfig.from_flags()
    d = FLAGS.as_dict()
    if d.get("debug_kernels"):
        from ..utils import debug

        debug.enable(d["debug_kernels"])          # before the first HIP call
    if d.get("backend") == "fake":
        return _main_fake(cfg, d)
    if d.get("backend") not in ("sim", "mi355x", None):
        raise SystemExit(f"unknown --backend {d.get('backend')!r} (sim | fake | mi355x)")
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    use_cuda = torch.cuda.is_available()
    device = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(device)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    ctrl_pg = world_pg = None
    if world > 1:
        dist.init_process_group("nccl" if use_cuda else "gloo", rank=rank, world_size=world,
                                device_id=device if use_cuda else None, timeout=timedelta(minutes=10))
        world_pg = dist.group.WORLD
        ctrl_pg = dist.new_group(backend="gloo")
    # the cluster is this node: world GPUs, one node (or virtual nodes)
    cfg.cluster = type(cfg.cluster)(**{**cfg.cluster.__dict__, "num_switch": 1, "num_node_p_switch": 1,
                                       "num_gpu_p_node": world})
    jobs = _trace_jobs(cfg, world)
    spool = Spool(d["spool"]) if (d["spool"] and rank == 0) else None
    if not jobs and spool is None and rank == 0:
        raise SystemExit("nothing to run: give --trace_file and/or --spool")
    log_path = cfg.log_path or ("live-" + time.strftime("%Y%m%d-%H-%M-%S", time.localtime()))
    out = log_path if os.path.isabs(log_path) else os.path.join("log", log_path)
    w = Worker(rank, world, device, world_pg, use_graph=use_cuda and d["graph"])
    s = run_replay(cfg, jobs, rank, world, device, ctrl_pg=ctrl_pg, world_pg=world_pg, worker=w,
                   quantum=d["quantum"], out_dir=out if rank == 0 else None,
                   max_rounds=10 ** 9, spool=spool)
    if rank == 0:
        print(json.dumps(s, default=str))
    if world > 1:
        dist.destroy_process_group()
    return s


if __name__ == "__main__":
    main()
