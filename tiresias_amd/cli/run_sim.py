"""Trace-driven simulation CLI, flag-compatible with the reference's
``python run_sim.py --scheme S --schedule P --trace_file T ...``
(``/root/reference/run_sim.py:1709-1756``).

Outputs go to ``log/<log_path>/`` (default ``log/result-<timestamp>``):
cluster.csv, job.csv (with JCT), gpu/cpu/memory/network.csv,
decisions.jsonl, summary.json, output.log.

Examples::

    python -m tiresias_amd.cli.run_sim --schedule dlas-gpu --scheme tiresias \
        --trace_file trace.csv --num_queue 3 --queue_limits 3600,36000
    python -m tiresias_amd.cli.run_sim --synthetic 500 --schedule gittins
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time

from ..config import FLAGS, SimConfig, define_flags
from ..config import flags as fl
from ..engine.sim import simulate
from ..trace import readers, synth


def _extra_flags():
    if "synthetic" in FLAGS:
        return
    fl.DEFINE_integer("synthetic", 0, "generate a Philly-like trace with this many jobs")
    fl.DEFINE_float("load", 1.2, "offered load for --synthetic")
    fl.DEFINE_string("trace_units", "auto", "live trace: ticks (reference /10000) or seconds")


def load_specs(cfg: SimConfig):
    d = FLAGS.as_dict()
    if d.get("synthetic"):
        return synth.philly_like_trace(d["synthetic"], cfg.cluster.num_gpus, load=d["load"],
                                       seed=cfg.seed)
    path = d.get("trace_file")
    if not path:
        raise SystemExit("--trace_file or --synthetic N is required")
    sch = readers.detect_schema(path)
    if sch == "live":
        # reference tick semantics: time / 10000, minutes * 0.5 per tick (schedule.py:187)
        scale = 0.5 if cfg.engine == "tick" else 60.0
        specs = readers.read_live_trace(path, time_div=10000.0 if cfg.engine == "tick" else 1.0,
                                        minutes_scale=scale, max_jobs=d.get("max_jobs", 0))
    else:
        specs = readers.read_tiresias_trace(path, time_unit=cfg.time_unit,
                                            duration_scale=cfg.duration_scale,
                                            max_jobs=d.get("max_jobs", 0))
    return specs


def main(argv=None) -> dict:
    define_flags()
    _extra_flags()
    FLAGS.parse(sys.argv[1:] if argv is None else argv)
    cfg = SimConfig.from_flags()
    backend = FLAGS.as_dict().get("backend", "sim")
    if backend == "fake":
        from . import run_cluster

        return run_cluster.main(sys.argv[1:] if argv is None else argv)
    if backend != "sim":
        raise SystemExit(f"--backend {backend}: run_sim drives the event simulator (sim) or the fake "
                         "executor (fake); real GPUs run through tiresias_amd.cli.run_cluster")
    log_path = cfg.log_path or ("result-" + time.strftime("%Y%m%d-%H-%M-%S", time.localtime()))
    out = log_path if os.path.isabs(log_path) else os.path.join("log", log_path)
    os.makedirs(out, exist_ok=True)
    logging.basicConfig(level=logging.DEBUG if cfg.verbose else logging.INFO,
                        handlers=[logging.FileHandler(os.path.join(out, "output.log"))]
                        + ([logging.StreamHandler(sys.stdout)] if cfg.verbose else []),
                        format="%(asctime)s %(levelname)s %(message)s")
    specs = load_specs(cfg)
    prior = None
    if cfg.gittins_prior:
        prior = readers.read_duration_prior(cfg.gittins_prior)
    logging.info("config: %s", json.dumps(cfg.to_dict(), default=str))
    logging.info("jobs: %d, cluster GPUs: %d", len(specs), cfg.cluster.num_gpus)
    s = simulate(cfg, specs, out_dir=out, prior=prior)
    logging.info("summary: %s", json.dumps(s))
    print(json.dumps(s))
    return s


if __name__ == "__main__":
    main()
