"""Online job-submission API of the live runtime (executor/spool.py,
cli/submit.py): queued and mid-run submissions, validation, status, shutdown."""
import json
import os
import threading
import time

import torch

from tiresias_amd.cli import submit as submit_cli
from tiresias_amd.config import ClusterSpec, SimConfig
from tiresias_amd.executor.cluster_runtime import Worker, run_replay
from tiresias_amd.executor.spool import Spool


def _cfg():
    return SimConfig(schedule="dlas-gpu", scheme="count", num_queue=2, queue_limits=[0.5],
                     cluster=ClusterSpec(num_switch=1, num_node_p_switch=1, num_gpu_p_node=1))


def test_spool_roundtrip_and_validation(tmp_path):
    sp = Spool(str(tmp_path / "spool"))
    assert submit_cli.main(["--spool", sp.root, "--model", "resnet_tiny", "--iterations", "3",
                            "--job-id", "a"]) == 0
    sp.submit("vgg_tiny", 1, duration=0.05, job_id="b")
    sp.submit("not_a_model", 1, iterations=3, job_id="bad")
    sp.submit("resnet_tiny", 4, iterations=3, job_id="toobig")
    sp.shutdown()
    out = str(tmp_path / "log")
    w = Worker(0, 1, torch.device("cpu"))
    s = run_replay(_cfg(), [], 0, 1, torch.device("cpu"), worker=w, quantum=0.05, out_dir=out,
                   spool=sp)
    assert s["finished"] == 2 and s["jobs"] == 2
    rej = sorted(os.listdir(os.path.join(sp.root, "rejected")))
    assert rej == ["bad.json", "toobig.json"]
    why = json.load(open(os.path.join(sp.root, "rejected", "bad.json")))["reason"]
    assert "unknown model" in why
    st = sp.status()
    assert st["finished"] == 2 and st["jobs"]["a"]["state"] == "FINISHED"
    assert st["jobs"]["a"]["iterations_done"] == 3 and st["jobs"]["a"]["jct_s"] > 0


def test_submit_while_running(tmp_path):
    sp = Spool(str(tmp_path / "spool"))
    sp.submit("resnet_tiny", 1, iterations=40, job_id="long")
    res = {}

    def serve():
        w = Worker(0, 1, torch.device("cpu"))
        res["s"] = run_replay(_cfg(), [], 0, 1, torch.device("cpu"), worker=w, quantum=0.05, spool=sp)

    th = threading.Thread(target=serve)
    th.start()
    t0 = time.time()
    while (sp.status() or {}).get("running", 0) == 0 and time.time() - t0 < 60:
        time.sleep(0.05)
    sp.submit("vgg_tiny", 1, iterations=2, job_id="short")   # arrives mid-run
    sp.shutdown()
    th.join(timeout=300)
    assert not th.is_alive()
    s = res["s"]
    assert s["finished"] == 2
    st = sp.status()
    # 2D-LAS: the short newcomer preempts the long job that already attained service
    assert st["jobs"]["short"]["jct_s"] < st["jobs"]["long"]["jct_s"]


def test_run_cluster_cli_trace(tmp_path):
    from tiresias_amd.cli import run_cluster
    from tiresias_amd.core.job import JobSpec
    from tiresias_amd.trace.readers import write_tiresias_trace

    tr = tmp_path / "t.csv"
    write_tiresias_trace(str(tr), [JobSpec("1", 0.0, 100.0, 1, model="resnet_tiny"),
                                   JobSpec("2", 50.0, 20.0, 1, model="vgg_tiny"),
                                   JobSpec("3", 60.0, 30.0, 1, model="unknown_net")])
    s = run_cluster.main(["--trace_file", str(tr), "--time_scale", "0.002", "--schedule", "dlas-gpu",
                          "--scheme", "count", "--num_queue", "2", "--queue_limits", "0.1",
                          "--default_model", "transformer_tiny", "--log_path", str(tmp_path / "live"),
                          "--quantum", "0.05"])
    assert s["finished"] == 3
    assert (tmp_path / "live" / "job.csv").exists()


def test_malformed_requests_are_rejected_not_fatal(tmp_path):
    """Untrusted spool files: garbage JSON, non-object JSON,
    non-numeric / negative / boolean fields and absurd batches are moved to
    rejected/ with a reason; valid jobs in the same poll still run."""
    sp = Spool(str(tmp_path / "spool"))
    inc = os.path.join(sp.root, "incoming")
    bad = {
        "garbage.json": "{not json",
        "list.json": json.dumps([1, 2, 3]),
        "strgpu.json": json.dumps({"job_id": "s", "model": "resnet_tiny", "num_gpu": "two", "iterations": 3}),
        "neg.json": json.dumps({"job_id": "n", "model": "resnet_tiny", "iterations": -4}),
        "booliter.json": json.dumps({"job_id": "b", "model": "resnet_tiny", "iterations": True}),
        "fraciter.json": json.dumps({"job_id": "f", "model": "resnet_tiny", "iterations": 2.5}),
        "hugebatch.json": json.dumps({"job_id": "h", "model": "resnet_tiny", "iterations": 2, "batch": 10 ** 9}),
        "nodur.json": json.dumps({"job_id": "d", "model": "resnet_tiny"}),
        "objid.json": json.dumps({"job_id": {"x": 1}, "model": "resnet_tiny", "iterations": 2}),
    }
    for name, text in bad.items():
        with open(os.path.join(inc, name), "w") as f:
            f.write(text)
    # non-UTF-8 bytes: UnicodeDecodeError is a ValueError, not a JSONDecodeError
    with open(os.path.join(inc, "latin1.json"), "wb") as f:
        f.write(b'{"job_id": "\xff\xfe", "model": "resnet_tiny"}')
    bad["latin1.json"] = None
    sp.submit("resnet_tiny", 1, iterations=2, job_id="ok")
    sp.shutdown()
    w = Worker(0, 1, torch.device("cpu"))
    s = run_replay(_cfg(), [], 0, 1, torch.device("cpu"), worker=w, quantum=0.05, spool=sp)
    assert s["finished"] == 1
    rej = set(os.listdir(os.path.join(sp.root, "rejected")))
    assert set(bad) <= rej
    assert os.listdir(inc) == []
    assert "positive integer" in json.load(open(os.path.join(sp.root, "rejected", "strgpu.json")))["reason"]
    why = json.load(open(os.path.join(sp.root, "rejected", "latin1.json.reason.json")))["reason"]
    assert "UnicodeDecodeError" in why
