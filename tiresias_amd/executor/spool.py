"""Job-submission API of the live cluster: a spool directory.

The reference has no online submission path — jobs only come from a trace
file read at start (``core/jobs/job_generator.py:165-207``). The live MI355X
runtime additionally accepts jobs while it runs: a client drops a JSON job
description into ``<spool>/incoming/`` (atomic rename, so a half-written file
is never seen); the rank-0 controller polls the spool every scheduling round,
validates each request, moves it to ``accepted/`` or ``rejected/`` (with the
reason) and hands it to the scheduler with ``submit_time = now``. The
controller publishes ``status.json`` (per-job state, attained service, JCT)
and stops serving when ``<spool>/shutdown`` exists and the cluster is idle.

Request schema (JSON)::

    {"job_id": "optional", "model": "resnet50", "num_gpu": 2,
     "iterations": 500,             # or "duration": seconds (-> iterations via
     "batch": null}                 #    the measured per-iteration estimate)
"""
from __future__ import annotations

import json
import os
import time
import uuid
from typing import Dict, List, Optional


def _atomic_write(path: str, obj) -> None:
    tmp = f"{path}.tmp.{os.getpid()}.{uuid.uuid4().hex[:6]}"
    with open(tmp, "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
    os.replace(tmp, path)


class Spool:
    def __init__(self, root: str):
        self.root = root
        for d in ("incoming", "accepted", "rejected"):
            os.makedirs(os.path.join(root, d), exist_ok=True)

    # ------------------------------------------------------------ client side
    def submit(self, model: str, num_gpu: int = 1, iterations: Optional[int] = None,
               duration: Optional[float] = None, job_id: Optional[str] = None,
               batch: Optional[int] = None) -> str:
        if iterations is None and duration is None:
            raise ValueError("give iterations or duration")
        jid = job_id or f"sub-{time.time_ns()}-{os.getpid()}"
        req = {"job_id": jid, "model": model, "num_gpu": int(num_gpu), "iterations": iterations,
               "duration": duration, "batch": batch, "submitted_wall": time.time()}
        _atomic_write(os.path.join(self.root, "incoming", f"{jid}.json"), req)
        return jid

    def shutdown(self) -> None:
        open(os.path.join(self.root, "shutdown"), "w").close()

    def status(self) -> Optional[Dict]:
        p = os.path.join(self.root, "status.json")
        if not os.path.exists(p):
            return None
        with open(p) as f:
            return json.load(f)

    # ------------------------------------------------------------ server side
    def poll(self) -> List[Dict]:
        inc = os.path.join(self.root, "incoming")
        out = []
        for name in sorted(os.listdir(inc)):
            if not name.endswith(".json"):
                continue
            path = os.path.join(inc, name)
            try:
                with open(path) as f:
                    req = json.load(f)
            except ValueError as e:
                # JSONDecodeError, and UnicodeDecodeError for non-UTF-8 bytes
                # (both ValueErrors): an untrusted file must never reach the
                # controller (rank 0) as an exception
                self._reject_raw(path, f"unparseable request: {type(e).__name__}: {e}")
                continue
            except OSError:
                continue                     # vanished / unreadable right now: retry next poll
            if not isinstance(req, dict):
                self._reject_raw(path, f"request must be a JSON object, got {type(req).__name__}")
                continue
            req["_path"] = path
            out.append(req)
        return out

    def _reject_raw(self, path: str, reason: str) -> None:
        """Move a request that cannot even be parsed to rejected/ (it would
        otherwise be re-read every round)."""
        dst = os.path.join(self.root, "rejected", os.path.basename(path))
        try:
            _atomic_write(dst + ".reason.json", {"reason": reason})
            os.replace(path, dst)
        except OSError:
            pass

    def resolve(self, req: Dict, ok: bool, reason: str = "") -> None:
        path = req.pop("_path")
        dst = os.path.join(self.root, "accepted" if ok else "rejected", os.path.basename(path))
        if not ok:
            req["reason"] = reason
            _atomic_write(dst, req)
            os.remove(path)
        else:
            os.replace(path, dst)

    def shutdown_requested(self) -> bool:
        return os.path.exists(os.path.join(self.root, "shutdown"))

    def publish(self, status: Dict) -> None:
        _atomic_write(os.path.join(self.root, "status.json"), status)
