"""Periodic durable job snapshots: restart from the last checkpoint after a
failure (SURVEY §5.3 "Restart from the last checkpoint (§5.4)").

Suspension (``executor/cluster_runtime.py``) keeps a preempted job's state in
HBM or pinned host memory of the rank that ran it -- which dies with the rank.
A DDP gang survives a lost member through its other replicas; a job whose
ONLY replica was on the lost rank needs state that outlives the process. The
worker therefore snapshots each running job every ``snapshot_s`` seconds of
its run time, off the critical path:

1. D2D clone of the state buffers on the job's compute stream (HBM-speed,
   ordered after the step that produced them; the next step may overwrite
   the originals immediately);
2. D2H of the clones into pinned host memory on a LOW-priority side stream,
   the clones ``record_stream``-ed there so the caching allocator reuses
   their HBM only after the copy;
3. a writer thread waits for the copy's event and writes
   ``<dir>/job<id>.pt`` atomically (tmp + rename); only then is the snapshot
   reported to the controller (``poll``), so a restart never reads a
   half-written file.

The reference has no failure model (``core/jobs/job.py:88`` declares
``failed_schedule`` and never uses it); its preemption keeps
``Task.time_processed`` (``core/jobs/job.py:49-51``), which is what a
restart from a snapshot restores to the snapshot's iteration instead.
"""
from __future__ import annotations

import os
import queue
import threading
from typing import Dict, List, Optional, Tuple

import torch

# state buffers a snapshot carries: everything Trainer.state_tensors() exposes
# except the bf16 compute shadow (rebuilt from the fp32 master on load)
_SKIP = ("shadow",)


class SnapshotWriter:
    def __init__(self, directory: str, device: torch.device):
        self.dir = directory
        os.makedirs(directory, exist_ok=True)
        self.device = torch.device(device)
        self._cuda = self.device.type == "cuda"
        self._stream = torch.cuda.Stream(self.device, priority=0) if self._cuda else None
        self._q: "queue.Queue" = queue.Queue()
        self._lock = threading.Lock()
        self._done: List[Tuple[str, int, str]] = []
        self._dropped: set = set()
        self._jobs: set = set()                 # every job this writer snapshotted
        self.written = 0
        self.bytes = 0
        self._th = threading.Thread(target=self._loop, name="snapshot-writer", daemon=True)
        self._th.start()

    def path_of(self, jid: str) -> str:
        return os.path.join(self.dir, f"job{jid}.pt")

    def snapshot(self, jid: str, trainer) -> None:
        state = {k: v for k, v in trainer.state_tensors().items() if k not in _SKIP}
        step = int(trainer.step_count)
        with self._lock:
            self._dropped.discard(jid)
            self._jobs.add(jid)
        if self._cuda:
            cur = torch.cuda.current_stream(self.device)
            clones = {k: v.clone() for k, v in state.items()}           # D2D, compute stream
            self._stream.wait_stream(cur)
            with torch.cuda.stream(self._stream):
                host = {k: torch.empty(v.shape, dtype=v.dtype, pin_memory=True) for k, v in clones.items()}
                for k, v in clones.items():
                    host[k].copy_(v, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._stream)
            for v in clones.values():
                v.record_stream(self._stream)
            del clones
        else:
            host = {k: v.detach().clone() for k, v in state.items()}
            ev = None
        self._q.put((jid, step, host, ev))

    def _loop(self) -> None:
        while True:
            item = self._q.get()
            if item is None:
                return
            if isinstance(item, threading.Event):
                item.set()
                continue
            jid, step, host, ev = item
            try:
                if ev is not None:
                    ev.synchronize()
                with self._lock:
                    if jid in self._dropped:
                        continue
                path = self.path_of(jid)
                tmp = path + ".tmp"
                torch.save({"job": jid, "step": step, "state": host}, tmp)
                os.replace(tmp, path)
                nb = sum(t.numel() * t.element_size() for t in host.values())
                with self._lock:
                    if jid in self._dropped:               # finished while being written
                        _unlink(path)
                        continue
                    self._done.append((jid, step, path))
                    self.written += 1
                    self.bytes += nb
            except Exception:
                pass                                       # a failed snapshot only loses durability

    def poll(self) -> List[Tuple[str, int, str]]:
        """Snapshots durably written since the last poll: (job, step, path)."""
        with self._lock:
            out, self._done = self._done, []
        return out

    def wrote(self, jid: str) -> bool:
        """This writer snapshotted the job at some point (it must also drop it)."""
        with self._lock:
            return jid in self._jobs

    def drop(self, jid: str) -> None:
        """The job finished: its snapshot is no longer needed (any queued
        write of it is discarded)."""
        with self._lock:
            self._dropped.add(jid)
            self._jobs.discard(jid)
        _unlink(self.path_of(jid))

    def flush(self, timeout: float = 60.0) -> None:
        """Wait until every snapshot queued so far is written."""
        done = threading.Event()
        self._q.put(done)
        done.wait(timeout)

    def close(self) -> None:
        self._q.put(None)
        self._th.join(timeout=30)


def _unlink(path: str) -> None:
    try:
        os.remove(path)
    except OSError:
        pass


def load_snapshot(path: str, trainer) -> int:
    """Restore a job's state from a snapshot file into ``trainer`` (H2D into
    its existing buffers); returns the snapshot's step. Only files this
    framework wrote are loaded, and with ``weights_only=True``."""
    d = torch.load(path, map_location="cpu", weights_only=True)
    st = trainer.state_tensors()
    for k, v in d["state"].items():
        if k in st:
            st[k].copy_(v, non_blocking=False)
    A = trainer.arena
    A.shadow.copy_(A.master.to(A.shadow.dtype))
    A.grad.zero_()
    trainer.step_count = int(d["step"])
    return int(d["step"])
