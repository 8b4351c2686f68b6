"""Control plane of the live cluster: round plans out, worker reports back,
and liveness (SURVEY §5.3 failure detection).

``StorePlane`` (default for distributed replays) carries the per-round
plan/report exchange over the c10d key-value store instead of collectives,
so a lost rank cannot wedge the surviving ones:

* rank 0 publishes ``plan/<epoch>/<round>``; workers block on it
  (``store.wait``), run, and publish ``rep/<epoch>/<round>/<rank>``;
* every worker also runs a HEARTBEAT thread on its own store connection,
  stamping ``hb/<rank>`` every ``hb_period`` seconds — independent of the
  training thread, so a rank busy in a long step, or stuck in a collective
  with a dead peer, still reads as alive;
* while gathering, rank 0 polls the report keys; a rank whose report is
  missing AND whose heartbeat is older than ``hb_timeout`` (5-10 s; never
  the 10-minute collective timeout) is declared LOST and returned to the
  controller, which re-plans around it (``Controller.rank_lost``).

``GlooPlane`` is the collective-based plane (``broadcast_object_list`` /
``gather_object`` on a gloo group) kept for comparison; a lost rank there
surfaces only as a collective error / timeout.
"""
from __future__ import annotations

import os
import pickle
import threading
import time
from datetime import timedelta
from typing import Dict, List, Optional, Sequence, Tuple

import torch.distributed as dist

_EPOCH = {"n": 0}


class ControllerLost(RuntimeError):
    pass


class GlooPlane:
    def __init__(self, pg, rank: int, world: int):
        self.pg, self.rank, self.world = pg, rank, world

    def bcast(self, plan, rnd: int):
        lst = [plan]
        dist.broadcast_object_list(lst, src=0, group=self.pg)
        return lst[0]

    def gather(self, rep, rnd: int, alive: Sequence[int]) -> Tuple[Optional[List], List[int]]:
        reps = [None] * self.world if self.rank == 0 else None
        dist.gather_object(rep, reps, dst=0, group=self.pg)
        return reps, []

    def close(self):
        pass


def _store_client(timeout_s: float):
    """A NEW connection to the job's TCP store (threads get their own)."""
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ["MASTER_PORT"])
    return dist.TCPStore(host, port, is_master=False, timeout=timedelta(seconds=timeout_s),
                         wait_for_workers=False)


class StorePlane:
    def __init__(self, rank: int, world: int, hb_period: float = 1.0, hb_timeout: float = 6.0,
                 plan_timeout: float = 600.0, store=None):
        self.rank, self.world = rank, world
        self.hb_period, self.hb_timeout = hb_period, hb_timeout
        self.plan_timeout = plan_timeout
        _EPOCH["n"] += 1                         # every rank replays in the same order
        self.prefix = f"tam/{_EPOCH['n']}"
        self.store = store or _store_client(plan_timeout)
        self._stop = threading.Event()
        self._hb: Optional[threading.Thread] = None
        self.dead: set = set()
        self.last_seen: Dict[int, float] = {}
        if rank != 0:
            self._hb = threading.Thread(target=self._beat, name=f"hb-{rank}", daemon=True)
            self._hb.start()

    # ----------------------------------------------------------- heartbeat
    def _beat(self):
        st = _store_client(30.0)
        while not self._stop.is_set():
            try:
                st.set(f"tam/hb/{self.rank}", repr(time.time()))
            except Exception:                    # store gone: controller lost, main thread notices
                return
            self._stop.wait(self.hb_period)

    def heartbeat_age(self, r: int) -> float:
        k = f"tam/hb/{r}"
        if not self.store.check([k]):
            return float("inf")
        return time.time() - float(self.store.get(k).decode())

    # ----------------------------------------------------------- plan / reports
    def _retry(self, fn, what: str, attempts: int = 3):
        """Run a store operation; a dropped connection (seen under heavy host
        load when a peer process dies) reconnects and retries before the
        controller is declared lost."""
        for i in range(attempts):
            try:
                return fn()
            except Exception as e:                # DistNetworkError / DistStoreError
                if i + 1 == attempts:
                    raise ControllerLost(f"{what}: {e}") from e
                time.sleep(0.2 * (i + 1))
                try:
                    self.store = _store_client(self.plan_timeout)
                except Exception:
                    pass

    def bcast(self, plan, rnd: int):
        key = f"{self.prefix}/plan/{rnd}"
        if self.rank == 0:
            self._retry(lambda: self.store.set(key, pickle.dumps(plan)), f"publish plan {rnd}")
            return plan

        def _get():
            self.store.wait([key], timedelta(seconds=self.plan_timeout))
            return self.store.get(key)

        return pickle.loads(self._retry(_get, f"no plan for round {rnd}"))

    def gather(self, rep, rnd: int, alive: Sequence[int]) -> Tuple[Optional[List], List[int]]:
        if self.rank != 0:
            data = pickle.dumps(rep)
            self._retry(lambda: self.store.set(f"{self.prefix}/rep/{rnd}/{self.rank}", data), f"report {rnd}")
            return None, []
        reps: List = [None] * self.world
        reps[0] = rep
        pending = [r for r in alive if r != 0 and r not in self.dead]
        newly: List[int] = []
        t0 = time.time()
        sleep = 0.0002
        while pending:
            left = []
            for r in pending:
                k = f"{self.prefix}/rep/{rnd}/{r}"
                if self.store.check([k]):
                    reps[r] = pickle.loads(self.store.get(k))
                    self.store.delete_key(k)
                else:
                    left.append(r)
            pending = left
            if not pending:
                break
            if time.time() - t0 > self.hb_timeout:
                for r in list(pending):
                    if self.heartbeat_age(r) > self.hb_timeout:
                        pending.remove(r)
                        self.dead.add(r)
                        newly.append(r)
            time.sleep(sleep)
            sleep = min(0.002, sleep * 1.5)
        if rnd > 0:
            try:
                self.store.delete_key(f"{self.prefix}/plan/{rnd - 1}")
            except Exception:
                pass
        return reps, newly

    def close(self):
        self._stop.set()
