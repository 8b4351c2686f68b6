"""Control plane of the live cluster: round plans out, worker reports back,
and liveness (SURVEY §5.3 failure detection).

``StorePlane`` (default for distributed replays) carries the per-round
plan/report exchange over the c10d key-value store instead of collectives,
so a lost rank cannot wedge the surviving ones:

* rank 0 publishes ``plan/<epoch>/<round>``; workers block on it
  (``store.wait``), run, and publish ``rep/<epoch>/<round>/<rank>``;
* every worker also runs a HEARTBEAT thread on its own store connection,
  bumping an increasing COUNTER under ``hb/<rank>`` every ``hb_period``
  seconds — independent of the training thread, so a rank busy in a long
  step, or stuck in a collective with a dead peer, still reads as alive;
* rank 0 runs a MONITOR thread that reads every counter each period and
  times, on its OWN monotonic clock, how long each one has gone without
  changing (no wall-clock timestamps cross hosts, so clock skew between
  hosts cannot make a healthy rank look dead): a rank whose counter is
  stale for ``hb_timeout`` (5-10 s; never the collective timeout) is
  declared LOST, published under ``<epoch>/dead``,
  and ``on_dead(r)`` runs at once -- on a separate thread, because rank 0's
  training thread may itself be stuck in a collective with the dead rank;
* every other rank's heartbeat thread also WATCHES ``<epoch>/dead`` and
  runs ``on_dead(r)`` for each newly dead rank: the runtime aborts every
  communicator containing it, so RCCL kernels spinning on the dead peer
  exit and the survivors report instead of hanging until the watchdog;
* while gathering, rank 0 polls the report keys; dead ranks are returned to
  the controller, which re-plans around them (``Controller.rank_lost``). A
  rank that is alive but silent is reported (stderr) every ``slow_report_s``
  and declared lost after ``hung_s`` -- ``gather`` never waits unboundedly.

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
                 plan_timeout: float = 600.0, store=None, on_dead=None, slow_report_s: float = 30.0,
                 hung_s: float = 900.0):
        self.rank, self.world = rank, world
        self.hb_period, self.hb_timeout = hb_period, hb_timeout
        self.plan_timeout = plan_timeout
        self.slow_report_s, self.hung_s = slow_report_s, hung_s
        _EPOCH["n"] += 1                         # every rank replays in the same order
        self.prefix = f"tam/{_EPOCH['n']}"
        self.store = store or _store_client(plan_timeout)
        self.on_dead = on_dead
        self._stop = threading.Event()
        self._hb: Optional[threading.Thread] = None
        self._lock = threading.Lock()
        self.dead: set = set()
        self._reported: set = set()              # dead ranks already returned by gather
        # rank -> (last heartbeat counter seen, monotonic time it changed)
        self._hb_seen: Dict[int, Tuple[Optional[bytes], float]] = {}
        self.t_start = time.monotonic()
        if rank != 0:
            self._hb = threading.Thread(target=self._beat, name=f"hb-{rank}", daemon=True)
        else:
            self._hb = threading.Thread(target=self._monitor, name="hb-monitor", daemon=True)
        self._hb.start()

    # ----------------------------------------------------------- heartbeat
    def _declare(self, dead_now) -> None:
        """Record newly dead ranks and run the abort callback (any thread)."""
        new = []
        with self._lock:
            for r in dead_now:
                if r not in self.dead and r != self.rank:
                    self.dead.add(r)
                    new.append(r)
        for r in new:
            if self.on_dead is not None:
                try:
                    self.on_dead(r)
                except Exception:
                    pass

    def _beat(self):
        st = _store_client(30.0)
        dkey = f"{self.prefix}/dead"
        seen = b""
        beat = 0
        while not self._stop.is_set():
            try:
                beat += 1
                st.set(f"tam/hb/{self.rank}", str(beat))
                if st.check([dkey]):
                    raw = st.get(dkey)
                    if raw != seen:
                        seen = raw
                        self._declare(pickle.loads(raw))
            except Exception:                    # store gone: controller lost, main thread notices
                return
            self._stop.wait(self.hb_period)

    def _monitor(self):
        """Rank 0: declare ranks whose heartbeat stopped, independent of the
        training thread (which may be blocked in a collective with them)."""
        st = _store_client(30.0)
        dkey = f"{self.prefix}/dead"
        while not self._stop.wait(self.hb_period):
            if time.monotonic() - self.t_start < self.hb_timeout:
                continue                         # grace: every heartbeat thread has started
            try:
                gone = [r for r in range(1, self.world)
                        if r not in self.dead and self._age(st, r) > self.hb_timeout]
                if gone:
                    self._declare(gone)
                    with self._lock:
                        st.set(dkey, pickle.dumps(sorted(self.dead)))
            except Exception:
                return

    def _age(self, st, r: int) -> float:
        """Seconds (rank 0's monotonic clock) since rank r's heartbeat counter
        last changed; a rank that never beat counts from this plane's start."""
        k = f"tam/hb/{r}"
        val = st.get(k) if st.check([k]) else None
        now = time.monotonic()
        with self._lock:
            last = self._hb_seen.get(r)
            if last is None or (val is not None and val != last[0]):
                last = (val, now if (last is not None or val is not None) else self.t_start)
                self._hb_seen[r] = last
            return now - last[1]

    def heartbeat_age(self, r: int) -> float:
        return self._age(self.store, r)

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

    # ----------------------------------------------------------- fill mode
    # (cluster_runtime.Worker.fill_step): a rank that finished its round's
    # share keeps stepping its job until the next plan is published and
    # posts its running step count under fill/<round>/<rank>; rank 0 reads
    # every count once, when it plans (the snapshot the plan echoes)
    def plan_ready(self, rnd: int) -> bool:
        return bool(self._retry(lambda: self.store.check([f"{self.prefix}/plan/{rnd}"]), f"plan {rnd} check"))

    def publish_fill(self, rnd: int, counts: Dict[str, int]) -> None:
        data = pickle.dumps(counts)
        self._retry(lambda: self.store.set(f"{self.prefix}/fill/{rnd}/{self.rank}", data), f"fill {rnd}")

    def read_fill(self, rnd: int, alive: Sequence[int]) -> Dict[int, Dict[str, int]]:
        out: Dict[int, Dict[str, int]] = {}
        for r in alive:
            if r == 0 or r in self.dead:
                continue
            k = f"{self.prefix}/fill/{rnd}/{r}"
            if self.store.check([k]):
                out[r] = pickle.loads(self.store.get(k))
        if rnd > 0:
            # every worker has seen plan rnd (it reported round rnd): none
            # writes fill/<rnd - 1> any more
            for r in alive:
                try:
                    self.store.delete_key(f"{self.prefix}/fill/{rnd - 1}/{r}")
                except Exception:
                    pass
        return out

    def gather(self, rep, rnd: int, alive: Sequence[int], fill=None) -> Tuple[Optional[List], List[int]]:
        """Rank 0: every live rank's report of round ``rnd``. ``fill(ready)``
        (Worker.fill_step) runs between polls -- rank 0 keeps stepping its
        own job while the slower ranks finish -- and is called with
        ready=True once every report is in, until it returns False (a gang
        agrees on stopping)."""
        if self.rank != 0:
            data = pickle.dumps(rep)
            self._retry(lambda: self.store.set(f"{self.prefix}/rep/{rnd}/{self.rank}", data), f"report {rnd}")
            return None, []
        reps: List = [None] * self.world
        reps[0] = rep
        pending = [r for r in alive if r != 0]
        t0 = time.monotonic()
        t_warn = t0
        sleep = 0.0002
        while True:
            if not pending:
                if fill is not None and fill(True):
                    continue
                break
            left = []
            for r in pending:
                if r in self.dead:
                    continue
                k = f"{self.prefix}/rep/{rnd}/{r}"
                if self.store.check([k]):
                    reps[r] = pickle.loads(self.store.get(k))
                    self.store.delete_key(k)
                else:
                    left.append(r)
            pending = left
            if not pending:
                continue
            # a step of rank 0's own job instead of sleeping
            stepped = fill is not None and fill(False)
            now = time.monotonic()
            if now - t0 > self.hb_timeout:
                # the monitor thread normally declares first; this covers a
                # monitor that is itself starved
                gone = [r for r in pending if self.heartbeat_age(r) > self.hb_timeout]
                if gone:
                    self._declare(gone)
                    self.store.set(f"{self.prefix}/dead", pickle.dumps(sorted(self.dead)))
            if now - t_warn > self.slow_report_s:
                t_warn = now
                import sys

                print(f"[control] round {rnd}: waiting {now - t0:.0f} s for ranks {pending} "
                      f"(heartbeats alive)", file=sys.stderr, flush=True)
            if now - t0 > self.hung_s:
                # alive but silent for longer than any collective may take:
                # treat as lost rather than wait forever
                self._declare(pending)
                self.store.set(f"{self.prefix}/dead", pickle.dumps(sorted(self.dead)))
            if not stepped:
                time.sleep(sleep)
                sleep = min(0.002, sleep * 1.5)
        with self._lock:
            newly = sorted(r for r in self.dead if r not in self._reported)
            self._reported |= set(newly)
        if rnd > 0:
            try:
                self.store.delete_key(f"{self.prefix}/plan/{rnd - 1}")
            except Exception:
                pass
        return reps, newly

    def finish(self, alive: Sequence[int], bound_s: float = 60.0) -> None:
        """End of replay: workers acknowledge the stop plan; rank 0 returns
        only once every live worker has (its process may host the store, so
        exiting early would strand a worker still reading the last plan)."""
        if self.rank != 0:
            try:
                self.store.set(f"{self.prefix}/done/{self.rank}", b"1")
            except Exception:
                pass
            return
        t0 = time.monotonic()
        for r in alive:
            if r == 0:
                continue
            k = f"{self.prefix}/done/{r}"
            while time.monotonic() - t0 < bound_s and r not in self.dead:
                if self.store.check([k]):
                    break
                time.sleep(0.002)

    def close(self):
        self._stop.set()
