"""Produce reference-parity fixtures by EXECUTING the reference's live simulator.

Copies the reference tree (``--reference``, read-only) into a scratch
directory, writes small live-schema traces there, runs the reference's
``run_sim.py`` (its fixed-tick loop, core/scheduling/schedule.py:178-212) for
each (schedule, scheme) pair, and parses per-job start/finish ticks and the
devices each job was placed on from the reference's own log
(``delta-time: N`` from job_generator.py:202, ``placing task J_worker0 at node
N - device D`` from infra/node.py:226, ``job J finish`` from schedule.py:156).

The traces are built so none of the reference defects that SURVEY.md §3
lists for the live path can change the outcome:
  * D1 (the loop ignores queued jobs): an anchor job runs until every other
    job has finished, so ``running > 0`` while anything is queued;
  * D8 (new arrival batches inserted at the queue head): no job arrives while
    another one is waiting;
  * D2 (reservation leak) and D6/D7 do not trigger on one node without
    migration.
The tool asserts that every job finished in the reference run before it
writes the fixture; ``tests/test_ref_parity.py`` replays the same traces
through ``TickSimulator`` and must reproduce every tick.

Usage: python tools/ref_parity.py --reference /root/reference \
           --out tests/fixtures/ref_parity.json
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

# (job_id, arrival tick, used_gpus, gpu_per_container, minutes); the reference runs minutes*0.5
# ticks (jobs_manager.py:226 via schedule.py:187 scale_factor=0.5).
TRACES = {
    # one 4-GPU node: blocking head, one placement per tick, ceil(0.5*minutes)
    "node4_blocking": dict(gpus_per_node=4, nodes=1, jobs=[
        ("0", 0, 1, 1, 60.0),      # anchor (30 ticks)
        ("1", 1, 2, 2, 5.0),       # placed 1, ends 1+3
        ("2", 2, 1, 1, 7.0),       # placed 2, ends 2+4
        ("3", 3, 2, 2, 3.0),       # needs 2, only 0 free -> waits until 1 ends at 4
        ("4", 8, 3, 3, 4.0),       # 3 free at 8 -> placed 8, ends 10
        ("5", 12, 3, 3, 9.0),      # placed 12, ends 17
        ("6", 13, 1, 1, 2.0),      # 0 free until 17 -> placed 17, ends 18
    ]),
    # two 4-GPU nodes: multi-worker gangs (workers of gpu_per_container GPUs)
    "two_node_gang": dict(gpus_per_node=4, nodes=2, jobs=[
        ("0", 0, 1, 1, 80.0),      # anchor (40 ticks)
        ("1", 1, 4, 2, 6.0),       # 2 workers x 2 GPUs
        ("2", 2, 2, 1, 10.0),      # 2 workers x 1 GPU
        ("3", 3, 4, 4, 4.0),       # whole node: waits for 1
        ("4", 12, 6, 2, 2.0),      # 3 workers x 2 GPUs across both nodes
        ("5", 20, 2, 2, 3.0),
        ("6", 26, 3, 1, 5.0),
    ]),
    # horus+ re-clustering with SEVERAL jobs queued at once (every arrival
    # batch pops the whole queue and k-means it again, jobs_manager.py:
    # 116-137): the queued jobs share one feature vector, so every centroid is
    # at distance 0 and each implementation's k-means puts them all in queue 0
    # whatever its random init -- the tick parity then pins the re-insert,
    # credit and look-ahead path deterministically. horus placement packs two
    # 50 %-utilisation jobs per GPU, so whole-node (4-GPU) jobs queue behind
    # the anchor + one running job. Horus policies only: under FIFO this trace
    # would trigger D8 (arrivals while jobs wait).
    "hplus_queue": dict(gpus_per_node=4, nodes=1, pairs=[("horus+", "horus+"), ("horus", "horus")], d2fix=True, jobs=[
        ("0", 0, 1, 1, 90.0),      # anchor (45 ticks)
        ("1", 1, 4, 4, 10.0),      # 1-3 share the node (packing)
        ("2", 2, 4, 4, 8.0),
        ("3", 3, 4, 4, 12.0),
        ("4", 4, 4, 4, 6.0),       # 4-8 queue: several waiting at once
        ("5", 5, 4, 4, 4.0),
        ("6", 6, 4, 4, 10.0),
        ("7", 7, 4, 4, 2.0),
        ("8", 8, 4, 4, 6.0),
    ]),
}
PAIRS = [("fifo", "yarn"), ("horus", "horus"), ("gandiva", "gandiva"), ("horus+", "horus+")]
# horus+ re-clusters the queue with UNSEEDED k-means (core/jobs/utils.py:36-67,
# np.random at :39/:62): the reference run is made reproducible by seeding
# numpy / random in the launching interpreter before run_sim.py executes --
# the reference's own code is not touched
SEEDED = "import random, runpy, sys, numpy; numpy.random.seed(0); random.seed(0); " \
         "sys.argv = ['run_sim.py'] + sys.argv[1:]; runpy.run_path('run_sim.py', run_name='__main__')"

# SEEDED with the reservation leak (infra/node.py:212-233) removed
# at run time: a task that does not fit on every device it needs leaves no
# device entry or cpu / mem reservation behind. The reference's files are
# not touched; the patch is applied in the launching interpreter.
D2FIX = "import infra.node as N\n" \
        "def _atomic(self, task, pack=False, _orig=N.Node.try_reserve_and_placed_task):\n" \
        "    before = {d: dict(dev.running_tasks) for d, dev in self.device_cache.items()}\n" \
        "    cpu, mem = self.cpu_used, self.mem_used\n" \
        "    ok = _orig(self, task, pack=pack)\n" \
        "    if not ok:\n" \
        "        for d, dev in self.device_cache.items():\n" \
        "            dev.running_tasks.clear(); dev.running_tasks.update(before[d])\n" \
        "        self.cpu_used, self.mem_used = cpu, mem\n" \
        "    return ok\n" \
        "N.Node.try_reserve_and_placed_task = _atomic\n"
SEEDED_D2FIX = "import random, runpy, sys, numpy; numpy.random.seed(0); random.seed(0); " \
               "sys.argv = ['run_sim.py'] + sys.argv[1:]; sys.path.insert(0, '.'); exec(%r); " \
               "runpy.run_path('run_sim.py', run_name='__main__')" % D2FIX

# horus+ k-means at FUNCTION level: the reference's own clusterize()
# (core/jobs/utils.py:36-67) executed in the scratch copy on heterogeneous
# job feature sets, numpy seeded per case. Trace-level parity cannot pin it:
# the same unseeded np.random stream also feeds horus_score's utilisation
# samples (core/scheduling/horus.py:36 -> infra/device.py:34) and the
# per-tick log (schedule.py:116), whose draw counts depend on every scoring
# call. Features: [#tasks, util avg, GPUs per worker, GPUs, util max,
# mem avg MiB, mem max MiB] with #tasks = GPUs / GPUs per worker.
KM_SCRIPT = r"""
import json, sys, numpy
sys.path.insert(0, '.')
from core.jobs.utils import clusterize
class J:
    def __init__(s, f):
        s.tasks = [0] * int(f[0]); s.gpu_utilization_avg = f[1]; s.gpu_per_worker = f[2]; s.gpus = f[3]
        s.gpu_utilization_max = f[4]; s.gpu_mem_avg = f[5]; s.gpu_mem_max = f[6]
out = []
for c in json.load(sys.stdin):
    numpy.random.seed(c["seed"])
    jobs = [J(f) for f in c["feats"]]
    cent, assign, loss = clusterize(jobs, k=c["k"])
    out.append({"cent": [jobs.index(x) for x in cent], "assign": [int(a) for a in assign], "loss": float(loss)})
print(json.dumps(out))
"""


def kmeans_cases():
    import random as _r
    cases = []
    for ci, (n, k, seed) in enumerate([(5, 2, 0), (12, 3, 1), (20, 3, 7), (33, 4, 3), (40, 2, 11), (9, 5, 2),
                                      (25, 3, 42), (16, 4, 5)]):
        rng = _r.Random(1000 + ci)
        feats = []
        for _ in range(n):
            gpw = rng.choice([1, 1, 2, 4])
            workers = rng.choice([1, 1, 2, 4, 8])
            ua = round(rng.uniform(5, 95), 1)
            um = round(min(100.0, ua + rng.uniform(0, 40)), 1)
            ma = round(rng.uniform(500, 30000), 2)
            mm = round(ma + rng.uniform(0, 4000), 2)
            feats.append([workers, ua, gpw, gpw * workers, um, ma, mm])
        cases.append({"seed": seed, "k": k, "feats": feats})
    return cases


def run_reference_kmeans(ref: str, cases) -> list:
    p = subprocess.run([sys.executable, "-c", KM_SCRIPT], cwd=ref, input=json.dumps(cases), capture_output=True,
                       text=True, timeout=300)
    if p.returncode != 0:
        raise RuntimeError(f"reference clusterize failed:\n{p.stderr[-2000:]}")
    return json.loads(p.stdout.strip().splitlines()[-1])


_DELTA = re.compile(r"delta-time: (\d+)")
_PLACE = re.compile(r"placing task (\S+?)_worker\d+ at node (\S+) - device (\d+)")
# horus / gandiva placement logs trial reservations (placing ... lines, also
# for trials that fail) before its commit, "placed task J_workerK at node N"
# (core/scheduling/algorithm.py:170): a job starts at its commit tick
_COMMIT = re.compile(r"\{algorithm:\d+\} INFO: placed task (\S+?)_worker\d+ at node (\S+)$")
_FINISH = re.compile(r"\{schedule:\d+\} INFO: job (\S+) finish")


def write_trace(path: str, jobs) -> None:
    with open(path, "w") as f:
        f.write("job_id,type,normalized_time,minutes,gpu_per_container,used_gpus,"
                "gpu_utilization_avg,gpu_utilization_max,memory_avg,memory_max,model_name\n")
        for jid, t, g, gpc, minutes in jobs:
            f.write(f"{jid},noninteractive,{t * 10000},{minutes},{gpc},{g},50,90,1048576,2097152,resnet50\n")


def parse_log(text: str):
    """Per job: start tick (the placement commit; the first reservation for
    yarn, which logs no trials), end tick, sorted [node, device] pairs of
    its reservations, and ``trial_ticks``: ticks with reservation lines but
    no commit (failed horus trials -- where the D2 leak happens)."""
    tick = 0
    out = {}
    for line in text.splitlines():
        m = _DELTA.search(line)
        if m:
            tick = int(m.group(1))
            continue
        m = _PLACE.search(line)
        if m:
            r = out.setdefault(m.group(1), {"start": None, "end": None, "devices": [], "resv": []})
            r["devices"].append([m.group(2), int(m.group(3))])
            r["resv"].append(tick)
            continue
        m = _COMMIT.search(line)
        if m:
            r = out[m.group(1)]
            if r["start"] is None or r.get("commit") is None:
                r["start"] = tick
            r["commit"] = tick
            continue
        m = _FINISH.search(line)
        if m:
            # release_finished_jobs runs after delta_time += 1 (schedule.py:190-192)
            out[m.group(1)]["end"] = tick + 1
    for r in out.values():
        r["devices"].sort()
        if r["start"] is None:                 # yarn: reservations are the placement
            r["start"] = r["resv"][0]
        trials = sorted(set(t for t in r.pop("resv") if t != r.get("commit", r["start"])))
        r.pop("commit", None)
        if trials:
            r["trial_ticks"] = trials
    return out


def run_reference(ref: str, work: str, name: str, spec: dict, schedule: str, scheme: str,
                  d2fix: bool = False) -> dict:
    write_trace(os.path.join(work, f"{name}.csv"), spec["jobs"])
    cmd = [sys.executable, "-c", SEEDED_D2FIX if d2fix else SEEDED, "--scheme", scheme, "--schedule", schedule,
           "--trace_file", f"../{name}.csv", "--num_switch", "1",
           "--num_node_p_switch", str(spec["nodes"]), "--num_gpu_p_node", str(spec["gpus_per_node"]),
           "--log_path", f"{name}_{schedule}"]
    p = subprocess.run(cmd, cwd=ref, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise RuntimeError(f"reference failed ({name}, {schedule}):\n{p.stderr[-2000:]}")
    res = parse_log(p.stderr + p.stdout)
    want = {j[0] for j in spec["jobs"]}
    done = {k for k, v in res.items() if v["end"] is not None}
    if done != want:
        raise RuntimeError(f"{name}/{schedule}: reference finished {sorted(done)} of {sorted(want)} "
                           "(a defect triggered; change the trace)")
    return res


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", required=True)
    ap.add_argument("--out", default="tests/fixtures/ref_parity.json")
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix="refparity_")
    try:
        ref = os.path.join(work, "ref")
        shutil.copytree(a.reference, ref, ignore=shutil.ignore_patterns("log", "*.pyc", "__pycache__"))
        fixture = {"generator": "tools/ref_parity.py (reference run_sim.py executed in a scratch copy)",
                   "traces": {}}
        for name, spec in TRACES.items():
            entry = {"gpus_per_node": spec["gpus_per_node"], "nodes": spec["nodes"],
                     "jobs": [list(j) for j in spec["jobs"]], "results": {}}
            for schedule, scheme in spec.get("pairs", PAIRS):
                try:
                    entry["results"][f"{schedule}/{scheme}"] = run_reference(ref, work, name, spec,
                                                                             schedule, scheme)
                except RuntimeError as e:
                    print(f"skip {name} {schedule}/{scheme}: {e}", file=sys.stderr)
                if spec.get("d2fix"):
                    # the same reference with only D2 removed (attribution run)
                    entry.setdefault("results_d2fix", {})[f"{schedule}/{scheme}"] = run_reference(
                        ref, work, name, spec, schedule, scheme, d2fix=True)
            fixture["traces"][name] = entry
        cases = kmeans_cases()
        for c, r in zip(cases, run_reference_kmeans(ref, cases)):
            c["reference"] = r
        fixture["kmeans"] = cases
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(fixture, f, indent=1, sort_keys=True)
        print(json.dumps({k: {p: {j: (r["start"], r["end"]) for j, r in v.items()}
                              for p, v in t["results"].items()}
                          for k, t in fixture["traces"].items()}, indent=1))
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
