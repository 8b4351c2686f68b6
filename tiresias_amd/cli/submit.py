"""Submit a job to a running live cluster, or query / stop it.

The live runtime (``python -m tiresias_amd.cli.run_cluster --spool DIR``)
polls ``DIR`` every scheduling round (see ``executor/spool.py``).

Examples::

    python -m tiresias_amd.cli.submit --spool /tmp/tam --model resnet50 --gpus 2 --iterations 800
    python -m tiresias_amd.cli.submit --spool /tmp/tam --model gnmt --duration 30
    python -m tiresias_amd.cli.submit --spool /tmp/tam --status
    python -m tiresias_amd.cli.submit --spool /tmp/tam --shutdown
"""
from __future__ import annotations

import argparse
import json
import sys

from ..executor.spool import Spool


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--spool", required=True)
    ap.add_argument("--model")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--iterations", type=int)
    ap.add_argument("--duration", type=float, help="seconds of service (converted to iterations)")
    ap.add_argument("--job-id")
    ap.add_argument("--batch", type=int)
    ap.add_argument("--status", action="store_true")
    ap.add_argument("--shutdown", action="store_true", help="stop serving once the cluster drains")
    a = ap.parse_args(argv)
    sp = Spool(a.spool)
    if a.status:
        print(json.dumps(sp.status(), indent=1))
        return 0
    if a.shutdown:
        sp.shutdown()
        print("shutdown requested")
        return 0
    if not a.model or (a.iterations is None and a.duration is None):
        ap.error("--model and one of --iterations / --duration are required")
    jid = sp.submit(a.model, a.gpus, iterations=a.iterations, duration=a.duration, job_id=a.job_id,
                    batch=a.batch)
    print(jid)
    return 0


if __name__ == "__main__":
    sys.exit(main())
