"""Host sanitizers over the native control plane: the event
core built with ASan + UBSan replays every policy it supports on seeded
traces -- plain and priced (checkpoint stalls, spread-gang network rate,
wait-vs-spread placement) -- and checks the engine invariants
(tools/sanitize.sh)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_sched_core_asan_ubsan(tmp_path):
    env = dict(os.environ, SKIP_HIP="1", N_JOBS="300")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh"), str(tmp_path)],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "SANITIZE OK" in r.stdout
    # the priced topology paths (checkpoint stalls, spread-gang network rate,
    # the wait-vs-spread rule) ran under ASan/UBSan too
    priced = [x for x in r.stdout.splitlines() if " ckpt=" in x]
    assert len(priced) >= 40, r.stdout[-2000:]
    assert any("tiresias ckpt=2 net=1 wait=1" in x and " spread=0 " not in x for x in priced)
    assert r.stdout.count("POOL OK") == 2                 # ASan+UBSan and TSan runs
    assert "ThreadSanitizer" not in r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
