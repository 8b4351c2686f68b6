import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device and the native library")
    config.addinivalue_line("markers", "multigpu: needs >= 2 GPUs")
    config.addinivalue_line("markers", "slow: long-running")


# the native library's tuning knobs (every *_policy / *_force setting) as
# they were when the library was loaded: the production configuration
PRODUCTION_POLICIES = None


def policy_state():
    import torch

    return list(torch.ops.tam.policy_state())


@pytest.fixture(scope="session")
def gpu():
    global PRODUCTION_POLICIES
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tiresias_amd.ops import _lib

    _lib.load(required=True)
    if PRODUCTION_POLICIES is None:
        PRODUCTION_POLICIES = policy_state()
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _restore_policies():
    """A test may force any kernel policy (a tile, a schedule, a split
    count); whatever it leaves behind is reset to the production values
    after it, so every later test -- the model-level parity tests above all
    -- runs the configuration production runs."""
    yield
    if PRODUCTION_POLICIES is not None:
        import torch

        if policy_state() != PRODUCTION_POLICIES:
            torch.ops.tam.policy_load(PRODUCTION_POLICIES)
