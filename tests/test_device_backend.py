"""Real-device backend (cluster/device.py): parsing on CPU, probing on GPU."""
import pytest

from tiresias_amd.cluster import device as D


def test_num_parsing():
    assert D._num({"value": 42, "unit": "%"}) == 42.0
    assert D._num("17 %") is None or D._num("17%") == 17.0
    assert D._num("N/A") is None and D._num(None) is None


def test_probe_cpu_host_is_empty_not_synthetic():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert D.probe_devices() == []
    spec = D.probe_cluster_spec()
    assert spec.num_gpu_p_node == 8          # falls back to the MI355X preset


@pytest.mark.gpu
def test_probe_real_gpu(gpu):
    devs = D.probe_devices()
    assert len(devs) >= 1
    d = devs[0]
    assert d.total_mb > 100_000 and 0 < d.free_mb <= d.total_mb     # MI355X: 288 GB HBM3E
    spec = D.probe_cluster_spec()
    assert spec.num_gpu_p_node == len(devs) and spec.gpu_memory_mb == pytest.approx(
        min(x.total_mb for x in devs))
    m = D.DeviceMonitor(period=0.0)
    assert m.sample()[0].index == 0


def test_background_monitor_never_blocks(monkeypatch):
    """Worker-side monitor: the amd-smi probe runs on a daemon thread;
    sample_own() only reads the cache (a slow CLI cannot stall a round)."""
    import threading
    import time

    started = threading.Event()

    def slow_smi():
        started.set()
        time.sleep(0.5)
        return {0: {"util_pct": 50.0, "vram_used_mb": 1.0}}

    monkeypatch.setattr(D, "smi_utilization", slow_smi)
    m = D.DeviceMonitor(period=10.0, device_index=None).start()
    assert started.wait(2.0)
    t0 = time.perf_counter()
    assert m.sample_own() is None                 # no device index / CPU host
    assert time.perf_counter() - t0 < 0.05
    m.stop()


@pytest.mark.gpu
def test_monitor_sample_own_gpu(gpu):
    m = D.DeviceMonitor(period=5.0, device_index=0).start()
    d = m.sample_own()
    assert d is not None and d.index == 0 and 0 < d.free_mb <= d.total_mb
    m.stop()
