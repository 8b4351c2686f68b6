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
