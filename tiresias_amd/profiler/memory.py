"""GPU memory / utilisation profiles of the workloads.

* ``MODEL_CKPT_MB`` + ``estimate_gpu_memory`` keep the reference's heuristic
  (``/root/reference/model/model_factory.py:19-106``: runtime-init memory +
  3x weights + activations, as a fraction of GPU capacity) for traces that
  only name a model — with the runtime-init constant and capacity updated for
  MI355X (ROCm runtime, 288 GB HBM3E) and no random noise (seeded callers add
  their own);
* ``measure(model)`` measures the real peak HBM of one training step of our
  kernels (``torch.cuda.max_memory_allocated``) and its iteration time — the
  numbers the scheduler's packing / HBM-suspension budget should use.
"""
from __future__ import annotations

import time
from typing import Dict, Optional

from .skew import model_profile

# checkpoint (fp32 weights) sizes in MB of the reference's models
MODEL_CKPT_MB = {
    "alexnet": 233.0, "vgg11": 507.0, "vgg16": 528.0, "vgg19": 548.0, "resnet18": 45.0,
    "resnet34": 83.0, "resnet50": 98.0, "resnet101": 171.0, "resnet152": 231.0,
    "inception3": 92.0, "inception4": 163.0, "densenet121": 31.0, "mobilenet": 17.0,
    "transformer": 240.0, "bert": 420.0, "gnmt": 870.0, "lstm": 200.0, "deepspeech": 144.0,
}
RUNTIME_INIT_MB = 700.0     # HIP runtime + RCCL + allocator pools per process (ROCm 7)


def weights_mb(model: str) -> float:
    try:
        return model_profile(model).total_mb
    except KeyError:
        return MODEL_CKPT_MB.get(model, 200.0)


def estimate_gpu_memory(model: str, batch: int = 32, capacity_mb: float = 288 * 1024,
                        act_mb_per_sample: float = 60.0) -> Dict[str, float]:
    w = weights_mb(model)
    total = RUNTIME_INIT_MB + 3.0 * w + act_mb_per_sample * batch
    return {"weights_mb": w, "total_mb": total, "fraction": min(1.0, total / capacity_mb)}


def measure(model: str, batch: Optional[int] = None, steps: int = 3) -> Dict[str, float]:
    import torch

    from ..executor.trainer import Trainer

    dev = torch.device("cuda", torch.cuda.current_device())
    torch.cuda.reset_peak_memory_stats(dev)
    base = torch.cuda.memory_allocated(dev)
    t = Trainer(model, dev, batch=batch)
    t.step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        t.step()
    torch.cuda.synchronize(dev)
    it = (time.perf_counter() - t0) / steps
    peak = torch.cuda.max_memory_allocated(dev) - base
    return {"model": model, "batch": t.batch, "peak_mb": peak / 2 ** 20,
            "state_mb": t.state_bytes() / 2 ** 20, "iter_s": it}
