"""Seeded synthetic trace generators.

* :class:`SampleTraceGenerator` — the reference's population sampler
  (``core/jobs/job_generator.py:14-162``): model size / iterations / duration
  / arrival drawn from built-in sample populations by cumulative-weight
  sampling, num_gpu ~ U[1,128), interval ~ U[20,44). Same populations, but an
  explicit ``random.Random(seed)`` (reference is unseeded, defect D10).
* :func:`philly_like_trace` — an NSDI'19 (Microsoft Philly) shaped workload
  for MI355X replays: GPU demand mostly 1 GPU with a power-of-two tail capped
  at the cluster size, heavy-tailed log-normal service times, Poisson
  arrivals at a target load, and a model mix over the four real workloads
  (ResNet-50 / VGG-16 / Transformer / GNMT). The real trace is not shipped
  with the reference (``.gitignore:13``) and there is no network, so every
  replay states that its trace is synthetic.
"""
from __future__ import annotations

import math
import random
from typing import Dict, List, Optional, Sequence

from ..core.job import JobSpec

MODEL_SAMPLE = [1.04, 1.27, 15.36, 108.48, 125.16, 125.16, 237.61, 330.52, 364.2, 462.77, 544.24,
                636.75, 664.1, 700., 798.28, 862.95]
ITER_SAMPLE = [1, 1, 1, 1, 1, 1, 109, 126, 133, 138, 141, 143, 144, 147, 157, 168, 175, 192, 193, 198,
               235, 237, 242, 253, 258, 272, 272, 274, 288, 326, 326, 362, 386, 391, 410, 438, 447,
               468, 473, 513, 513, 521, 521, 525, 581, 606, 607, 775, 775, 789, 822, 864, 864, 892,
               903, 949, 1011, 1085, 1360, 1501, 2178, 2239, 2275, 3304, 3469, 4861]
DURATION_SAMPLE = [121] * 21 + [122] * 4 + [123] * 3 + [124, 125, 125, 126, 126, 126, 126, 127, 128,
                                                         130, 131, 133, 135, 138, 141, 143, 147, 152,
                                                         155, 158, 164, 171, 180, 189, 196, 209, 230,
                                                         263, 305, 368, 536, 1800]
ARRIVAL_SAMPLE = [10, 100, 500, 1000, 3000, 5000, 10000]


def cdf(samples: Sequence[float]) -> List[float]:
    n = len(samples)
    return [i / (n - 1) for i in range(n)] if n > 1 else [1.0]


class SampleTraceGenerator:
    def __init__(self, seed: int = 0):
        self.rng = random.Random(seed)
        self.populations = {"model": list(MODEL_SAMPLE), "duration": list(DURATION_SAMPLE),
                            "itter": list(ITER_SAMPLE), "arrival": list(ARRIVAL_SAMPLE)}

    def set_population(self, name: str, samples: Sequence[float]) -> None:
        if not samples:
            raise ValueError("population cannot be empty")
        self.populations[name] = list(samples)

    def sample(self, name: str, k: int) -> List[float]:
        pop = self.populations[name]
        # cum_weights = the reference's cdf(): first element has weight 0
        return self.rng.choices(pop, cum_weights=cdf(pop), k=k)

    def generate_trace(self, number: int) -> Dict[str, list]:
        return {
            "model": self.sample("model", number),
            "duration": self.sample("duration", number),
            "itter": self.sample("itter", number),
            "arrival": self.sample("arrival", number),
            "num_gpu": [self.rng.randrange(1, 128) for _ in range(number)],
            "interval": [self.rng.randrange(20, 44) for _ in range(number)],
            "job_id": list(range(number)),
        }

    def generate_specs(self, number: int, max_gpu: Optional[int] = None) -> List[JobSpec]:
        tr = self.generate_trace(number)
        t = 0.0
        out = []
        for i in range(number):
            t += tr["interval"][i]
            g = tr["num_gpu"][i] if max_gpu is None else min(tr["num_gpu"][i], max_gpu)
            out.append(JobSpec(job_id=str(i), submit_time=t, duration=float(tr["duration"][i]),
                               num_gpu=int(g), iterations=int(tr["itter"][i]),
                               interval=float(tr["interval"][i])))
        return out


# Philly-like job-size distribution (fraction of jobs by GPU count; NSDI'19
# reports most jobs single-GPU with a long multi-GPU tail)
PHILLY_GPU_DIST = [(1, 0.70), (2, 0.10), (4, 0.10), (8, 0.07), (16, 0.02), (32, 0.01)]
# model mix for MI355X replays, with measured-style GPU util / memory profiles
MODEL_PROFILES = {
    "resnet50": dict(util=(85, 98), mem_gb=(14, 18), weight=0.35),
    "vgg16": dict(util=(80, 97), mem_gb=(12, 16), weight=0.20),
    "transformer": dict(util=(70, 95), mem_gb=(10, 20), weight=0.30),
    "gnmt": dict(util=(55, 85), mem_gb=(16, 30), weight=0.15),
}


def philly_like_trace(num_jobs: int, cluster_gpus: int, load: float = 1.0, seed: int = 0,
                      median_duration: float = 600.0, sigma: float = 1.5,
                      max_duration: float = 86400.0 * 2, models: Optional[Dict[str, dict]] = None,
                      gpu_dist=PHILLY_GPU_DIST) -> List[JobSpec]:
    """Poisson arrivals tuned so the offered GPU load ~= ``load`` x cluster."""
    rng = random.Random(seed)
    models = models or MODEL_PROFILES
    names = list(models)
    weights = [models[m]["weight"] for m in names]
    dist = [(g, p) for g, p in gpu_dist if g <= cluster_gpus]
    tot = sum(p for _, p in dist)
    gs = [g for g, _ in dist]
    ps = [p / tot for _, p in dist]
    mu = math.log(median_duration)
    durs, gpus = [], []
    for _ in range(num_jobs):
        durs.append(min(max_duration, max(1.0, rng.lognormvariate(mu, sigma))))
        gpus.append(rng.choices(gs, weights=ps)[0])
    mean_work = sum(d * g for d, g in zip(durs, gpus)) / num_jobs
    rate = load * cluster_gpus / mean_work          # jobs per second
    t = 0.0
    out = []
    for i in range(num_jobs):
        m = rng.choices(names, weights=weights)[0]
        prof = models[m]
        ua = rng.uniform(prof["util"][0], (prof["util"][0] + prof["util"][1]) / 2)
        umax = rng.uniform(ua, prof["util"][1])
        mem_max = rng.uniform(*prof["mem_gb"]) * 1024
        out.append(JobSpec(job_id=str(i), submit_time=round(t, 3), duration=round(durs[i], 3),
                           num_gpu=gpus[i], model=m, gpu_util_avg=round(ua, 2),
                           gpu_util_max=round(umax, 2), gpu_mem_avg=round(mem_max * 0.85, 1),
                           gpu_mem_max=round(mem_max, 1)))
        t += rng.expovariate(rate)
    return out
