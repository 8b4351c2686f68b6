"""tiresias_amd — an MI355X-native deep-learning cluster scheduler with the
capabilities of Tiresias (NSDI'19): discretized 2D-LAS and Gittins-index
scheduling, skew-aware consolidated/spread placement, checkpoint preemption,
and real DDP workloads (ResNet-50, VGG-16, Transformer-base, GNMT) running on
hand-written gfx950 HIP kernels with RCCL over xGMI.
"""
__version__ = "0.1.0"
