"""qfedx_amd - MI355X-native privacy-preserving quantum federated learning.

Capabilities of Nidszxh/QFedX (reference snapshot at /root/reference) re-designed for AMD MI355X:
PyTorch-ROCm + hand-written gfx950 HIP kernels (statevector passes, adjoint/param-shift gradients,
client-batched TinyCNN, fused DP/SecAgg/FedAvg reduce) + RCCL over xGMI, one process per GPU.
"""
__version__ = "0.1.0"

from .config import ExperimentConfig, load_config, apply_overrides  # noqa: F401
