"""MI355X-native data-parallel CNN training template (PyTorch-ROCm + HIP/CDNA4 kernels + RCCL)."""
__version__ = "0.1.0"
