"""Reference-compatible import path: ``from model import SimpleCNN`` (reference model.py).

The implementation lives in ``ddp_amd.models.simple_cnn``: same topology, parameter
names and state_dict, MI355X-native parameter layouts and HIP kernels on the GPU.
"""
from ddp_amd.models.simple_cnn import SimpleCNN  # noqa: F401

__all__ = ["SimpleCNN"]
