"""Reference-compatible import path: ``from utils import setup, cleanup`` (reference utils.py).

``setup(rank, world_size, backend=None)`` joins the process group (RCCL on MI355X,
gloo on CPU) and binds the local-rank GPU; ``cleanup()`` tears it down.  Same log lines.
"""
from ddp_amd.parallel.process_group import cleanup, setup  # noqa: F401

__all__ = ["setup", "cleanup"]
