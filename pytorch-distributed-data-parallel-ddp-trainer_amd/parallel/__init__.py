from .process_group import (setup, cleanup, native_comm, local_rank, default_backend, ensure_master_env, free_port,
                            resolve_backend)
from .launcher import launch, under_torchrun, default_world_size
from .ddp import DistributedDataParallel, DDP, bucket_plan, bucket_ranges
from .xgmi import create_xgmi

__all__ = ["setup", "cleanup", "native_comm", "local_rank", "default_backend", "ensure_master_env",
           "free_port", "resolve_backend", "launch", "under_torchrun", "default_world_size", "DistributedDataParallel",
           "DDP", "bucket_plan", "bucket_ranges", "create_xgmi"]
