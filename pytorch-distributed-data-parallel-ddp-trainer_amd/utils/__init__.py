from .checkpoint import (checkpoint_path, discover_latest, build_checkpoint, save_checkpoint,
                         load_checkpoint, resume)

__all__ = ["checkpoint_path", "discover_latest", "build_checkpoint", "save_checkpoint",
           "load_checkpoint", "resume"]
