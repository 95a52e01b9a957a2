"""Loader for the in-tree gfx950 extension ``ddp_amd._C``.

Policy (no silent fallbacks on the GPU): if a HIP device is visible, every op in
``ddp_amd.ops`` runs its HIP kernel and :func:`require` raises when the
extension cannot be imported.  The pure-PyTorch reference implementations are
only used for tensors that live on the CPU (the CPU/gloo plumbing configuration
and the CPU unit tests).

The in-tree binary must have been built from the tree's own sources: the source hash
embedded at link time (``_build.source_hash``) is compared before the library is loaded,
and a mismatch raises :class:`StaleBinaryError` (``DDP_AMD_SKIP_SOURCE_CHECK=1`` skips it;
``DDP_AMD_NATIVE_SO`` A/B variants are not checked).
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err: BaseException | None = None


class StaleBinaryError(RuntimeError):
    """The in-tree ``_C.so`` was built from other sources than the tree it runs from."""


def check_binary(so: str | None = None, csrc: str | None = None) -> tuple[bool, str]:
    """(ok, message): whether the source hash embedded in ``so`` (default: the in-tree
    ``_C.so``) equals the hash of ``csrc`` (default: the repo's ``csrc``).  A tree without
    ``csrc`` (an installed copy) is not checked."""
    from . import _build

    so = so or so_path()
    csrc = csrc or _build.CSRC
    if not os.path.isdir(csrc):
        return True, "no csrc tree next to the package: not checked"
    have = _build.binary_hash(so)
    want = _build.source_hash(csrc)
    if have == want:
        return True, f"source hash {want}"
    return False, (f"{so} was built from sources {have or '<no hash: pre-round-6 build>'}, but the tree "
                   f"hashes to {want}: a source changed after the last build - rebuild with "
                   "`python -c 'import __graft_entry__ as g; g.build()'`")


def _try_import():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return _mod
        try:
            import torch  # noqa: F401  (loads torch's HIP runtime + RCCL first)

            variant = os.environ.get("DDP_AMD_NATIVE_SO")
            if not variant and os.environ.get("DDP_AMD_SKIP_SOURCE_CHECK") != "1":
                # the binary must come from THIS tree's sources (checked before loading it: a
                # stale library once mapped could not be replaced in this process)
                ok, msg = check_binary()
                if not ok:
                    raise StaleBinaryError(msg)
            if variant:  # A/B experiments: another build of the same extension
                import sys
                from importlib import util as _ilu

                spec = _ilu.spec_from_file_location(__package__ + "._C", variant)
                _mod = _ilu.module_from_spec(spec)
                spec.loader.exec_module(_mod)
                sys.modules[__package__ + "._C"] = _mod
            else:
                _mod = importlib.import_module(__package__ + "._C")
            import atexit

            atexit.register(_mod._mark_exiting)  # no HIP/RCCL teardown during interpreter exit
        except BaseException as e:  # ImportError, OSError (bad .so), ...
            _err = e
        return _mod


def available() -> bool:
    return _try_import() is not None


def require():
    """Return the native module or raise a RuntimeError explaining how to build it
    (:class:`StaleBinaryError` when the binary does not match the sources)."""
    m = _try_import()
    if m is None:
        if isinstance(_err, StaleBinaryError):
            raise StaleBinaryError(str(_err))
        raise RuntimeError(
            "ddp_amd native extension (_C.so) is not importable: "
            f"{_err!r}.  Build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `python -m ddp_amd._build` (hipcc --offload-arch=gfx950).")
    return m


def build_if_needed(verbose: bool = False):
    """Build the extension in-tree if sources changed (used by tests / entry points)."""
    global _mod, _err
    from . import _build

    _build.build(verbose=verbose)
    with _lock:
        _mod, _err = None, None
    return require()


def so_path() -> str:
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "_C.so")
