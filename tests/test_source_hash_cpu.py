"""the shipped _C.so is tied to the sources it was built from.

``_build.py`` embeds a hash of every file under ``csrc`` (plus the compile flags) in the
binary; ``native.require()`` recomputes it over the tree and refuses a binary built from
other sources, so a forgotten rebuild cannot silently test old kernels on the GPU box.
"""
import os
import shutil

import pytest

from ddp_amd import _build, native


def test_shipped_binary_matches_tree():
    if not os.path.exists(native.so_path()):
        pytest.skip("no in-tree _C.so (run __graft_entry__.build() first)")
    ok, msg = native.check_binary()
    assert ok, msg
    assert _build.binary_hash() == _build.source_hash()


def _fake_so(path, digest):
    with open(path, "wb") as f:
        f.write(b"\x7fELF" + b"\0" * 100 + _build.HASH_MARKER + digest.encode() + b"\0" * 50)


def test_touched_source_is_refused_and_rebuild_clears_it(tmp_path):
    csrc = tmp_path / "csrc"
    shutil.copytree(_build.CSRC, csrc)
    so = str(tmp_path / "_C.so")
    _fake_so(so, _build.source_hash(str(csrc)))  # "built" from this tree
    assert native.check_binary(so, str(csrc))[0]
    # touching a kernel source (one comment byte) makes the binary stale ...
    hip = csrc / "kernels" / "allreduce.hip"
    hip.write_text(hip.read_text() + "\n// touched\n")
    ok, msg = native.check_binary(so, str(csrc))
    assert not ok and "rebuild" in msg
    # ... so does a new header, and a changed compile flag set
    h2 = _build.source_hash(str(csrc))
    (csrc / "kernels" / "extra.h").write_text("#pragma once\n")
    assert _build.source_hash(str(csrc)) != h2
    # a rebuild (the binary now carries the new hash) clears it
    _fake_so(so, _build.source_hash(str(csrc)))
    assert native.check_binary(so, str(csrc))[0]


def test_flags_are_part_of_the_hash(monkeypatch):
    h = _build.source_hash()
    monkeypatch.setitem(_build.KERNEL_FLAGS, "conv3x3.hip", ["-fno-slp-vectorize", "-O1"])
    assert _build.source_hash() != h


def test_binary_without_marker_is_stale(tmp_path):
    so = str(tmp_path / "_C.so")
    with open(so, "wb") as f:
        f.write(b"\x7fELF" + b"\0" * 64)
    ok, msg = native.check_binary(so)
    assert not ok and "pre-round-6" in msg


def test_require_raises_stale_binary(monkeypatch, tmp_path):
    """require() itself refuses (before loading the library) - the GPU fixture turns this into
    a session failure instead of testing the old kernels."""
    so = str(tmp_path / "_C.so")
    _fake_so(so, "0" * _build.HASH_LEN)
    monkeypatch.setattr(native, "so_path", lambda: so)
    monkeypatch.setattr(native, "_mod", None)
    monkeypatch.setattr(native, "_err", None)
    monkeypatch.delenv("DDP_AMD_NATIVE_SO", raising=False)
    monkeypatch.delenv("DDP_AMD_SKIP_SOURCE_CHECK", raising=False)
    with pytest.raises(native.StaleBinaryError, match="rebuild"):
        native.require()
