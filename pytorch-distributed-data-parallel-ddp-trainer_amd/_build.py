"""Native build driver for the gfx950 extension (``ddp_amd._C``).

Everything native is compiled IN-TREE with the system ``hipcc`` (ROCm 7.2) for
``--offload-arch=gfx950`` and linked against the HIP runtime / RCCL that ship
inside the installed PyTorch wheel (``torch/lib``), so exactly one HIP runtime
and one RCCL are mapped into the process (torch's).  No hipify step, no
``torch.utils.cpp_extension`` JIT cache: the ``.so`` lands next to this file and
travels with the repo snapshot to the GPU box.

Layout of the native sources (``<repo>/csrc``):

* ``kernels/*.hip``  - device code + thin ``extern`` launchers.  These TUs do NOT
  include torch headers, so they compile in seconds.
* ``runtime/*.cpp``  - host runtime (RCCL communicator, gradient reducer, fused
  step engine + hipGraph capture).  Plain HIP host API, no torch headers.
* ``bindings.cpp``   - the only TU that includes ``torch/extension.h``; converts
  ``at::Tensor`` to raw pointers / streams and exposes everything via pybind11.

Objects are rebuilt only when their source or a ``csrc`` header they include (their
``-MD`` depfile) is newer than the object, or their command line changed; the link step
is skipped when the ``.so`` is newer than every object.

The binary is tied to its sources: every build embeds
:func:`source_hash` - a SHA-256 over every file under ``csrc`` (relative path +
bytes) and the compile flags - as the string ``DDP_AMD_SRC_HASH=<hex>`` in ``_C.so``.
``native.require()`` recomputes the hash of the tree it runs from and refuses a
binary built from other sources (:func:`binary_hash` reads the marker without loading
the library), so a forgotten rebuild cannot silently test old kernels.
"""
from __future__ import annotations

import concurrent.futures as _cf
import glob
import hashlib
import json
import mmap
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO_DIR, "csrc")
BUILD_DIR = os.path.join(REPO_DIR, "build", "native")
SO_PATH = os.path.join(PKG_DIR, "_C.so")
ARCH = os.environ.get("DDP_AMD_ARCH", "gfx950")


def _torch_dirs():
    import torch

    tdir = os.path.dirname(torch.__file__)
    return tdir, os.path.join(tdir, "include"), os.path.join(tdir, "lib")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build ddp_amd._C)")


def _headers_mtime() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    hs += glob.glob(os.path.join(CSRC, "**", "*.cuh"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _deps(obj: str):
    """The csrc headers an object was built from (its ``-MD`` depfile), or None."""
    try:
        with open(obj + ".d") as f:
            text = f.read().replace("\\\n", " ")
    except OSError:
        return None
    files = text.split(":", 1)[1].split() if ":" in text else []
    return [f for f in files if os.path.abspath(f).startswith(CSRC + os.sep)]


def _needs(obj: str, src: str, hdr_mtime: float, cmd=None) -> bool:
    """Rebuild when the object is missing, older than its source or any csrc header it
    includes (its depfile; without one: any csrc header), or was built by a different command
    line (flags change: the ``.cmd`` sidecar differs)."""
    if not os.path.exists(obj):
        return True
    if cmd is not None:
        try:
            with open(obj + ".cmd") as f:
                if f.read() != " ".join(cmd):
                    return True
        except OSError:
            return True
    t = os.path.getmtime(obj)
    deps = _deps(obj)
    if deps is not None:
        return any(not os.path.exists(d) or os.path.getmtime(d) > t for d in [src, *deps])
    return os.path.getmtime(src) > t or hdr_mtime > t


# per-TU device flags.  conv3x3.hip: no SLP vectorizer - it packed the 16-lane DPP
# reductions' adds into v_pk_add_f32, which cannot take a DPP operand, so every step became
# v_mov 0 + v_mov_dpp + add (the conv1 weight-gradient reduction of the dgrad role: 750 ->
# 400 VALU instructions with the adds folded into v_add_f32_dpp)
KERNEL_FLAGS = {"conv3x3.hip": ["-fno-slp-vectorize"], "conv3x3_bwd.hip": ["-fno-slp-vectorize"]}
COMMON_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__"]
DEVICE_FLAGS = ["-munsafe-fp-atomics"]
BIND_FLAGS = ["-O2", "-DUSE_ROCM", "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H"]
SOURCE_EXTS = (".hip", ".cpp", ".h", ".cuh", ".hpp")
HASH_MARKER = b"DDP_AMD_SRC_HASH="
HASH_LEN = 40


def source_hash(csrc: str = CSRC) -> str:
    """Hash of everything the binary is built from: each source file under ``csrc``
    (relative path + bytes, sorted) and the path-independent compile flags (the repo sits
    at another path on the GPU box, so absolute include paths are left out)."""
    h = hashlib.sha256()
    files = sorted(p for p in glob.glob(os.path.join(csrc, "**", "*"), recursive=True)
                   if os.path.isfile(p) and p.endswith(SOURCE_EXTS))
    for p in files:
        h.update(os.path.relpath(p, csrc).replace(os.sep, "/").encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    sig = dict(arch=ARCH, common=COMMON_FLAGS, device=DEVICE_FLAGS, kernel=KERNEL_FLAGS, bind=BIND_FLAGS)
    h.update(json.dumps(sig, sort_keys=True).encode())
    return h.hexdigest()[:HASH_LEN]


def binary_hash(so_path: str = SO_PATH) -> str | None:
    """The source hash embedded in a built ``_C.so`` (None: no marker - a binary from
    before round 6, or not ours).  Reads the file; does not load it."""
    try:
        with open(so_path, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as mm:
            i = mm.find(HASH_MARKER)
            if i < 0:
                return None
            return mm[i + len(HASH_MARKER):i + len(HASH_MARKER) + HASH_LEN].decode("ascii", "replace")
    except (OSError, ValueError):
        return None


def _hash_source_file() -> str:
    """(Re)write the generated TU that embeds the source hash; untouched when unchanged,
    so an unchanged tree relinks nothing."""
    path = os.path.join(BUILD_DIR, "source_hash.cpp")
    text = ("// generated by _build.py: the sources this binary was built from\n"
            f'extern "C" const char ddp_amd_source_hash_str[] = "{HASH_MARKER.decode()}{source_hash()}";\n')
    try:
        with open(path) as f:
            if f.read() == text:
                return path
    except OSError:
        pass
    with open(path, "w") as f:
        f.write(text)
    return path


def _compile_cmds():
    hipcc = _hipcc()
    _, tinc, _ = _torch_dirs()
    rocm_inc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "include")
    common = [*COMMON_FLAGS, "-I", rocm_inc, "-I", CSRC]
    cmds = []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(BUILD_DIR, "k_" + os.path.basename(src) + ".o")
        cmds.append((src, obj, [hipcc, f"--offload-arch={ARCH}", *common, *KERNEL_FLAGS.get(os.path.basename(src), []),
                                *DEVICE_FLAGS, "-MD", "-MF", obj + ".d", "-c", src, "-o", obj]))
    for src in sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))):
        obj = os.path.join(BUILD_DIR, "r_" + os.path.basename(src) + ".o")
        # host-only TUs: still driven by hipcc so hip_runtime.h resolves, but no device code
        cmds.append((src, obj, [hipcc, *common, "-x", "c++", "-MD", "-MF", obj + ".d", "-c", src, "-o", obj]))
    bsrc = os.path.join(CSRC, "bindings.cpp")
    bobj = os.path.join(BUILD_DIR, "bindings.o")
    hsrc = _hash_source_file()
    cmds.append((hsrc, os.path.join(BUILD_DIR, "source_hash.o"), ["g++", "-fPIC", "-c", hsrc, "-o",
                                                                  os.path.join(BUILD_DIR, "source_hash.o")]))
    cmds.append((bsrc, bobj, [
        hipcc, *common[:-2], "-x", "c++", "-I", CSRC, *BIND_FLAGS,
        f"-D_GLIBCXX_USE_CXX11_ABI={int(_cxx11_abi())}",
        "-I", tinc, "-I", os.path.join(tinc, "torch", "csrc", "api", "include"),
        "-I", sysconfig.get_paths()["include"], "-w", "-MD", "-MF", bobj + ".d", "-c", bsrc, "-o", bobj]))
    return cmds


def _cxx11_abi() -> bool:
    import torch

    return bool(torch._C._GLIBCXX_USE_CXX11_ABI)


def build(verbose: bool = False, jobs: int | None = None, force: bool = False) -> str:
    """Compile every HIP/C++ source for gfx950 and link ``_C.so`` in-tree.

    Returns the path of the shared object.  Raises ``RuntimeError`` with the
    compiler output on failure.
    """
    os.makedirs(BUILD_DIR, exist_ok=True)
    hdr = _headers_mtime()
    cmds = _compile_cmds()
    todo = [(s, o, c) for (s, o, c) in cmds if force or _needs(o, s, hdr, c)]
    jobs = jobs or min(8, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), max(1, len(todo)))

    def run(item):
        src, obj, cmd = item
        if verbose:
            print("[ddp_amd build]", " ".join(cmd), flush=True)
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{p.stdout}")
        with open(obj + ".cmd", "w") as f:
            f.write(" ".join(cmd))
        return src

    if todo:
        with _cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            for fut in _cf.as_completed([ex.submit(run, t) for t in todo]):
                fut.result()

    objs = [o for (_, o, _) in cmds]
    if force or todo or not os.path.exists(SO_PATH) or \
            max(os.path.getmtime(o) for o in objs) > os.path.getmtime(SO_PATH):
        _, _, tlib = _torch_dirs()
        # Link with the host compiler so hipcc does not add the system libamdhip64
        # (ROCm 7.2) next to torch's bundled runtime: one HIP runtime per process.
        tmp = SO_PATH + ".tmp"
        cmd = ["g++", "-shared", "-fPIC", *objs, "-o", tmp, "-L", tlib,
               "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
               "-lamdhip64", "-lrccl", f"-Wl,-rpath,{tlib}"]
        if verbose:
            print("[ddp_amd build]", " ".join(cmd), flush=True)
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"link failed\n{p.stdout}")
        os.replace(tmp, SO_PATH)
    return SO_PATH


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build(verbose=True, force=force))
