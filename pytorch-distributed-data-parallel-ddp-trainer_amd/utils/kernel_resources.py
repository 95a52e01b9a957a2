"""Per-kernel resource usage of the built gfx950 code objects (scratch guard).

Every kernel TU is compiled to ``build/native/k_<tu>.o``; its ``.hip_fatbin`` section holds
the gfx950 code object, whose AMDHSA metadata note lists, per kernel, the private-segment
(scratch) size, the VGPR / SGPR spill counts and the register counts.  A register spill or a
scratch array in a hot kernel is a silent slowdown (round 3 lost 1.4 % to 78 spilled VGPRs in
the default conv backward before anyone read the compiler's report), so
``tests/test_kernel_resources_cpu.py`` fails the build on any.

    python -m ddp_amd.utils.kernel_resources       # table of every kernel with its resources
"""
from __future__ import annotations

import glob
import os
import re
import subprocess
import tempfile

LLVM = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
FIELDS = ("private_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count", "vgpr_count",
          "agpr_count", "sgpr_count", "group_segment_fixed_size")


def _tool(name: str) -> str:
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else name


def code_object_notes(obj: str) -> str:
    """The AMDHSA metadata note text of the gfx950 code object inside a host object."""
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "dev.co")
        subprocess.run([_tool("llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "o")],
                       check=True, capture_output=True)
        subprocess.run([_tool("clang-offload-bundler"), "--type=o", f"--targets={TARGET}", f"--input={fat}",
                        f"--output={co}", "--unbundle"], check=True, capture_output=True)
        return subprocess.run([_tool("llvm-readelf"), "--notes", co], check=True, capture_output=True,
                              text=True).stdout


def parse_kernels(notes: str) -> list[dict]:
    """[{name, private_segment_fixed_size, vgpr_spill_count, ...}] from a metadata note."""
    out, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s*(?:- )?\.(\w+):\s*(\S.*)?$", line)
        if not m:
            continue
        key, val = m.group(1), (m.group(2) or "").strip()
        if key == "name" and val.startswith("_Z"):
            cur = {"name": val}
            out.append(cur)
        elif cur is not None and key in FIELDS:
            try:
                cur[key] = int(val)
            except ValueError:
                pass
    return out


def demangle(names: list[str]) -> list[str]:
    try:
        p = subprocess.run([_tool("llvm-cxxfilt")], input="\n".join(names), capture_output=True, text=True,
                           check=True)
        return p.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return names


def all_kernels(build_dir: str | None = None) -> dict[str, list[dict]]:
    """{translation unit: [kernel dicts]} for every built kernel object."""
    if build_dir is None:
        from .. import _build

        build_dir = _build.BUILD_DIR
    res = {}
    for obj in sorted(glob.glob(os.path.join(build_dir, "k_*.o"))):
        tu = os.path.basename(obj)[2:-2]
        ks = parse_kernels(code_object_notes(obj))
        for k, dn in zip(ks, demangle([k["name"] for k in ks])):
            k["demangled"] = dn
        res[tu] = ks
    return res


def offenders(kernels: dict[str, list[dict]]) -> list[tuple[str, str, dict]]:
    """Kernels with scratch or VGPR spills (memory traffic): (tu, demangled name, resources).
    SGPR spills are not counted: they go to VGPR lanes (v_writelane / v_readlane), not to
    memory, and the table shows them."""
    bad = []
    for tu, ks in kernels.items():
        for k in ks:
            if k.get("private_segment_fixed_size", 0) or k.get("vgpr_spill_count", 0):
                bad.append((tu, k.get("demangled", k["name"]), k))
    return bad


if __name__ == "__main__":
    for tu, ks in all_kernels().items():
        for k in ks:
            print(f"{tu:18s} vgpr {k.get('vgpr_count', '?'):>3} agpr {k.get('agpr_count', '?'):>3} "
                  f"scratch {k.get('private_segment_fixed_size', '?'):>5} spill {k.get('vgpr_spill_count', '?'):>3} "
                  f"sgpr-spill {k.get('sgpr_spill_count', '?'):>3} "
                  f"lds {k.get('group_segment_fixed_size', '?'):>6}  {k.get('demangled', k['name'])[:150]}")
