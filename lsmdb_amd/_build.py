"""Build helpers: the HIP codec library (gfx950) and the CPU oracle (test infrastructure)."""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lsmdb_amd", "csrc")
LIB = os.path.join(ROOT, "lsmdb_amd", "liblsmgpu.so")
SOURCES = ["api.hip", "decode.hip", "decode_wsc.hip", "encode.hip", "open_tables.hip", "merge.hip", "bloom.hip", "probe.hip"]
HEADERS = ["codec_common.hpp", "decode_common.hpp", "kernels.hpp", os.path.join("..", "..", "include", "lsmgpu.h")]
ARCH = os.environ.get("LSMGPU_ARCH", "gfx950")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force: bool = False, verbose: bool = True) -> str:
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    if not force and not _stale(LIB, deps):
        return LIB
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-o", LIB] + [os.path.join(CSRC, s) for s in SOURCES]
    if os.environ.get("LSMGPU_BUILD_STAMPS"):  # diagnostic build: per-phase s_memtime stamps
        cmd.insert(1, "-DLSMGPU_STAMPS")
        cmd[cmd.index(LIB)] = LIB.replace("liblsmgpu.so", "liblsmgpu_stamps.so")
    if verbose:
        print("[build]", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    return LIB


def build_oracle(verbose: bool = True) -> str:
    out = os.path.join(ROOT, "oracle", "build", "libsstref.so")
    cmd = ["make", "-C", os.path.join(ROOT, "oracle"), "-s"]
    if verbose:
        print("[build]", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    build_lib(force="--force" in sys.argv)
    build_oracle()
