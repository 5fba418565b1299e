"""Build helpers: the HIP codec library (gfx950) and the CPU oracle (test infrastructure)."""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lsmdb_amd", "csrc")
LIB = os.path.join(ROOT, "lsmdb_amd", "liblsmgpu.so")
SOURCES = ["api.hip", "decode.hip", "decode_wsc.hip", "encode.hip", "open_tables.hip", "merge.hip", "bloom.hip", "probe.hip"]
HEADERS = ["codec_common.hpp", "decode_common.hpp", "kernels.hpp", "host_io.hpp", "copy_pool.hpp",
           os.path.join("..", "..", "include", "lsmgpu.h")]
ARCH = os.environ.get("LSMGPU_ARCH", "gfx950")
FLAGS = ("hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def compile_cmd(flags: list[str], src: str, out: str, flavor: str) -> list[str]:
    """hipcc line for one source.  A fixed compilation-unit id: clang derives __hip_cuid_* from
    the (per-process temporary) output path otherwise, so every rebuild would change the
    library's sha256 -- the key of profiles/pmc_traffic.json (tests/test_build.py)."""
    cuid = f"-cuid=lsmgpu_{flavor}_{os.path.splitext(src)[0]}"
    return flags + [cuid, "-c", "-o", out, os.path.join(CSRC, src)]


def build_lib(force: bool = False, verbose: bool = True) -> str:
    """Each source compiled to its own object in parallel, then one link.  Every flavor (the
    product library, the LSMGPU_BUILD_DIAG diagnostic one) has its own object directory, and
    objects and the library are written to temporary names renamed into place, so two builds at
    once (two bench ranks, two test processes) never read each other's half-written files."""
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    flags = list(FLAGS)
    lib, flavor = LIB, "default"
    # the diagnostic build (kernels.hpp): the rejected variants, A/B knobs, timing ablations and
    # per-phase s_memtime stamps; the product library compiles only the adopted paths
    if os.environ.get("LSMGPU_BUILD_DIAG") or os.environ.get("LSMGPU_BUILD_STAMPS"):
        flags.append("-DLSMGPU_DIAG")
        lib, flavor = LIB.replace("liblsmgpu.so", "liblsmgpu_diag.so"), "diag"
    if not force and not _stale(lib, deps):
        return lib
    objdir = os.path.join(ROOT, "lsmdb_amd", "build", flavor)
    os.makedirs(objdir, exist_ok=True)
    tag = f".{os.getpid()}.tmp"
    jobs, objs = [], []
    for s in SOURCES:
        obj = os.path.join(objdir, os.path.splitext(s)[0] + ".o")
        objs.append(obj)
        cmd = compile_cmd(flags, s, obj + tag, flavor)
        if verbose:
            print("[build]", " ".join(cmd), file=sys.stderr)
        jobs.append(subprocess.Popen(cmd, cwd=CSRC))
    codes = [j.wait() for j in jobs]  # every job finishes before any error is raised
    if any(codes):
        for o in objs:
            if os.path.exists(o + tag):
                os.remove(o + tag)
        raise subprocess.CalledProcessError(max(codes), "hipcc")
    for o in objs:
        os.replace(o + tag, o)
    cmd = flags + ["-shared", "-o", lib + tag] + objs
    if verbose:
        print("[build]", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(lib + tag, lib)
    return lib


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
