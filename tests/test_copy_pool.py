"""CPU check of the parallel memcpy behind the library's host staging
(lsmdb_amd/csrc/copy_pool.hpp, used by host_io.hpp for pageable .sst bytes and output arrays --
a Go heap buffer under LoadToRAM, table/table.go:117-123,329-338): random sizes and offsets,
several pool sizes, pools reused across copies, every byte compared.  No GPU."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_copy_pool(tmp_path):
    exe = tmp_path / "copy_pool_check"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-pthread", "-I",
                    os.path.join(ROOT, "lsmdb_amd", "csrc"),
                    os.path.join(ROOT, "tests", "copy_pool_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "60"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads(out.stdout)
    assert r["fails"] == 0 and r["copies"] == 300
