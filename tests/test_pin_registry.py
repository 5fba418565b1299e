"""CPU model check of the host-pinning registry behind lsmgpu_host_register
(lsmdb_amd/csrc/pin_registry.hpp): overlapping, page-sharing, nested, repeated and re-used
ranges never pin a page twice, keep every live range's pages pinned, unpin nothing another range
still uses, and leak nothing; host copies are cut so no piece crosses a pinned segment's border.
The reference's default LoadToRAM mode makes Table.mmap a Go heap buffer (options.go:76,
table/table.go:117-123,329-338): exactly such ranges.  No GPU."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pin_registry_model(tmp_path):
    exe = tmp_path / "pin_registry_check"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "lsmdb_amd", "csrc"),
                    os.path.join(ROOT, "tests", "pin_registry_check.cpp"), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe), "20000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads(out.stdout)
    assert r["fails"] == 0 and r["registers"] > 5000 and r["unregisters"] > 5000
    assert r["recuts"] > 20  # segments shared in part by several ranges were re-cut
