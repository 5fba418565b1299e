"""ctypes binding of the C ABI in include/lsmgpu.h (lsmdb_amd/liblsmgpu.so).

This is the same surface a cgo shim binds.  There is no fallback: if the
HIP library is missing, importing the codec fails loudly.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_int, c_int32, c_int64, c_uint8, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblsmgpu.so")
# diagnostics only: an alternate in-tree build (e.g. liblsmgpu_diag.so, LSMGPU_BUILD_DIAG=1)
if os.environ.get("LSMGPU_LIB_VARIANT"):
    LIB_PATH = os.path.join(_HERE, f"liblsmgpu_{os.environ['LSMGPU_LIB_VARIANT']}.so")

# ---- status codes (include/lsmgpu.h)
OK = 0
ERR_ARG = 1
ERR_BAD_TAIL = 2
ERR_CAPACITY = 3
ERR_HIP = 4
ERR_KEY_LEN = 5
ERR_VALUE_LEN = 6
ERR_TOO_LARGE = 7
ERR_INTERNAL = 8
ERR_NO_DEVICE = 9
ERR_CORRUPT = 10
ERR_HOST_PINNED = 11

BLK_OK = 0
BLK_VALUE_OVERFLOW = 1
BLK_FIRST_PLEN = 2
BLK_TRUNC_HEADER = 3
BLK_PREFIX_OOB = 4
BLK_RANGE = 5

MODE_MATERIALIZE = 1
MODE_VIEW = 2

# every symbol include/lsmgpu.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = (
    "lsmgpu_open",
    "lsmgpu_close",
    "lsmgpu_set_stream",
    "lsmgpu_get_stream",
    "lsmgpu_synchronize",
    "lsmgpu_set_kernel_timing",
    "lsmgpu_kernel_times",
    "lsmgpu_strerror",
    "lsmgpu_last_error",
    "lsmgpu_abi_version",
    "lsmgpu_parse_index",
    "lsmgpu_open_tables_async",
    "lsmgpu_merge_runs_async",
    "lsmgpu_cut_tables_async",
    "lsmgpu_encode_tables_async",
    "lsmgpu_bloom_params",
    "lsmgpu_bloom_build_async",
    "lsmgpu_bloom_json_async",
    "lsmgpu_bloom_has_async",
    "lsmgpu_cut_tables_ex_async",
    "lsmgpu_bloom_tables_async",
    "lsmgpu_encode_tables_gather_async",
    "lsmgpu_bloom_tables_gather_async",
    "lsmgpu_decode_blocks",
    "lsmgpu_decode_blocks_async",
    "lsmgpu_encode_blocks",
    "lsmgpu_encode_blocks_async",
    "lsmgpu_plan_blocks",
    "lsmgpu_encode_values",
    "lsmgpu_compact_tables",
    "lsmgpu_compact_result",
    "lsmgpu_stream_probe_async",
    "lsmgpu_host_register",
    "lsmgpu_host_unregister",
    "lsmgpu_host_alloc",
    "lsmgpu_host_free",
)

COMPACT_BLOOM = 1


class LsmgpuDecoded(ctypes.Structure):
    _fields_ = [
        ("key_data", c_void_p),
        ("key_cap", c_uint64),
        ("key_end", c_void_p),
        ("val_data", c_void_p),
        ("val_cap", c_uint64),
        ("val_end", c_void_p),
        ("view", c_void_p),
        ("ent_cap", c_uint64),
        ("blk_first", c_void_p),
        ("blk_status", c_void_p),
        ("n_entries", c_uint64),
        ("key_bytes", c_uint64),
        ("val_bytes", c_uint64),
        ("first_bad_block", c_int64),
        ("n_bad_blocks", c_uint64),
    ]


class Tables(ctypes.Structure):
    """lsmgpu_tables (include/lsmgpu.h): batched OpenTable outputs, device pointers."""
    _fields_ = [
        ("nblk", c_void_p),
        ("blk_base", c_void_p),
        ("bloom_off", c_void_p),
        ("bloom_len", c_void_p),
        ("status", c_void_p),
        ("smallest", c_void_p),
        ("biggest", c_void_p),
        ("blk_off", c_void_p),
        ("blk_len", c_void_p),
        ("key_off", c_void_p),
        ("key_len", c_void_p),
        ("order", c_void_p),
        ("blk_cap", c_uint64),
    ]


class Runs(ctypes.Structure):
    """lsmgpu_runs (include/lsmgpu.h): sorted runs of one key / value stream, device pointers."""
    _fields_ = [("key_data", c_void_p), ("key_end", c_void_p), ("val_data", c_void_p),
                ("val_end", c_void_p), ("run_first", c_void_p), ("nruns", c_uint32),
                ("n", c_uint64)]


class Merged(ctypes.Structure):
    """lsmgpu_merged (include/lsmgpu.h): merge output, device pointers."""
    _fields_ = [("key_data", c_void_p), ("key_cap", c_uint64), ("key_end", c_void_p),
                ("val_data", c_void_p), ("val_cap", c_uint64), ("val_end", c_void_p),
                ("src", c_void_p), ("ent_cap", c_uint64)]


class LsmgpuError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = _LIB.lsmgpu_strerror(code).decode() if _LIB is not None else str(code)
        if code == ERR_HIP and _LIB is not None and hasattr(_LIB, "lsmgpu_last_error"):
            msg += f" [{_LIB.lsmgpu_last_error().decode()}]"  # the failing HIP call
        super().__init__(f"{what}: {msg} (code {code})" if what else f"{msg} (code {code})")


def _load() -> ctypes.CDLL:
    # PyTorch ships its own HIP runtime (torch/lib/libamdhip64.so, soname libamdhip64.so.7).
    # Import it FIRST so liblsmgpu.so's libamdhip64.so.7 dependency binds to that same
    # runtime: one HIP runtime per process, so torch-allocated device buffers and streams are
    # valid in the codec (loading /opt/rocm's runtime first leaves torch with no devices).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP codec first (python -c "
            "'import __graft_entry__ as g; g.build()')"
        )
    lib = ctypes.CDLL(LIB_PATH)
    u8p, u32p, u64p = POINTER(c_uint8), POINTER(c_uint32), POINTER(c_uint64)
    del u8p, u32p, u64p
    lib.lsmgpu_open.argtypes = [c_int, POINTER(c_void_p)]
    lib.lsmgpu_open.restype = c_int
    lib.lsmgpu_close.argtypes = [c_void_p]
    lib.lsmgpu_close.restype = None
    lib.lsmgpu_set_stream.argtypes = [c_void_p, c_void_p]
    lib.lsmgpu_set_stream.restype = c_int
    lib.lsmgpu_get_stream.argtypes = [c_void_p]
    lib.lsmgpu_get_stream.restype = c_void_p
    lib.lsmgpu_synchronize.argtypes = [c_void_p]
    lib.lsmgpu_synchronize.restype = c_int
    lib.lsmgpu_set_kernel_timing.argtypes = [c_void_p, c_int]
    lib.lsmgpu_set_kernel_timing.restype = c_int
    lib.lsmgpu_kernel_times.argtypes = [c_void_p, ctypes.POINTER(ctypes.c_float),
                                        ctypes.POINTER(ctypes.c_float)]
    lib.lsmgpu_kernel_times.restype = c_int
    lib.lsmgpu_strerror.argtypes = [c_int]
    lib.lsmgpu_strerror.restype = ctypes.c_char_p
    if hasattr(lib, "lsmgpu_last_error"):
        lib.lsmgpu_last_error.argtypes = []
        lib.lsmgpu_last_error.restype = ctypes.c_char_p
    lib.lsmgpu_abi_version.argtypes = []
    lib.lsmgpu_abi_version.restype = c_int
    lib.lsmgpu_parse_index.argtypes = [c_void_p, c_uint64, c_void_p, c_void_p, c_uint64,
                                       POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64)]
    lib.lsmgpu_parse_index.restype = c_int
    lib.lsmgpu_decode_blocks.argtypes = [c_void_p, c_void_p, c_uint64, c_int, c_void_p, c_void_p,
                                         c_uint64, c_int, POINTER(LsmgpuDecoded)]
    lib.lsmgpu_decode_blocks.restype = c_int
    lib.lsmgpu_decode_blocks_async.argtypes = [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p,
                                               c_uint64, c_uint32, c_int, POINTER(LsmgpuDecoded),
                                               c_void_p]
    lib.lsmgpu_decode_blocks_async.restype = c_int
    lib.lsmgpu_encode_blocks.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64,
                                         c_int, c_uint32, c_uint32, c_void_p, c_uint64,
                                         POINTER(c_uint64), POINTER(c_uint64), c_void_p, c_uint64,
                                         POINTER(c_uint64)]
    lib.lsmgpu_encode_blocks.restype = c_int
    lib.lsmgpu_encode_blocks_async.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_uint64, c_uint32, c_void_p, c_uint64, c_uint64,
                                               c_uint64, c_void_p, c_uint64, c_void_p]
    lib.lsmgpu_encode_blocks_async.restype = c_int
    lib.lsmgpu_plan_blocks.argtypes = [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_void_p,
                                       c_uint64, POINTER(c_uint64)]
    lib.lsmgpu_plan_blocks.restype = c_int
    lib.lsmgpu_encode_values.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_uint64, c_int, c_void_p, c_uint64, c_void_p,
                                         POINTER(c_uint64)]
    lib.lsmgpu_encode_values.restype = c_int
    lib.lsmgpu_open_tables_async.argtypes = [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p,
                                             c_uint32, POINTER(Tables), c_void_p]
    lib.lsmgpu_open_tables_async.restype = c_int
    lib.lsmgpu_merge_runs_async.argtypes = [c_void_p, POINTER(Runs), POINTER(Merged), c_void_p]
    lib.lsmgpu_merge_runs_async.restype = c_int
    lib.lsmgpu_cut_tables_async.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, c_uint32,
                                            ctypes.c_int64, c_void_p, c_void_p, c_void_p,
                                            c_uint32, c_void_p]
    lib.lsmgpu_cut_tables_async.restype = c_int
    lib.lsmgpu_encode_tables_async.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_uint64, c_uint64, c_uint64, c_uint32, c_void_p,
                                               c_void_p, c_void_p, c_uint32, c_uint64, c_void_p,
                                               c_void_p]
    lib.lsmgpu_encode_tables_async.restype = c_int
    lib.lsmgpu_bloom_params.argtypes = [c_uint64, POINTER(c_uint64), POINTER(c_uint64),
                                        POINTER(c_uint64)]
    lib.lsmgpu_bloom_params.restype = c_int
    lib.lsmgpu_bloom_build_async.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p,
                                             c_uint64, c_uint64, c_void_p]
    lib.lsmgpu_bloom_build_async.restype = c_int
    lib.lsmgpu_bloom_json_async.argtypes = [c_void_p, c_void_p, c_uint64, c_uint64, c_void_p,
                                            c_uint64]
    lib.lsmgpu_bloom_json_async.restype = c_int
    lib.lsmgpu_bloom_has_async.argtypes = [c_void_p, c_void_p, c_uint64, c_uint64, c_void_p,
                                           c_void_p, c_uint64, c_void_p]
    lib.lsmgpu_bloom_has_async.restype = c_int
    lib.lsmgpu_cut_tables_ex_async.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, c_uint32,
                                               ctypes.c_int64, c_uint32, c_void_p, c_void_p,
                                               c_void_p, c_uint32, c_void_p]
    lib.lsmgpu_cut_tables_ex_async.restype = c_int
    lib.lsmgpu_bloom_tables_async.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_uint32, c_void_p, c_void_p, c_uint64, c_void_p]
    lib.lsmgpu_bloom_tables_async.restype = c_int
    lib.lsmgpu_encode_tables_gather_async.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p,
                                                      c_void_p, c_void_p, c_void_p, c_void_p,
                                                      c_uint64, c_uint64, c_uint64, c_uint32,
                                                      c_void_p, c_void_p, c_void_p, c_uint32,
                                                      c_uint64, c_void_p, c_void_p]
    lib.lsmgpu_encode_tables_gather_async.restype = c_int
    lib.lsmgpu_bloom_tables_gather_async.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p,
                                                     c_void_p, c_void_p, c_uint32, c_void_p,
                                                     c_void_p, c_uint64, c_void_p]
    lib.lsmgpu_bloom_tables_gather_async.restype = c_int
    lib.lsmgpu_compact_tables.argtypes = [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p,
                                          c_uint32, ctypes.c_int64, c_uint32, POINTER(c_uint64),
                                          POINTER(c_uint32)]
    lib.lsmgpu_compact_tables.restype = c_int
    lib.lsmgpu_compact_result.argtypes = [c_void_p, c_void_p, c_uint64, c_void_p, c_uint64]
    lib.lsmgpu_compact_result.restype = c_int
    lib.lsmgpu_stream_probe_async.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_uint64,
                                              c_uint32]
    lib.lsmgpu_stream_probe_async.restype = c_int
    if os.environ.get("LSMGPU_LIB_VARIANT") and not hasattr(lib, "lsmgpu_host_register"):
        return lib  # diagnostics: an earlier round's build (same-box A/B of its kernels)
    lib.lsmgpu_host_register.argtypes = [c_void_p, c_void_p, c_uint64]
    lib.lsmgpu_host_register.restype = c_int
    lib.lsmgpu_host_unregister.argtypes = [c_void_p, c_void_p]
    lib.lsmgpu_host_unregister.restype = c_int
    if hasattr(lib, "lsmgpu_host_alloc"):  # (ABI >= 4; diagnostics may load an older build)
        lib.lsmgpu_host_alloc.argtypes = [c_void_p, c_uint64, POINTER(c_void_p)]
        lib.lsmgpu_host_alloc.restype = c_int
        lib.lsmgpu_host_free.argtypes = [c_void_p, c_void_p]
        lib.lsmgpu_host_free.restype = c_int
    return lib


_LIB = None
_LIB = _load()


def lib() -> ctypes.CDLL:
    return _LIB


def check(code: int, what: str = "") -> None:
    if code != OK:
        raise LsmgpuError(code, what)


__all__ = [n for n in dir() if not n.startswith("__")]
_ = (c_int32,)
