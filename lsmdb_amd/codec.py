"""Python face of the HIP SST block codec (C ABI: include/lsmgpu.h).

`Codec` owns one `lsmgpu_ctx` (HIP stream + look-back scratch) on one device.  Two families:

* host-buffer calls (`decode_host`, `encode_host`, `encode_values_host`): the library stages
  through HBM -- the path a cgo caller with an mmap'd .sst takes;
* device-resident calls (`decode_device_async`, `encode_device_async`): every pointer is a
  torch CUDA tensor; nothing is synchronised (what bench.py times).

No CPU fallback exists: every call runs the gfx950 kernels or raises.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_uint64, c_void_p
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _lib
from ._lib import (LsmgpuDecoded, LsmgpuError, MODE_MATERIALIZE, MODE_VIEW, check, lib)


def _ptr(a) -> Optional[int]:
    """Address of a numpy array / torch tensor / bytes-like (None passes through)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data if a.size else (a.ctypes.data or None)
    if hasattr(a, "data_ptr"):
        return a.data_ptr() or None
    raise TypeError(f"unsupported buffer type {type(a)}")


def _np_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data.view(np.uint8).reshape(-1))
    return np.frombuffer(memoryview(data), dtype=np.uint8)


# ------------------------------------------------------------------ table.go:177-215
def parse_index(sst) -> tuple[np.ndarray, np.ndarray, int, int]:
    """Table.readIndex's tail parse: returns (blk_off, blk_len, bloom_off, bloom_len)."""
    buf = _np_u8(sst)
    n = c_uint64(0)
    bo, bl = c_uint64(0), c_uint64(0)
    rc = lib().lsmgpu_parse_index(_ptr(buf), buf.size, None, None, 0, byref(n), byref(bo), byref(bl))
    if rc not in (_lib.OK, _lib.ERR_CAPACITY):
        raise LsmgpuError(rc, "parse_index")
    off = np.zeros(max(n.value, 1), dtype=np.uint32)
    ln = np.zeros(max(n.value, 1), dtype=np.uint32)
    check(lib().lsmgpu_parse_index(_ptr(buf), buf.size, _ptr(off), _ptr(ln), off.size, byref(n),
                                   byref(bo), byref(bl)), "parse_index")
    return off[: n.value], ln[: n.value], bo.value, bl.value


def plan_blocks(key_end: np.ndarray, vs_end: np.ndarray, entries_per_block: int = 100,
                block_bytes: int = 0) -> np.ndarray:
    """Block plan (first entry of each block + end sentinel) of Builder.Add's cut rule."""
    ke = np.ascontiguousarray(key_end, dtype=np.uint32)
    ve = np.ascontiguousarray(vs_end, dtype=np.uint32)
    nb = c_uint64(0)
    check(lib().lsmgpu_plan_blocks(_ptr(ke), _ptr(ve), ke.size, entries_per_block, block_bytes,
                                   None, 0, byref(nb)), "plan_blocks")
    out = np.zeros(nb.value + 1, dtype=np.uint32)
    check(lib().lsmgpu_plan_blocks(_ptr(ke), _ptr(ve), ke.size, entries_per_block, block_bytes,
                                   _ptr(out), out.size, byref(nb)), "plan_blocks")
    return out


@dataclass
class HostDecoded:
    """A decoded batch in host memory (SoA, Table.Iterator order)."""
    n_entries: int
    key_data: np.ndarray
    key_end: np.ndarray
    val_data: np.ndarray
    val_end: np.ndarray
    view: Optional[np.ndarray]
    blk_first: np.ndarray
    blk_status: np.ndarray
    first_bad_block: int
    n_bad_blocks: int

    def key(self, i: int) -> bytes:
        a = int(self.key_end[i - 1]) if i else 0
        return self.key_data[a: int(self.key_end[i])].tobytes()

    def value(self, i: int) -> bytes:
        a = int(self.val_end[i - 1]) if i else 0
        return self.val_data[a: int(self.val_end[i])].tobytes()


@dataclass
class DeviceDecodeBuffers:
    """Device output buffers of a decode (torch CUDA tensors); built by Codec.alloc_decode."""
    key_data: object = None
    key_end: object = None
    val_data: object = None
    val_end: object = None
    view: object = None
    blk_first: object = None
    blk_status: object = None
    result: object = None
    ent_cap: int = 0
    struct: LsmgpuDecoded = field(default_factory=LsmgpuDecoded)

    def bind(self) -> LsmgpuDecoded:
        s = self.struct
        s.key_data = _ptr(self.key_data)
        s.key_cap = self.key_data.numel() if self.key_data is not None else 0
        s.key_end = _ptr(self.key_end)
        s.val_data = _ptr(self.val_data)
        s.val_cap = self.val_data.numel() if self.val_data is not None else 0
        s.val_end = _ptr(self.val_end)
        s.view = _ptr(self.view)
        s.ent_cap = self.ent_cap
        s.blk_first = _ptr(self.blk_first)
        s.blk_status = _ptr(self.blk_status)
        return s


class Codec:
    """One lsmgpu_ctx on one HIP device (use one per thread, like a Go Builder/Iterator)."""

    def __init__(self, device: int = 0):
        self.device = device
        self._ctx = c_void_p()
        check(lib().lsmgpu_open(device, byref(self._ctx)), f"lsmgpu_open({device})")

    # -- lifecycle
    def close(self) -> None:
        if self._ctx:
            lib().lsmgpu_close(self._ctx)
            self._ctx = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_stream(self, stream_handle: Optional[int]) -> None:
        check(lib().lsmgpu_set_stream(self._ctx, stream_handle), "set_stream")

    def stream_handle(self) -> int:
        return lib().lsmgpu_get_stream(self._ctx) or 0

    def synchronize(self) -> None:
        check(lib().lsmgpu_synchronize(self._ctx), "synchronize")

    # -- diagnostics: per-kernel HIP-event timing of walk-scan-copy decodes
    def set_kernel_timing(self, on: bool) -> None:
        check(lib().lsmgpu_set_kernel_timing(self._ctx, 1 if on else 0), "set_kernel_timing")

    def kernel_times(self) -> tuple:
        """(walk ms, copy ms) of the last timed walk-scan-copy decode (waits for it)."""
        import ctypes
        w, c = ctypes.c_float(), ctypes.c_float()
        check(lib().lsmgpu_kernel_times(self._ctx, ctypes.byref(w), ctypes.byref(c)),
              "kernel_times")
        return float(w.value), float(c.value)

    def stream_probe_async(self, kind: int, src, dst, nbytes: int, wg_per_cu: int) -> None:
        """Diagnostics: a streaming copy (kind 0 / 2 nt) or read (1 / 3 nt) of nbytes."""
        check(lib().lsmgpu_stream_probe_async(self._ctx, kind, _ptr(src), _ptr(dst), nbytes,
                                              wg_per_cu), "stream_probe_async")

    # -- host memory.  Pageable arrays are staged through the ctx's own page-locked buffers;
    # host_alloc memory is DMA'd directly (include/lsmgpu.h, ABI 4)
    def host_alloc(self, nbytes: int) -> np.ndarray:
        """A u8 array of nbytes in page-locked memory (lsmgpu_host_alloc), freed with the array."""
        import weakref
        p = c_void_p()
        check(lib().lsmgpu_host_alloc(self._ctx, max(int(nbytes), 1), byref(p)), "host_alloc")
        buf = (ctypes.c_uint8 * max(int(nbytes), 1)).from_address(p.value)
        weakref.finalize(buf, lib().lsmgpu_host_free, None, p.value)
        return np.frombuffer(buf, np.uint8, count=int(nbytes))

    def host_register(self, arr) -> None:
        """ABI-3 compatibility: records the array's range (nothing is page-locked)."""
        check(lib().lsmgpu_host_register(self._ctx, _ptr(arr), arr.nbytes), "host_register")

    def host_unregister(self, arr) -> None:
        check(lib().lsmgpu_host_unregister(self._ctx, _ptr(arr)), "host_unregister")

    # -- decode, host buffers (table.Table path)
    def _host_zeros(self, n: int, dtype, pinned: bool) -> np.ndarray:
        if not pinned:
            return np.zeros(n, dtype=dtype)
        a = self.host_alloc(max(n, 1) * np.dtype(dtype).itemsize).view(dtype)[:n]
        a[:] = 0
        return a

    def decode_host(self, data, blk_off: np.ndarray, blk_len: np.ndarray,
                    mode: int = MODE_MATERIALIZE | MODE_VIEW, pinned_out: bool = False) -> HostDecoded:
        """pinned_out: the output arrays live in host_alloc memory (DMA'd directly, no staging)."""
        buf = _np_u8(data)
        off = np.ascontiguousarray(blk_off, dtype=np.uint32)
        ln = np.ascontiguousarray(blk_len, dtype=np.uint32)
        nblk = off.size
        key_cap = val_cap = max(int(buf.size), 16)
        ent_cap = max(int(ln.astype(np.uint64).sum()) // 10 + 1, 1)
        # MODE_VIEW alone: the view index only (key/value arrays come back empty); any other
        # mode also materializes, so the HostDecoded accessors work
        eff = mode if mode == MODE_VIEW else mode | MODE_MATERIALIZE
        for _attempt in range(2):
            z = lambda n, t: self._host_zeros(n, t, pinned_out)  # noqa: E731
            kd = z(key_cap, np.uint8)
            vd = z(val_cap, np.uint8)
            ke = z(ent_cap, np.uint32)
            ve = z(ent_cap, np.uint32)
            vw = z(ent_cap, np.uint64) if mode & MODE_VIEW else None
            bf = z(nblk + 1, np.uint32)
            bs = z(max(nblk, 1), np.int32)
            d = LsmgpuDecoded()
            d.key_data, d.key_cap, d.key_end = _ptr(kd), kd.size, _ptr(ke)
            d.val_data, d.val_cap, d.val_end = _ptr(vd), vd.size, _ptr(ve)
            d.view, d.ent_cap = _ptr(vw), ent_cap
            d.blk_first, d.blk_status = _ptr(bf), _ptr(bs)
            rc = lib().lsmgpu_decode_blocks(self._ctx, _ptr(buf), buf.size, 0, _ptr(off), _ptr(ln),
                                            nblk, eff, byref(d))
            if rc == _lib.ERR_CAPACITY:  # plen>0 blocks can expand keys: retry with exact sizes
                key_cap = max(int(d.key_bytes), 16)
                val_cap = max(int(d.val_bytes), 16)
                ent_cap = max(int(d.n_entries), 1)
                continue
            check(rc, "decode_blocks")
            n = int(d.n_entries)
            return HostDecoded(n, kd[: d.key_bytes], ke[:n], vd[: d.val_bytes], ve[:n],
                               vw[:n] if vw is not None else None, bf, bs[:nblk],
                               int(d.first_bad_block), int(d.n_bad_blocks))
        raise LsmgpuError(_lib.ERR_CAPACITY, "decode_blocks")

    # -- decode, device-resident (benchmarked path)
    def alloc_decode(self, data_len: int, total_block_bytes: int, nblk: int, mode: int,
                     ent_cap: Optional[int] = None):
        import torch
        dev = torch.device("cuda", self.device)
        ent_cap = ent_cap if ent_cap is not None else total_block_bytes // 10 + 1
        b = DeviceDecodeBuffers(ent_cap=ent_cap)
        if mode & MODE_MATERIALIZE:
            b.key_data = torch.empty(max(total_block_bytes, 16), dtype=torch.uint8, device=dev)
            b.val_data = torch.empty(max(total_block_bytes, 16), dtype=torch.uint8, device=dev)
            b.key_end = torch.empty(ent_cap, dtype=torch.int32, device=dev)
            b.val_end = torch.empty(ent_cap, dtype=torch.int32, device=dev)
        if mode & MODE_VIEW:
            b.view = torch.empty(ent_cap, dtype=torch.int64, device=dev)
        b.blk_first = torch.empty(nblk + 1, dtype=torch.int32, device=dev)
        b.blk_status = torch.empty(max(nblk, 1), dtype=torch.int32, device=dev)
        b.result = torch.zeros(8, dtype=torch.int64, device=dev)
        b.bind()
        return b

    def decode_device_async(self, data, blk_off, blk_len, max_blk_len: int, mode: int,
                            bufs: DeviceDecodeBuffers, data_len: Optional[int] = None) -> None:
        n = blk_off.numel()
        dl = data.numel() if data_len is None else data_len
        check(lib().lsmgpu_decode_blocks_async(self._ctx, _ptr(data), dl, _ptr(blk_off),
                                               _ptr(blk_len), n, max_blk_len, mode,
                                               byref(bufs.struct), _ptr(bufs.result)),
              "decode_blocks_async")

    # -- encode
    def encode_host(self, keys, key_end, vs, vs_end, entries_per_block: int = 100,
                    block_bytes: int = 0):
        """Builder.Add x n + Finish (minus bloom): returns (sst_without_bloom, data_len, restarts)."""
        kb = _np_u8(keys) if len(keys) else np.zeros(1, np.uint8)
        vb = _np_u8(vs) if len(vs) else np.zeros(1, np.uint8)
        ke = np.ascontiguousarray(key_end, dtype=np.uint32)
        ve = np.ascontiguousarray(vs_end, dtype=np.uint32)
        n = ke.size
        out_len, data_len, nr = c_uint64(0), c_uint64(0), c_uint64(0)
        rc = lib().lsmgpu_encode_blocks(self._ctx, _ptr(kb), _ptr(ke), _ptr(vb), _ptr(ve), n, 0,
                                        entries_per_block, block_bytes, _ptr(np.zeros(1, np.uint8)),
                                        0, byref(out_len), byref(data_len), None, 0, byref(nr))
        if rc != _lib.ERR_CAPACITY:
            check(rc, "encode_blocks")
        out = np.zeros(out_len.value, dtype=np.uint8)
        rs = np.zeros(max(nr.value, 1), dtype=np.uint32)
        check(lib().lsmgpu_encode_blocks(self._ctx, _ptr(kb), _ptr(ke), _ptr(vb), _ptr(ve), n, 0,
                                         entries_per_block, block_bytes, _ptr(out), out.size,
                                         byref(out_len), byref(data_len), _ptr(rs), rs.size,
                                         byref(nr)), "encode_blocks")
        return out.tobytes(), int(data_len.value), rs[: nr.value]

    def encode_device_async(self, keys, key_end, vs, vs_end, n: int, key_total: int,
                            vs_total: int, out, flags, entries_per_block: int = 100,
                            blk_first=None, nblocks: int = 0) -> None:
        check(lib().lsmgpu_encode_blocks_async(self._ctx, _ptr(keys), _ptr(key_end), _ptr(vs),
                                               _ptr(vs_end), n, entries_per_block,
                                               _ptr(blk_first), nblocks, key_total, vs_total,
                                               _ptr(out), out.numel(), _ptr(flags)),
              "encode_blocks_async")

    def encode_values_host(self, meta, user_meta, expires_at, values, value_end):
        """ValueStruct.EncodeTo for a batch: returns (vs bytes, vs_end)."""
        m = np.ascontiguousarray(meta, dtype=np.uint8)
        um = np.ascontiguousarray(user_meta, dtype=np.uint8)
        ex = np.ascontiguousarray(expires_at, dtype=np.uint64)
        vb = _np_u8(values) if len(values) else np.zeros(1, np.uint8)
        ve = np.ascontiguousarray(value_end, dtype=np.uint32)
        n = m.size
        if n == 0:
            return b"", np.zeros(0, np.uint32)
        cap = int(ve[-1]) + 12 * n + 16
        out = np.zeros(cap, dtype=np.uint8)
        end = np.zeros(n, dtype=np.uint32)
        ln = c_uint64(0)
        check(lib().lsmgpu_encode_values(self._ctx, _ptr(m), _ptr(um), _ptr(ex), _ptr(vb), _ptr(ve),
                                         n, 0, _ptr(out), out.size, _ptr(end), byref(ln)),
              "encode_values")
        return out[: ln.value].tobytes(), end


    # -- batched table open (OpenTable index work, table.go:88-144,177-269)
    def open_tables_device(self, data, sst_off, sst_len, blk_cap: int) -> dict:
        """ntables SSTs resident in `data` (device u8 tensor), table t = data[sst_off[t]:
        +sst_len[t]] (device i64 tensors).  Returns the device output tensors (asynchronous on
        the codec's stream); see lsmgpu_tables in include/lsmgpu.h."""
        import torch
        dev = data.device
        nt = sst_off.numel()
        i32 = dict(dtype=torch.int32, device=dev)
        o = dict(nblk=torch.empty(max(nt, 1), **i32), blk_base=torch.empty(nt + 1, **i32),
                 bloom_off=torch.empty(max(nt, 1), **i32), bloom_len=torch.empty(max(nt, 1), **i32),
                 status=torch.empty(max(nt, 1), **i32), smallest=torch.empty(3 * max(nt, 1), **i32),
                 biggest=torch.empty(5 * max(nt, 1), **i32),
                 blk_off=torch.empty(max(blk_cap, 1), **i32), blk_len=torch.empty(max(blk_cap, 1), **i32),
                 key_off=torch.empty(max(blk_cap, 1), **i32), key_len=torch.empty(max(blk_cap, 1), **i32),
                 order=torch.empty(max(blk_cap, 1), **i32),
                 result=torch.zeros(8, dtype=torch.int64, device=dev))
        st = _lib.Tables(*[_ptr(o[k]) for k in ("nblk", "blk_base", "bloom_off", "bloom_len", "status",
                                                "smallest", "biggest", "blk_off", "blk_len",
                                                "key_off", "key_len", "order")], blk_cap)
        check(lib().lsmgpu_open_tables_async(self._ctx, _ptr(data), data.numel(), _ptr(sst_off),
                                             _ptr(sst_len), nt, byref(st), _ptr(o["result"])),
              "open_tables_async")
        return o

    def open_tables_host(self, ssts, blk_cap: Optional[int] = None) -> list:
        """OpenTable's index work for a list of SST images (bytes) in one batch on the GPU.
        Per table: status, nblk, bloom span, blk_off/blk_len/key_off/key_len/order (numpy,
        table-relative), smallest / biggest (bytes or None)."""
        import torch
        raws = [bytes(x) for x in ssts]
        offs, pos = [], 0
        for r in raws:
            offs.append(pos)
            pos += len(r)
        buf = np.frombuffer(b"".join(raws) + b"\0" * 16, np.uint8)
        if blk_cap is None:
            blk_cap = sum(max(len(r) // 13, 1) for r in raws)  # a block is >= 13 B
        d = torch.from_numpy(buf.copy()).to(self.device)
        d_off = torch.tensor(offs, dtype=torch.int64, device=self.device)
        d_len = torch.tensor([len(r) for r in raws], dtype=torch.int64, device=self.device)
        o = self.open_tables_device(d, d_off, d_len, blk_cap)
        self.synchronize()
        h = {k: v.cpu().numpy().view(np.uint32) for k, v in o.items() if k != "result"}
        out = []
        for t, r in enumerate(raws):
            b0, b1 = int(h["blk_base"][t]), int(h["blk_base"][t + 1])
            stt = int(h["status"].view(np.int32)[t])
            sm, bg = h["smallest"][3 * t: 3 * t + 3], h["biggest"][5 * t: 5 * t + 5]
            ok = stt in (0, 6)
            out.append(dict(
                status=stt, nblk=int(h["nblk"][t]), bloom_off=int(h["bloom_off"][t]),
                bloom_len=int(h["bloom_len"][t]),
                blk_off=h["blk_off"][b0:b1].copy() if ok else None,
                blk_len=h["blk_len"][b0:b1].copy() if ok else None,
                key_off=h["key_off"][b0:b1].copy() if ok else None,
                key_len=h["key_len"][b0:b1].copy() if ok else None,
                order=h["order"][b0:b1].copy() if ok else None,
                smallest=r[int(sm[1]): int(sm[1]) + int(sm[2])] if ok and sm[0] else None,
                biggest=(r[int(bg[1]): int(bg[1]) + int(bg[2])] + r[int(bg[3]): int(bg[3]) + int(bg[4])])
                if ok and bg[0] else None))
        return out


    # -- k-way merge (MergeIterator, y/iterator.go:74-202)
    def merge_device(self, key_data, key_end, val_data, val_end, run_first, n: int,
                     gather: bool = True) -> dict:
        """Sorted runs [run_first[r], run_first[r+1]) of one device SoA stream -> merged SoA
        (asynchronous).  Returns device tensors key_data/key_end/val_data/val_end/src/result."""
        import torch
        dev = key_end.device
        kcap = int(key_data.numel()) if gather else 0
        vcap = int(val_data.numel()) if gather and val_data is not None else 0
        o = dict(key_end=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                 val_end=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                 src=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                 key_data=torch.empty(max(kcap, 16), dtype=torch.uint8, device=dev) if gather else None,
                 val_data=torch.empty(max(vcap, 16), dtype=torch.uint8, device=dev) if vcap else None,
                 result=torch.zeros(8, dtype=torch.int64, device=dev))
        runs = _lib.Runs(_ptr(key_data), _ptr(key_end), _ptr(val_data), _ptr(val_end),
                         _ptr(run_first), run_first.numel() - 1, n)
        out = _lib.Merged(_ptr(o["key_data"]), kcap, _ptr(o["key_end"]), _ptr(o["val_data"]),
                          vcap, _ptr(o["val_end"]), _ptr(o["src"]), max(n, 1))
        check(lib().lsmgpu_merge_runs_async(self._ctx, byref(runs), byref(out), _ptr(o["result"])),
              "merge_runs_async")
        return o

    def merge_host(self, key_data, key_end, val_data, val_end, run_first):
        """Host arrays in, host arrays out: (keys bytes, key_end, vals bytes, val_end, src,
        flags)."""
        import torch
        ke = np.ascontiguousarray(key_end, dtype=np.uint32)
        ve = np.ascontiguousarray(val_end, dtype=np.uint32)
        rf = np.ascontiguousarray(run_first, dtype=np.uint32)
        n = int(rf[-1])
        t = lambda a, dt: torch.from_numpy(np.array(a, copy=True).view(dt)).to(self.device)
        kd = t(np.frombuffer(bytes(key_data) + b"\0" * 16, np.uint8), np.uint8)
        vd = t(np.frombuffer(bytes(val_data) + b"\0" * 16, np.uint8), np.uint8)
        o = self.merge_device(kd, t(ke, np.int32), vd, t(ve, np.int32), t(rf, np.int32), n)
        self.synchronize()
        r = o["result"].cpu().numpy()
        m, kb, vb = int(r[0]), int(r[1]), int(r[2])
        return (o["key_data"][:kb].cpu().numpy().tobytes(),
                o["key_end"][:m].cpu().numpy().view(np.uint32),
                o["val_data"][:vb].cpu().numpy().tobytes(),
                o["val_end"][:m].cpu().numpy().view(np.uint32),
                o["src"][:m].cpu().numpy().view(np.uint32), int(r[3]))


    # -- compaction output tables (Builder.ReachedCapacity cut + one encode over every table)
    def cut_tables_device(self, key_end, vs_end, n: int, cap: int, entries_per_block: int = 100,
                          tables_cap: int = 4096, bloom: bool = False) -> dict:
        """lsmgpu_cut_tables_ex_async (asynchronous): device tensors tbl_first / tbl_blk /
        tbl_out / result; bloom=True reserves each table's bloom tail (complete .sst files)."""
        import torch
        dev = key_end.device
        o = dict(tbl_first=torch.empty(tables_cap + 1, dtype=torch.int32, device=dev),
                 tbl_blk=torch.empty(tables_cap + 1, dtype=torch.int32, device=dev),
                 tbl_out=torch.empty(tables_cap + 1, dtype=torch.int64, device=dev),
                 result=torch.zeros(8, dtype=torch.int64, device=dev),
                 tables_cap=tables_cap, epb=entries_per_block, n=n)
        check(lib().lsmgpu_cut_tables_ex_async(self._ctx, _ptr(key_end), _ptr(vs_end), n,
                                               entries_per_block, cap, 1 if bloom else 0,
                                               _ptr(o["tbl_first"]), _ptr(o["tbl_blk"]),
                                               _ptr(o["tbl_out"]), tables_cap, _ptr(o["result"])),
              "cut_tables_ex_async")
        o["bloom"] = bloom
        return o

    def bloom_tables_device(self, cut: dict, keys, key_end, out, flags, src=None) -> None:
        """Fill the bloom tails of a bloom=True cut's tables (after encode_tables_device);
        reads the cut's small tbl_first / tbl_out arrays back to the host (synchronizes).
        src: gather mode -- key i of the tables is key src[i] of keys / key_end
        (lsmgpu_bloom_tables_gather_async)."""
        import torch
        nt = int(cut["ntables"])
        if "bloom_host" not in cut:  # the cut's arrays on the host, once
            tf = cut["tbl_first"][: nt + 1].cpu().numpy().view(np.uint32).copy()
            to = cut["tbl_out"][: nt + 1].cpu().numpy().view(np.uint64).copy()
            per = [bloom_params(int(tf[t + 1] - tf[t]))[0] // 64 for t in range(nt)]
            words = max([sum(per[g: g + 32]) for g in range(0, nt, 32)], default=8)
            # the scratch stays alive with the cut (the stream may still be using it)
            cut["bloom_host"] = (tf, to, words,
                                 torch.empty(words, dtype=torch.int64, device=key_end.device))
        tf, to, words, scratch = cut["bloom_host"]
        if src is not None:
            check(lib().lsmgpu_bloom_tables_gather_async(self._ctx, _ptr(keys), _ptr(key_end),
                                                         _ptr(src), _ptr(tf), _ptr(to), nt,
                                                         _ptr(out), _ptr(scratch), words,
                                                         _ptr(flags)), "bloom_tables_gather_async")
            return
        check(lib().lsmgpu_bloom_tables_async(self._ctx, _ptr(keys), _ptr(key_end), _ptr(tf),
                                              _ptr(to), nt, _ptr(out), _ptr(scratch), words,
                                              _ptr(flags)), "bloom_tables_async")

    def encode_tables_device(self, cut: dict, keys, key_end, vs, vs_end, key_total: int,
                             vs_total: int, out, flags) -> None:
        """lsmgpu_encode_tables_async over a cut (asynchronous)."""
        n, epb, tc = cut["n"], cut["epb"], cut["tables_cap"]
        check(lib().lsmgpu_encode_tables_async(self._ctx, _ptr(keys), _ptr(key_end), _ptr(vs),
                                               _ptr(vs_end), n, key_total, vs_total, epb,
                                               _ptr(cut["tbl_first"]), _ptr(cut["tbl_blk"]),
                                               _ptr(cut["tbl_out"]), tc, (n + epb - 1) // epb + tc,
                                               _ptr(out), _ptr(flags)), "encode_tables_async")

    def encode_tables_gather_device(self, cut: dict, keys, key_end, vs, vs_end, src,
                                    out_key_end, out_vs_end, key_total: int, vs_total: int, out,
                                    flags) -> None:
        """lsmgpu_encode_tables_gather_async over a cut (asynchronous): table entry i is source
        entry src[i] of keys / key_end, vs / vs_end, placed by the merged ends out_key_end /
        out_vs_end (a merge_device(..., gather=False) output)."""
        n, epb, tc = cut["n"], cut["epb"], cut["tables_cap"]
        check(lib().lsmgpu_encode_tables_gather_async(
            self._ctx, _ptr(keys), _ptr(key_end), _ptr(vs), _ptr(vs_end), _ptr(src),
            _ptr(out_key_end), _ptr(out_vs_end), n, key_total, vs_total, epb,
            _ptr(cut["tbl_first"]), _ptr(cut["tbl_blk"]), _ptr(cut["tbl_out"]), tc,
            (n + epb - 1) // epb + tc, _ptr(out), _ptr(flags)), "encode_tables_gather_async")

    def compact_tables_device(self, keys, key_end, vs, vs_end, n: int, key_total: int,
                              vs_total: int, cap: int, entries_per_block: int = 100,
                              tables_cap: int = 4096, bloom: bool = False) -> dict:
        """Cut the sorted stream into compactBuildTables' output tables and encode them all;
        synchronizes once to size the output.  Returns device tensors: out (images back to
        back -- complete .sst files with bloom=True), tbl_first / tbl_blk / tbl_out, result,
        flags (bloom: bloom_flags)."""
        import torch
        o = self.cut_tables_device(key_end, vs_end, n, cap, entries_per_block, tables_cap, bloom)
        self.synchronize()
        r = o["result"].cpu().numpy()
        if r[3]:
            raise LsmgpuError(_lib.ERR_CAPACITY, "cut_tables: more tables than tables_cap")
        o["ntables"], o["bytes"] = int(r[0]), int(r[2])
        o["out"] = torch.empty(max(o["bytes"], 16) + 16, dtype=torch.uint8, device=key_end.device)
        o["flags"] = torch.zeros(4, dtype=torch.int32, device=key_end.device)
        self.encode_tables_device(o, keys, key_end, vs, vs_end, key_total, vs_total, o["out"],
                                  o["flags"])
        if bloom:
            o["bloom_flags"] = torch.zeros(1, dtype=torch.int32, device=key_end.device)
            self.bloom_tables_device(o, keys, key_end, o["out"], o["bloom_flags"])
        return o

    # -- the whole compaction data path for host tables (levels.go:239-298)
    def compact_host(self, ssts, run_first, max_table_size: int, bloom: bool = False) -> list:
        """compactBuildTables' data path in one call (lsmgpu_compact_tables): input .sst images
        (bytes), iterator r = tables [run_first[r], run_first[r+1]) in MergeIterator order;
        returns the output tables' images (complete .sst files with bloom=True, else Finish
        minus the bloom tail)."""
        raws = [np.frombuffer(bytes(x) + b"\0", np.uint8) for x in ssts]
        ptrs = (ctypes.c_void_p * max(len(raws), 1))(*[_ptr(r) for r in raws])
        lens = np.array([r.size - 1 for r in raws] or [0], dtype=np.uint64)
        rf = np.ascontiguousarray(run_first, dtype=np.uint32)
        out_len, nt = c_uint64(0), ctypes.c_uint32(0)
        check(lib().lsmgpu_compact_tables(self._ctx, ptrs, _ptr(lens), len(raws), _ptr(rf),
                                          rf.size - 1, max_table_size,
                                          _lib.COMPACT_BLOOM if bloom else 0, byref(out_len),
                                          byref(nt)), "compact_tables")
        out = np.zeros(max(out_len.value, 1), dtype=np.uint8)
        offs = np.zeros(nt.value + 1, dtype=np.uint64)
        check(lib().lsmgpu_compact_result(self._ctx, _ptr(out), out.size, _ptr(offs), offs.size),
              "compact_result")
        return [out[int(offs[t]): int(offs[t + 1])].tobytes() for t in range(nt.value)]

    # -- bloom tail (table/builder.go:164-195 Finish, table/table.go:301 DoesNotHave)
    def bloom_build_device(self, keys, key_end, n: int) -> dict:
        """Finish's filter over n keys WITH ts on the device (asynchronous): device tensors
        bitset / json / flags plus bits, locs, json_len."""
        import torch
        dev = key_end.device
        bits, locs, jl = bloom_params(n)
        o = dict(bitset=torch.empty(bits // 64, dtype=torch.int64, device=dev),
                 json=torch.empty(jl, dtype=torch.uint8, device=dev),
                 flags=torch.zeros(1, dtype=torch.int32, device=dev),
                 bits=bits, locs=locs, json_len=jl)
        check(lib().lsmgpu_bloom_build_async(self._ctx, _ptr(keys), _ptr(key_end), n,
                                             _ptr(o["bitset"]), bits, locs, _ptr(o["flags"])),
              "bloom_build_async")
        check(lib().lsmgpu_bloom_json_async(self._ctx, _ptr(o["bitset"]), bits, locs,
                                            _ptr(o["json"]), jl), "bloom_json_async")
        return o

    def bloom_tail_host(self, keys: bytes, key_end: np.ndarray) -> bytes:
        """bf.JSONMarshal() of Finish's filter for host keys (with ts); raises ValueError for
        a key of <= 8 B (y.go:98 AssertTruef)."""
        import torch
        ke = np.ascontiguousarray(key_end, dtype=np.uint32)
        n = int(ke.size)
        kd = torch.from_numpy(np.frombuffer(bytes(keys) + b"\0" * 16, np.uint8).copy()).to(self.device)
        o = self.bloom_build_device(kd, torch.from_numpy(ke.view(np.int32).copy()).to(self.device), n)
        self.synchronize()
        if int(o["flags"].cpu()[0]) & 1:
            raise ValueError("bloom: a key of <= 8 B (y.go:98 AssertTruef)")
        return o["json"].cpu().numpy().tobytes()

    def bloom_has_device(self, bitset, bits: int, locs: int, keys, key_end, n: int):
        """Has(key) for n keys as given (no ts) -> device u8 tensor (asynchronous)."""
        import torch
        has = torch.empty(max(n, 1), dtype=torch.uint8, device=key_end.device)
        check(lib().lsmgpu_bloom_has_async(self._ctx, _ptr(bitset), bits, locs, _ptr(keys),
                                           _ptr(key_end), n, _ptr(has)), "bloom_has_async")
        return has

    def bloom_has_cached(self, dev_bitset, locs: int, keys: list) -> np.ndarray:
        """Has(key) for host keys against a filter already on the device (int64 tensor)."""
        import torch
        n = len(keys)
        if n == 0:
            return np.zeros(0, bool)
        ke = np.cumsum([len(k) for k in keys], dtype=np.uint64).astype(np.uint32)
        t = lambda a: torch.from_numpy(a.copy()).to(self.device)
        kd = t(np.frombuffer(b"".join(bytes(k) for k in keys) + b"\0" * 16, np.uint8))
        has = self.bloom_has_device(dev_bitset, int(dev_bitset.numel()) * 64, locs, kd,
                                    t(ke.view(np.int32)), n)
        self.synchronize()
        return has[:n].cpu().numpy().astype(bool)

    def bloom_has_host(self, bitset: np.ndarray, locs: int, keys: list) -> np.ndarray:
        """Table.DoesNotHave's complement for a batch of host keys (no ts): bool array."""
        import torch
        bs = np.ascontiguousarray(bitset).view(np.uint64)
        bits = int(bs.size) * 64
        ke = np.cumsum([len(k) for k in keys], dtype=np.uint64).astype(np.uint32)
        n = len(keys)
        if n == 0:
            return np.zeros(0, bool)
        t = lambda a: torch.from_numpy(a.copy()).to(self.device)
        kd = t(np.frombuffer(b"".join(bytes(k) for k in keys) + b"\0" * 16, np.uint8))
        has = self.bloom_has_device(t(bs.view(np.int64)), bits, locs, kd, t(ke.view(np.int32)), n)
        self.synchronize()
        return has[:n].cpu().numpy().astype(bool)


def bloom_params(key_count: int) -> tuple[int, int, int]:
    """bbloom.New(float64(key_count), 0.01): (filter bits, setLocs, JSONMarshal length)."""
    bits, locs, jl = c_uint64(), c_uint64(), c_uint64()
    check(lib().lsmgpu_bloom_params(key_count, byref(bits), byref(locs), byref(jl)), "bloom_params")
    return bits.value, locs.value, jl.value


_DEFAULT: dict[int, Codec] = {}


def default_codec(device: Optional[int] = None) -> Codec:
    """Process-wide Codec per device (lazily opened)."""
    if device is None:
        device = 0
    c = _DEFAULT.get(device)
    if c is None:
        c = _DEFAULT[device] = Codec(device)
    return c


__all__ = ["Codec", "HostDecoded", "DeviceDecodeBuffers", "parse_index", "plan_blocks",
           "default_codec", "MODE_MATERIALIZE", "MODE_VIEW"]
_ = ctypes
