"""Host-side binding of the MI355X permessage-deflate engine.

The engine itself is `libbeast_pmd.so` (HIP kernels + the C ABI declared in
include/beast_pmd.h).  This module is plumbing around it: torch provides the
device memory and the stream, ctypes passes raw device pointers.  There is no
CPU fallback: if the library or a GPU is missing every call raises.

Batch layout (struct of arrays, all device tensors):
    data  uint8  [total]      payload bytes, message i at off[i] .. off[i]+len[i]
    off   int64  [n]          byte offsets (uint64 in the C ABI)
    len   int32  [n]          byte lengths (uint32 in the C ABI)
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import build as _build

_LIB = None

# zlib::error names (include/boost/beast/zlib/error.hpp:48-138)
ERRORS = ("ok", "need_buffers", "end_of_stream", "need_dict", "stream_error", "invalid_block_type",
          "invalid_stored_length", "too_many_symbols", "invalid_code_lengths", "invalid_bit_length_repeat",
          "missing_eob", "invalid_literal_length", "invalid_distance_code", "invalid_distance",
          "over_subscribed_length", "incomplete_length_set", "general")
F_RAW = 1


class BpmdError(RuntimeError):
    pass


class _Cfg(ctypes.Structure):
    _fields_ = [("level", ctypes.c_int), ("window_bits", ctypes.c_int), ("mem_level", ctypes.c_int),
                ("strategy", ctypes.c_int), ("flags", ctypes.c_uint32)]


def lib():
    """Load libbeast_pmd.so (building it first if this checkout has none)."""
    global _LIB
    if _LIB is None:
        # BPMD_LIB selects a diagnostic variant (e.g. libbeast_pmd_prof.so)
        path = os.environ.get("BPMD_LIB", _build.LIB)
        if not os.path.exists(path):
            _build.build()
        L = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        L.bpmd_init.restype = ctypes.c_int
        L.bpmd_version.restype = ctypes.c_char_p
        L.bpmd_deflate_upper_bound.argtypes = [ctypes.c_size_t]
        L.bpmd_deflate_upper_bound.restype = ctypes.c_size_t
        L.bpmd_inflate_batch.argtypes = [ctypes.POINTER(_Cfg), vp, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp, vp]
        L.bpmd_inflate_batch.restype = ctypes.c_int
        if hasattr(L, "bpmd_deflate_batch"):
            L.bpmd_deflate_batch.argtypes = [ctypes.POINTER(_Cfg), vp, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp, vp]
            L.bpmd_deflate_batch.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _check(r: int, what: str):
    if r != 0:
        names = {-1: "invalid_argument", -2: "domain_error", -3: "hip_error", -4: "no_device"}
        raise BpmdError(f"{what}: {names.get(r, r)}")


def _ptr(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


def _stream_handle(stream):
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def upper_bound(n: int) -> int:
    """deflate_upper_bound (include/boost/beast/zlib/deflate_stream.hpp:402-410)."""
    return lib().bpmd_deflate_upper_bound(n)


def slot_offsets(cap: torch.Tensor, align: int = 16) -> torch.Tensor:
    """Exclusive prefix sum of slot capacities rounded up to `align` bytes."""
    c = (cap.to(torch.int64) + (align - 1)) // align * align
    off = torch.zeros_like(c)
    if c.numel() > 1:
        off[1:] = torch.cumsum(c[:-1], 0)
    return off


@dataclass
class Batch:
    data: torch.Tensor   # uint8
    off: torch.Tensor    # int64
    len: torch.Tensor    # int32

    @property
    def n(self) -> int:
        return int(self.len.numel())

    def message(self, i: int) -> bytes:
        o, l = int(self.off[i]), int(self.len[i])
        return bytes(self.data[o:o + l].cpu().numpy().tobytes())

    @staticmethod
    def from_host(msgs, device="cuda", align: int = 16) -> "Batch":
        """Pack a list of bytes (or numpy arrays) into one device batch."""
        lens = np.array([len(m) for m in msgs], dtype=np.int64)
        pad = (lens + (align - 1)) // align * align
        off = np.zeros(len(msgs), dtype=np.int64)
        if len(msgs) > 1:
            off[1:] = np.cumsum(pad[:-1])
        buf = np.zeros(int(pad.sum()) + 16, dtype=np.uint8)
        for i, m in enumerate(msgs):
            a = np.frombuffer(bytes(m), dtype=np.uint8) if not isinstance(m, np.ndarray) else m
            buf[off[i]:off[i] + len(a)] = a
        return Batch(torch.from_numpy(buf).to(device), torch.from_numpy(off).to(device),
                     torch.from_numpy(lens.astype(np.int32)).to(device))

    @staticmethod
    def from_arrays(data: np.ndarray, off: np.ndarray, lens: np.ndarray, device="cuda") -> "Batch":
        d = torch.from_numpy(np.ascontiguousarray(data, dtype=np.uint8))
        return Batch(d.to(device), torch.from_numpy(np.asarray(off, dtype=np.int64)).to(device),
                     torch.from_numpy(np.asarray(lens, dtype=np.int32)).to(device))

    def to_host(self):
        return [self.message(i) for i in range(self.n)]


@dataclass
class Result:
    out: Batch           # out.len = produced bytes
    cap: torch.Tensor    # int32 slot capacities
    status: torch.Tensor  # int32 zlib::error per message


def inflate_batch(src: Batch, out_cap, window_bits: int = 15, raw: bool = False, stream=None,
                  out: torch.Tensor | None = None, out_off: torch.Tensor | None = None) -> Result:
    """Inflate every message of `src` on the current GPU (asynchronous on `stream`).

    `out_cap` (int or int32 tensor): output capacity per message.  Messages
    that would produce more report status need_buffers and keep `cap` bytes.
    """
    L = lib()
    dev = src.data.device
    n = src.n
    if isinstance(out_cap, int):
        cap = torch.full((n,), out_cap, dtype=torch.int32, device=dev)
    else:
        cap = out_cap.to(device=dev, dtype=torch.int32)
    if out_off is None:
        out_off = slot_offsets(cap)
    if out is None:
        total = int(out_off[-1].item() + cap[-1].item()) if n else 0
        out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    cfg = _Cfg(0, window_bits, 8, 0, F_RAW if raw else 0)
    _check(L.bpmd_inflate_batch(ctypes.byref(cfg), _ptr(src.data), _ptr(src.off), _ptr(src.len), n, _ptr(out),
                                _ptr(out_off), _ptr(cap), _ptr(out_len), _ptr(status), _stream_handle(stream)),
           "bpmd_inflate_batch")
    return Result(Batch(out, out_off, out_len), cap, status)


def deflate_batch(src: Batch, level: int = 6, window_bits: int = 15, mem_level: int = 4, strategy: int = 0,
                  stream=None, out_cap=None, out: torch.Tensor | None = None,
                  out_off: torch.Tensor | None = None) -> Result:
    """Deflate every message of `src` into a permessage-deflate payload
    (tail stripped) on the current GPU, asynchronous on `stream`.

    Slots default to deflate_upper_bound(len) bytes, which always suffices.
    """
    L = lib()
    dev = src.data.device
    n = src.n
    if out_cap is None:
        ln = src.len.to(torch.int64)
        cap = (ln + (ln + 7) // 8 + (ln + 63) // 64 + 11).to(torch.int32)
    elif isinstance(out_cap, int):
        cap = torch.full((n,), out_cap, dtype=torch.int32, device=dev)
    else:
        cap = out_cap.to(device=dev, dtype=torch.int32)
    if out_off is None:
        out_off = slot_offsets(cap)
    if out is None:
        total = int(out_off[-1].item() + cap[-1].item()) if n else 0
        out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    cfg = _Cfg(level, window_bits, mem_level, strategy, 0)
    _check(L.bpmd_deflate_batch(ctypes.byref(cfg), _ptr(src.data), _ptr(src.off), _ptr(src.len), n, _ptr(out),
                                _ptr(out_off), _ptr(cap), _ptr(out_len), _ptr(status), _stream_handle(stream)),
           "bpmd_deflate_batch")
    return Result(Batch(out, out_off, out_len), cap, status)
