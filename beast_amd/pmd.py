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
F_EXACT = 2   # deflate: bit-identical to Beast (BPMD_F_EXACT)
# utf8_checker verdicts (bpmd_utf8) and websocket::error::bad_frame_payload
UTF8_VALID, UTF8_INCOMPLETE, UTF8_INVALID = 0, 1, 2
BAD_FRAME_PAYLOAD = 256


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
        L.bpmd_deflate_batch.argtypes = [ctypes.POINTER(_Cfg), vp, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp, vp]
        L.bpmd_diag_set_wave_walk.argtypes = [ctypes.c_int]
        L.bpmd_diag_bp_counters.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
        L.bpmd_inflate_reserve.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.bpmd_inflate_reserve.restype = ctypes.c_int
        L.bpmd_shard_ranges.argtypes = [vp, ctypes.c_uint32, ctypes.c_int, vp]
        L.bpmd_inflate_batch_multi.argtypes = [ctypes.POINTER(_Cfg), vp, ctypes.c_int, vp]
        L.bpmd_deflate_batch_multi.argtypes = [ctypes.POINTER(_Cfg), vp, ctypes.c_int, vp]
        L.bpmd_deflate_batch.restype = ctypes.c_int
        u32 = ctypes.c_uint32
        L.bpmd_mask_batch.argtypes = [vp, vp, vp, u32, vp, vp, vp]
        L.bpmd_utf8_check_batch.argtypes = [vp, vp, vp, u32, vp, vp]
        L.bpmd_frame_wire_size.argtypes = [ctypes.c_uint64, u32, ctypes.c_int]
        L.bpmd_frame_wire_size.restype = ctypes.c_uint64
        L.bpmd_frame_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, u32, u32, vp, vp, vp]
        L.bpmd_read_batch.argtypes = [ctypes.POINTER(_Cfg), vp, vp, vp, vp, vp, u32, vp, vp, vp, vp, vp, vp]
        L.bpmd_write_batch.argtypes = [ctypes.POINTER(_Cfg), vp, vp, vp, vp, u32, vp, vp, vp, vp, vp, vp]
        L.bpmd_inflate_takeover_batch.argtypes = [ctypes.POINTER(_Cfg), vp, vp, vp, vp, u32, vp, vp, vp, vp, vp, vp]
        L.bpmd_slide_batch.argtypes = [vp, vp, vp, vp, u32, vp]
        L.bpmd_deflate_takeover_batch.argtypes = [ctypes.POINTER(_Cfg), vp, vp, vp, vp, u32, vp, vp, vp, vp, vp, vp]
        L.bpmd_deflate_takeover_batch.restype = ctypes.c_int
        L.bpmd_batcher_create.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_int, u32, ctypes.c_size_t, ctypes.c_size_t,
                                          u32, ctypes.POINTER(vp)]
        L.bpmd_batcher_submit.argtypes = [vp, vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp, vp]
        L.bpmd_batcher_flush.argtypes = [vp]
        L.bpmd_batcher_destroy.argtypes = [vp]
        L.bpmd_batcher_destroy.restype = None
        for f in ("bpmd_batcher_create", "bpmd_batcher_submit", "bpmd_batcher_flush", "bpmd_mask_batch", "bpmd_utf8_check_batch", "bpmd_read_batch", "bpmd_write_batch",
                  "bpmd_inflate_takeover_batch", "bpmd_slide_batch"):
            getattr(L, f).restype = ctypes.c_int
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


def inflate_reserve(in_bytes: int, out_bytes: int, n_long: int, stream=None) -> None:
    """bpmd_inflate_reserve: size `stream`'s block-parallel decode workspace
    for batches whose long payloads total at most in_bytes / out_bytes /
    n_long, so that no call on it waits to size it (include/beast_pmd.h)."""
    _check(lib().bpmd_inflate_reserve(_stream_handle(stream), in_bytes, out_bytes, n_long), "bpmd_inflate_reserve")


def bp_counters(reset: bool = True) -> list:
    """bpmd_diag_bp_counters: [0] payloads resolved block-parallel, [1] their
    segments, [2] resolve fallbacks to the wave kernel, [3] capacity spills
    to it (pmd_inflate_bp.hip)."""
    c = (ctypes.c_ulonglong * 12)()
    _check(lib().bpmd_diag_bp_counters(c, 1 if reset else 0), "bpmd_diag_bp_counters")
    return list(c)


def deflate_batch(src: Batch, level: int = 6, window_bits: int = 15, mem_level: int = 4, strategy: int = 0,
                  stream=None, out_cap=None, out: torch.Tensor | None = None,
                  out_off: torch.Tensor | None = None, exact: bool = False) -> Result:
    """Deflate every message of `src` into a permessage-deflate payload
    (tail stripped) on the current GPU, asynchronous on `stream`.

    Slots default to deflate_upper_bound(len) bytes, which always suffices.
    exact=True (BPMD_F_EXACT): payloads bit-identical to Beast's deflater.
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
    cfg = _Cfg(level, window_bits, mem_level, strategy, F_EXACT if exact else 0)
    _check(L.bpmd_deflate_batch(ctypes.byref(cfg), _ptr(src.data), _ptr(src.off), _ptr(src.len), n, _ptr(out),
                                _ptr(out_off), _ptr(cap), _ptr(out_len), _ptr(status), _stream_handle(stream)),
           "bpmd_deflate_batch")
    return Result(Batch(out, out_off, out_len), cap, status)


# ------------------------------------------------------------------------
# Frame passes

def _optr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _keys(key, n: int, dev):
    """Per-message 32-bit masking keys (frame-header order, stream_impl.hpp:866-870)
    as an int32 device tensor holding the same bits; None stays None."""
    if key is None:
        return None
    if isinstance(key, torch.Tensor):
        if key.dtype == torch.int32:
            return key.to(dev).contiguous()
        key = key.cpu().numpy()
    a = np.array(np.broadcast_to(np.asarray(key, dtype=np.int64) & 0xFFFFFFFF, (n,)), dtype=np.uint32)
    return torch.from_numpy(a.view(np.int32)).to(dev)


def _u8(v, n: int, dev):
    if v is None:
        return None
    if isinstance(v, torch.Tensor):
        return v.to(device=dev, dtype=torch.uint8).contiguous()
    a = np.array(np.broadcast_to(np.asarray(v, dtype=np.uint8), (n,)), dtype=np.uint8)
    return torch.from_numpy(a).to(dev)


def mask_batch(b: Batch, key, phase=None, stream=None) -> None:
    """Beast's mask_inplace (websocket/detail/mask.ipp:38-59) over every message
    of `b`, in place; `phase` = bytes of the frame already masked, mod 4."""
    L = lib()
    dev = b.data.device
    k = _keys(key, b.n, dev)
    ph = _u8(phase, b.n, dev)
    _check(L.bpmd_mask_batch(_ptr(b.data), _ptr(b.off), _ptr(b.len), b.n, _optr(k), _optr(ph),
                             _stream_handle(stream)), "bpmd_mask_batch")


def frame_counts(lens: torch.Tensor, frame_max: int) -> torch.Tensor:
    """Frames per message (an empty payload is one empty frame)."""
    lens = lens.to(torch.int64)
    return torch.clamp((lens + frame_max - 1) // frame_max, min=1)


def frame_wire_sizes(lens: torch.Tensor, frame_max: int, masked: bool) -> torch.Tensor:
    """bpmd_frame_wire_size per message, on the lengths' device."""
    lens = lens.to(torch.int64)
    k = frame_counts(lens, frame_max)
    last = lens - (k - 1) * frame_max
    hdr = lambda x: torch.where(x <= 125, 2, torch.where(x <= 65535, 4, 10)) + (4 if masked else 0)  # noqa: E731
    full = torch.full_like(lens, frame_max)
    return lens + (k - 1) * hdr(full) + hdr(last)


def frame_plan(b: Batch, frame_max: int = 4096, masked: bool = False):
    """Wire sizes, wire offsets, total bytes and (masked) each message's first
    key index for bpmd_frame_batch; reusable across calls on same-shaped batches."""
    dev = b.data.device
    n = b.n
    sizes = frame_wire_sizes(b.len, frame_max, masked)
    woff = torch.zeros(n, dtype=torch.int64, device=dev)
    if n > 1:
        woff[1:] = torch.cumsum(sizes, 0)[:-1]
    total = int(sizes.sum().item()) if n else 0
    kb = nkeys = None
    if masked:
        cnt = frame_counts(b.len, frame_max)
        nkeys = int(cnt.sum().item())
        kb = torch.zeros(n, dtype=torch.int32, device=dev)
        if n > 1:
            kb[1:] = torch.cumsum(cnt, 0)[:-1].to(torch.int32)
    return {"frame_max": frame_max, "masked": masked, "sizes": sizes.to(torch.int32), "woff": woff, "total": total,
            "key_base": kb, "n_keys": nkeys}


def frame_batch(b: Batch, frame_max: int = 4096, op=2, compressed=True, keys=None, stream=None, plan=None,
                wire: torch.Tensor | None = None) -> Batch:
    """The wire bytes of every message of `b` (write.hpp:463-545 frame loop,
    frame.hpp:134-175 headers): frames of at most frame_max payload bytes,
    opcode `op` (per message or one value) and RSV1 when `compressed` on the
    first frame, FIN on the last; `keys` (client role) holds one key per
    frame, message by message (frame_counts gives how many), and masks each
    frame with its own key.  Returns one wire message per input message;
    `plan` (frame_plan) and `wire` skip the sizing and allocation."""
    L = lib()
    dev = b.data.device
    n = b.n
    masked = keys is not None
    if plan is None:
        plan = frame_plan(b, frame_max, masked)
    if plan["frame_max"] != frame_max or plan["masked"] != masked:
        raise BpmdError("frame_batch: plan made for another frame size or role")
    if wire is None:
        wire = torch.empty(plan["total"] + 16, dtype=torch.uint8, device=dev)
    opt = _u8(op, n, dev)
    fl = _u8(1 if compressed is True else 0 if compressed is False else compressed, n, dev)
    kt = None
    if masked:
        nk = int(keys.numel()) if isinstance(keys, torch.Tensor) else len(keys)
        kt = _keys(keys, nk, dev)
        if kt.numel() < plan["n_keys"]:
            raise BpmdError("frame_batch: keys must hold one key per frame (frame_counts)")
    _check(L.bpmd_frame_batch(_ptr(b.data), _ptr(b.off), _ptr(b.len), _optr(opt), _optr(fl), _optr(kt),
                              _optr(plan["key_base"]), frame_max, n, _ptr(wire), _ptr(plan["woff"]),
                              _stream_handle(stream)), "bpmd_frame_batch")
    return Batch(wire, plan["woff"], plan["sizes"])


def utf8_check_batch(b: Batch, stream=None, result: torch.Tensor | None = None) -> torch.Tensor:
    """utf8_checker verdict per message (UTF8_VALID / UTF8_INCOMPLETE / UTF8_INVALID)."""
    L = lib()
    res = result if result is not None else torch.empty(b.n, dtype=torch.int32, device=b.data.device)
    _check(L.bpmd_utf8_check_batch(_ptr(b.data), _ptr(b.off), _ptr(b.len), b.n, _ptr(res), _stream_handle(stream)),
           "bpmd_utf8_check_batch")
    return res


def _out_slots(n: int, dev, out_cap, out, out_off):
    if isinstance(out_cap, int):
        cap = torch.full((n,), out_cap, dtype=torch.int32, device=dev)
    else:
        cap = out_cap.to(device=dev, dtype=torch.int32)
    if out_off is None:
        out_off = slot_offsets(cap)
    if out is None:
        total = int(out_off[-1].item() + cap[-1].item()) if n else 0
        out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    return cap, out, out_off


def read_batch(src: Batch, out_cap, key=None, text=None, window_bits: int = 15, raw: bool = False, stream=None,
               out: torch.Tensor | None = None, out_off: torch.Tensor | None = None) -> Result:
    """Receive path, fused (read.hpp:1284-1385): unmask with `key` (per message,
    or None), inflate, and check the output of `text` messages; a text message
    that is not UTF-8 gets status BAD_FRAME_PAYLOAD.  `src` is not modified."""
    L = lib()
    dev = src.data.device
    n = src.n
    cap, out, out_off = _out_slots(n, dev, out_cap, out, out_off)
    k = _keys(key, n, dev)
    t = _u8(text, n, dev)
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    cfg = _Cfg(0, window_bits, 8, 0, F_RAW if raw else 0)
    _check(L.bpmd_read_batch(ctypes.byref(cfg), _ptr(src.data), _ptr(src.off), _ptr(src.len), _optr(k), _optr(t), n,
                             _ptr(out), _ptr(out_off), _ptr(cap), _ptr(out_len), _ptr(status), _stream_handle(stream)),
           "bpmd_read_batch")
    return Result(Batch(out, out_off, out_len), cap, status)


def write_batch(src: Batch, key=None, level: int = 6, window_bits: int = 15, mem_level: int = 4, strategy: int = 0,
                stream=None, out_cap=None, out: torch.Tensor | None = None,
                out_off: torch.Tensor | None = None, exact: bool = False) -> Result:
    """Send path, fused (write.hpp:655-703): deflate_batch with each payload
    masked by `key` in the kernel's output stores (client role)."""
    L = lib()
    dev = src.data.device
    n = src.n
    if out_cap is None:
        ln = src.len.to(torch.int64)
        out_cap = (ln + (ln + 7) // 8 + (ln + 63) // 64 + 11).to(torch.int32)
    cap, out, out_off = _out_slots(n, dev, out_cap, out, out_off)
    k = _keys(key, n, dev)
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    cfg = _Cfg(level, window_bits, mem_level, strategy, F_EXACT if exact else 0)
    _check(L.bpmd_write_batch(ctypes.byref(cfg), _ptr(src.data), _ptr(src.off), _ptr(src.len), _optr(k), n,
                              _ptr(out), _ptr(out_off), _ptr(cap), _ptr(out_len), _ptr(status),
                              _stream_handle(stream)), "bpmd_write_batch")
    return Result(Batch(out, out_off, out_len), cap, status)


# ------------------------------------------------------------------------
# Context takeover

def _check_unique(conn, n):
    """One message per connection per call: two messages of one connection
    would share an output position and history and overwrite each other."""
    if n and int(torch.unique(conn).numel()) != n:
        raise BpmdError("a connection appears more than once in one batch; submit its messages in separate calls")


class TakeoverInflater:
    """Receive side of context-takeover connections: Beast's inflater keeps its
    window across messages (impl_base.hpp:192-202; inflate_stream::clear() is a
    no-op, inflate_stream.ipp:49-53).  Each connection owns a device buffer of
    2 * 2^window_bits + max_msg bytes holding its latest output; message k of a
    connection is decoded right after its earlier output, whose last
    2^window_bits bytes are the window.  When a buffer cannot take the next
    message, its window slides to the front on the device (bpmd_slide_batch).
    Bookkeeping stays on the device except for that fullness test."""

    def __init__(self, n_conn: int, window_bits: int = 15, max_msg: int = 1 << 16, device="cuda"):
        self.wbits = window_bits
        self.W = 1 << window_bits
        self.max_msg = max_msg
        self.slot = (2 * self.W + max_msg + 15) // 16 * 16
        self.buf = torch.zeros(n_conn * self.slot + 16, dtype=torch.uint8, device=device)
        self.base = torch.arange(n_conn, dtype=torch.int64, device=device) * self.slot
        self.pos = torch.zeros(n_conn, dtype=torch.int64, device=device)

    def inflate(self, src: Batch, out_cap, conn=None, stream=None) -> Result:
        """Inflate src's messages, message i continuing connection conn[i]
        (default i); at most one message per connection per call."""
        L = lib()
        dev = self.buf.device
        n = src.n
        conn = torch.arange(n, device=dev) if conn is None else torch.as_tensor(conn, device=dev).long()
        _check_unique(conn, n)
        cap = torch.full((n,), out_cap, dtype=torch.int32, device=dev) if isinstance(out_cap, int) \
            else out_cap.to(device=dev, dtype=torch.int32)
        if int(cap.max().item() if n else 0) > self.max_msg:
            raise BpmdError("out_cap exceeds max_msg")
        pos = self.pos[conn]
        full = pos + cap.to(torch.int64) > self.slot
        if n and bool(full.any()):
            idx = conn[full]
            keep = torch.minimum(self.pos[idx], torch.tensor(self.W, device=dev))
            p32 = self.pos[idx].to(torch.int32)
            k32 = keep.to(torch.int32)
            b64 = self.base[idx].contiguous()
            _check(L.bpmd_slide_batch(_ptr(self.buf), _ptr(b64), _ptr(p32), _ptr(k32), int(idx.numel()),
                                      _stream_handle(stream)), "bpmd_slide_batch")
            self.pos[idx] = keep
            pos = self.pos[conn]
        hist = torch.minimum(pos, torch.tensor(self.W, device=dev)).to(torch.int32)
        out_off = (self.base[conn] + pos).contiguous()
        out_len = torch.empty(n, dtype=torch.int32, device=dev)
        status = torch.empty(n, dtype=torch.int32, device=dev)
        cfg = _Cfg(0, self.wbits, 8, 0, 0)
        _check(L.bpmd_inflate_takeover_batch(ctypes.byref(cfg), _ptr(src.data), _ptr(src.off), _ptr(src.len),
                                             _ptr(hist), n, _ptr(self.buf), _ptr(out_off), _ptr(cap), _ptr(out_len),
                                             _ptr(status), _stream_handle(stream)), "bpmd_inflate_takeover_batch")
        # a connection whose message failed is left where it was: its window
        # is undefined from here on (the reference's stream goes BAD), so the
        # caller drops it (check_stop_now fails the websocket connection)
        self.pos[conn] = pos + torch.where(status == 0, out_len, torch.zeros_like(out_len)).to(torch.int64)
        return Result(Batch(self.buf, out_off, out_len), cap, status)


# ------------------------------------------------------------------------
# Cross-connection micro-batcher

_DONE = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int32, ctypes.c_size_t)


class Completion:
    """Result of one submitted message: wait() returns (status, bytes)."""

    def __init__(self, cap: int):
        import threading
        self.buf = ctypes.create_string_buffer(max(cap, 1))
        self.cap = cap
        self.event = threading.Event()
        self.status = None
        self.length = 0

    def wait(self, timeout=None):
        if not self.event.wait(timeout):
            raise TimeoutError("message not completed")
        return self.status, self.buf.raw[:self.length]


class Batcher:
    """Host-buffer front end that coalesces single messages from many
    connections (threads) into batch launches (bpmd_batcher_*)."""

    def __init__(self, op: str = "inflate", level: int = 6, window_bits: int = 15, mem_level: int = 4,
                 strategy: int = 0, raw: bool = False, max_msgs: int = 4096, max_in_bytes: int = 16 << 20,
                 max_out_bytes: int = 64 << 20, max_delay_us: int = 200):
        import threading
        self.L = lib()
        self.op = op
        cfg = _Cfg(level, window_bits, mem_level, strategy, F_RAW if raw else 0)
        h = ctypes.c_void_p()
        _check(self.L.bpmd_batcher_create(ctypes.byref(cfg), 0 if op == "inflate" else 1, max_msgs, max_in_bytes,
                                          max_out_bytes, max_delay_us, ctypes.byref(h)), "bpmd_batcher_create")
        self._h = h
        self._lock = threading.Lock()
        self._pending = {}
        self._next = 1
        self._cb = _DONE(self._done)

    def _done(self, user, status, n):
        with self._lock:
            c = self._pending.pop(user)
        c.status, c.length = int(status), int(n)
        c.event.set()

    def submit(self, data: bytes, out_cap: int) -> Completion:
        data = bytes(data)
        c = Completion(out_cap)
        with self._lock:
            key = self._next
            self._next += 1
            self._pending[key] = c
        src = ctypes.create_string_buffer(data, max(len(data), 1))
        r = self.L.bpmd_batcher_submit(self._h, src, len(data), c.buf, out_cap, self._cb, ctypes.c_void_p(key))
        if r:
            with self._lock:
                self._pending.pop(key, None)
            _check(r, "bpmd_batcher_submit")
        return c

    def flush(self):
        _check(self.L.bpmd_batcher_flush(self._h), "bpmd_batcher_flush")

    def close(self):
        if self._h:
            self.L.bpmd_batcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TakeoverDeflater:
    """Send side of context-takeover connections: Beast's deflater keeps its
    window across messages unless no_context_takeover was negotiated
    (impl_base.hpp:156-166).  Each connection's plaintext accumulates in a
    device buffer; message k is placed right after the connection's earlier
    plaintext, whose last 4 KiB its matches may reach into.  Payloads decode
    with any inflater that keeps its window (TakeoverInflater, Beast's)."""

    HIST = 4096

    def __init__(self, n_conn: int, level: int = 6, window_bits: int = 15, mem_level: int = 4,
                 max_msg: int = 1 << 16, device="cuda"):
        self.cfg = _Cfg(level, window_bits, mem_level, 0, 0)
        self.max_msg = max_msg
        self.slot = (2 * self.HIST + max_msg + 15) // 16 * 16
        self.buf = torch.zeros(n_conn * self.slot + 16, dtype=torch.uint8, device=device)
        self.base = torch.arange(n_conn, dtype=torch.int64, device=device) * self.slot
        self.pos = torch.zeros(n_conn, dtype=torch.int64, device=device)

    def deflate(self, src: Batch, conn=None, stream=None) -> Result:
        L = lib()
        dev = self.buf.device
        n = src.n
        conn = torch.arange(n, device=dev) if conn is None else torch.as_tensor(conn, device=dev).long()
        _check_unique(conn, n)
        lens = src.len.to(torch.int64)
        if n and int(lens.max().item()) > self.max_msg:
            raise BpmdError("message exceeds max_msg")
        full = self.pos[conn] + lens > self.slot
        if n and bool(full.any()):
            idx = conn[full]
            keep = torch.minimum(self.pos[idx], torch.tensor(self.HIST, device=dev))
            p32, k32, b64 = self.pos[idx].to(torch.int32), keep.to(torch.int32), self.base[idx].contiguous()
            _check(L.bpmd_slide_batch(_ptr(self.buf), _ptr(b64), _ptr(p32), _ptr(k32), int(idx.numel()),
                                      _stream_handle(stream)), "bpmd_slide_batch")
            self.pos[idx] = keep
        pos = self.pos[conn]
        in_off = (self.base[conn] + pos).contiguous()
        total = int(lens.sum().item()) if n else 0
        if total:   # place the messages after each connection's plaintext
            start = torch.cumsum(lens, 0) - lens
            j = torch.arange(total, device=dev) - torch.repeat_interleave(start, lens)
            self.buf[torch.repeat_interleave(in_off, lens) + j] = src.data[torch.repeat_interleave(src.off, lens) + j]
        hist = torch.minimum(pos, torch.tensor(self.HIST, device=dev)).to(torch.int32)
        cap = (lens + (lens + 7) // 8 + (lens + 63) // 64 + 11).to(torch.int32)
        out_off = slot_offsets(cap)
        out = torch.empty(int(out_off[-1].item() + cap[-1].item()) + 16 if n else 16, dtype=torch.uint8,
                          device=dev)
        out_len = torch.empty(n, dtype=torch.int32, device=dev)
        status = torch.empty(n, dtype=torch.int32, device=dev)
        in_len = src.len.to(torch.int32).contiguous()
        _check(L.bpmd_deflate_takeover_batch(ctypes.byref(self.cfg), _ptr(self.buf), _ptr(in_off), _ptr(in_len),
                                             _ptr(hist), n, _ptr(out), _ptr(out_off), _ptr(cap), _ptr(out_len),
                                             _ptr(status), _stream_handle(stream)), "bpmd_deflate_takeover_batch")
        self.pos[conn] = pos + lens
        return Result(Batch(out, out_off, out_len), cap, status)


# ------------------------------------------------- one process, several GPUs

class _Shard(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("stream", ctypes.c_void_p), ("d_in", ctypes.c_void_p),
                ("d_in_off", ctypes.c_void_p), ("d_in_len", ctypes.c_void_p), ("n_msgs", ctypes.c_uint32),
                ("d_out", ctypes.c_void_p), ("d_out_off", ctypes.c_void_p), ("d_out_cap", ctypes.c_void_p),
                ("d_out_len", ctypes.c_void_p), ("d_status", ctypes.c_void_p)]


def shard_ranges(lens, n_parts: int):
    """bpmd_shard_ranges: [(start, end)] byte-balanced contiguous ranges."""
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    starts = np.zeros(n_parts + 1, dtype=np.uint32)
    _check(lib().bpmd_shard_ranges(lens.ctypes.data_as(ctypes.c_void_p), len(lens), n_parts,
                                   starts.ctypes.data_as(ctypes.c_void_p)), "bpmd_shard_ranges")
    return [(int(starts[i]), int(starts[i + 1])) for i in range(n_parts)]


def _multi(fn, cfg, parts):
    """parts: [(src Batch, out buffer, out_off, cap, out_len, status, stream)]."""
    arr = (_Shard * len(parts))()
    for i, (src, out, out_off, cap, out_len, status, stream) in enumerate(parts):
        arr[i] = _Shard(src.data.device.index or 0, _stream_handle(stream), _ptr(src.data), _ptr(src.off),
                        _ptr(src.len), src.n, _ptr(out), _ptr(out_off), _ptr(cap), _ptr(out_len), _ptr(status))
    totals = np.zeros(len(parts), dtype=np.uint64)
    _check(fn(ctypes.byref(cfg), arr, len(parts), totals.ctypes.data_as(ctypes.c_void_p)), fn.__name__)
    return totals


def inflate_batch_multi(srcs, out_caps, window_bits: int = 15, streams=None):
    """bpmd_inflate_batch_multi over shards (each a Batch on its own device):
    returns ([Result], per-shard output byte totals)."""
    streams = streams or [None] * len(srcs)
    parts, res = [], []
    for src, c, st in zip(srcs, out_caps, streams):
        dev = src.data.device
        cap = torch.full((src.n,), c, dtype=torch.int32, device=dev) if isinstance(c, int) else c.to(dev)
        off = slot_offsets(cap)
        out = torch.empty((int(off[-1].item() + cap[-1].item()) if src.n else 0) + 16, dtype=torch.uint8, device=dev)
        out_len = torch.empty(src.n, dtype=torch.int32, device=dev)
        status = torch.empty(src.n, dtype=torch.int32, device=dev)
        parts.append((src, out, off, cap, out_len, status, st))
        res.append(Result(Batch(out, off, out_len), cap, status))
    totals = _multi(lib().bpmd_inflate_batch_multi, _Cfg(0, window_bits, 8, 0, 0), parts)
    return res, totals


def deflate_batch_multi(srcs, level: int = 6, window_bits: int = 15, mem_level: int = 4, strategy: int = 0,
                        streams=None):
    """bpmd_deflate_batch_multi over shards; slots of deflate_upper_bound."""
    streams = streams or [None] * len(srcs)
    parts, res = [], []
    for src, st in zip(srcs, streams):
        dev = src.data.device
        l64 = src.len.to(torch.int64)
        cap = (l64 + (l64 + 7) // 8 + (l64 + 63) // 64 + 11).to(torch.int32)
        off = slot_offsets(cap)
        out = torch.empty((int(off[-1].item() + cap[-1].item()) if src.n else 0) + 16, dtype=torch.uint8, device=dev)
        out_len = torch.empty(src.n, dtype=torch.int32, device=dev)
        status = torch.empty(src.n, dtype=torch.int32, device=dev)
        parts.append((src, out, off, cap, out_len, status, st))
        res.append(Result(Batch(out, off, out_len), cap, status))
    totals = _multi(lib().bpmd_deflate_batch_multi, _Cfg(level, window_bits, mem_level, strategy, 0), parts)
    return res, totals
