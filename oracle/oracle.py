"""ctypes front-end for the CPU oracle (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  The product path (beast_amd/) never does.

`liboracle.so` is the clean-room C restatement of Beast's zlib + pmd framing
(see bzo.h); `_ref/libzref.so` is the reference's vendored zlib 1.3.1,
compiled in place from /root/reference by oracle/Makefile (present only where
it could be built).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

# zlib::error values (include/boost/beast/zlib/error.hpp:48-138)
ERRORS = {
    0: "ok", 1: "need_buffers", 2: "end_of_stream", 3: "need_dict", 4: "stream_error",
    5: "invalid_block_type", 6: "invalid_stored_length", 7: "too_many_symbols",
    8: "invalid_code_lengths", 9: "invalid_bit_length_repeat", 10: "missing_eob",
    11: "invalid_literal_length", 12: "invalid_distance_code", 13: "invalid_distance",
    14: "over_subscribed_length", 15: "incomplete_length_set", 16: "general",
}
ERROR_CODES = {v: k for k, v in ERRORS.items()}

FLUSH = {"none": 0, "block": 1, "partial": 2, "sync": 3, "full": 4, "finish": 5, "trees": 6}
STRATEGY = {"normal": 0, "filtered": 1, "huffman": 2, "rle": 3, "fixed": 4}


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.bzo_inflate_new.restype = ctypes.c_void_p
        L.bzo_deflate_new.restype = ctypes.c_void_p
        L.bzo_inflate_free.argtypes = [ctypes.c_void_p]
        L.bzo_deflate_free.argtypes = [ctypes.c_void_p]
        L.bzo_inflate_reset.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.bzo_inflate_write.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.bzo_deflate_reset_params.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 4
        L.bzo_deflate_reset.argtypes = [ctypes.c_void_p]
        L.bzo_deflate_write.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.bzo_deflate_upper_bound.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.bzo_deflate_upper_bound.restype = ctypes.c_size_t
        L.bzo_deflate_upper_bound_free.argtypes = [ctypes.c_size_t]
        L.bzo_deflate_upper_bound_free.restype = ctypes.c_size_t
        L.bzo_pmd_deflate_msg.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                          ctypes.c_void_p, ctypes.c_size_t]
        L.bzo_pmd_deflate_msg.restype = ctypes.c_long
        L.bzo_pmd_inflate_msg.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                          ctypes.c_void_p, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_size_t), ctypes.c_int]
        vp = ctypes.c_void_p
        L.bzo_pmd_deflate_batch.argtypes = [ctypes.c_int] * 4 + [vp] * 3 + [ctypes.c_uint32] + [vp] * 5 + [ctypes.c_int]
        L.bzo_pmd_inflate_batch.argtypes = [ctypes.c_int, ctypes.c_int] + [vp] * 3 + [ctypes.c_uint32] + [vp] * 5 + [ctypes.c_int]
        L.bzo_mask.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint]
        L.bzo_mask.restype = ctypes.c_uint
        L.bzo_frame_wire_size.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]
        L.bzo_frame_wire_size.restype = ctypes.c_size_t
        L.bzo_frame_write.argtypes = [vp, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint, ctypes.c_int, vp,
                                      ctypes.c_uint64]
        L.bzo_frame_write.restype = ctypes.c_size_t
        L.bzo_utf8_reset.argtypes = [vp]
        L.bzo_utf8_write.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t]
        L.bzo_utf8_finish.argtypes = [vp]
        L.bzo_utf8_check.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.bzo_utf8_check_batch.argtypes = [vp, vp, vp, ctypes.c_uint32, vp]
        _LIB = L
    return _LIB


def _load_zshim(path):
    if not os.path.exists(path):
        return None
    R = ctypes.CDLL(path)
    R.zref_deflate.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_ulong,
                                                   ctypes.c_void_p, ctypes.c_ulong]
    R.zref_deflate.restype = ctypes.c_long
    R.zref_inflate.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                               ctypes.c_ulong, ctypes.POINTER(ctypes.c_int)]
    R.zref_inflate.restype = ctypes.c_long
    vp = ctypes.c_void_p
    R.zref_batch.argtypes = [ctypes.c_int] * 4 + [vp] * 3 + [ctypes.c_uint32] + [vp] * 4 + [ctypes.c_int]
    R.zref_batch.restype = ctypes.c_int
    if hasattr(R, "zref_version"):
        R.zref_version.restype = ctypes.c_char_p
    return R


def ref():
    """The reference's own zlib 1.3.1 (None when it could not be built)."""
    global _REF
    if _REF is None:
        _REF = _load_zshim(os.path.join(HERE, "_ref", "libzref.so"))
    return _REF


_ZSYS = None


def zsys():
    """The image's system zlib behind the same shim (None when absent): an
    extra CPU-baseline column, not a parity reference."""
    global _ZSYS
    if _ZSYS is None:
        _ZSYS = _load_zshim(os.path.join(HERE, "libzsys.so"))
    return _ZSYS


class ZParams(ctypes.Structure):
    _fields_ = [("next_in", ctypes.c_void_p), ("avail_in", ctypes.c_size_t),
                ("total_in", ctypes.c_size_t), ("next_out", ctypes.c_void_p),
                ("avail_out", ctypes.c_size_t), ("total_out", ctypes.c_size_t),
                ("data_type", ctypes.c_int)]


def _buf(b: bytes):
    return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) if b else None


def upper_bound(n: int) -> int:
    """deflate_upper_bound (zlib/deflate_stream.hpp:402-410)."""
    return lib().bzo_deflate_upper_bound_free(n)


def pmd_deflate(data: bytes, level=6, wbits=15, mem_level=4, strategy=0) -> bytes:
    L = lib()
    z = L.bzo_deflate_new()
    try:
        r = L.bzo_deflate_reset_params(z, level, wbits, mem_level, strategy)
        if r:
            raise ValueError("invalid deflate parameters")
        cap = upper_bound(len(data)) + 64
        out = ctypes.create_string_buffer(cap)
        src = ctypes.create_string_buffer(data, len(data)) if data else None
        n = L.bzo_pmd_deflate_msg(z, src, len(data), out, cap)
        if n < 0:
            raise RuntimeError(f"deflate failed: {ERRORS.get(-n, -n)}")
        return out.raw[:n]
    finally:
        L.bzo_deflate_free(z)


def pmd_inflate(payload: bytes, cap: int = 1 << 20, wbits=15, raw=False):
    """Returns (status, output bytes)."""
    L = lib()
    z = L.bzo_inflate_new()
    try:
        if L.bzo_inflate_reset(z, wbits):
            raise ValueError("windowBits out of range")
        out = ctypes.create_string_buffer(max(cap, 1))
        got = ctypes.c_size_t(0)
        src = ctypes.create_string_buffer(payload, len(payload)) if payload else None
        st = L.bzo_pmd_inflate_msg(z, src, len(payload), out, cap, ctypes.byref(got), 1 if raw else 0)
        return st, out.raw[:got.value]
    finally:
        L.bzo_inflate_free(z)


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def deflate_batch(data: np.ndarray, off: np.ndarray, lens: np.ndarray, level=6, wbits=15,
                  mem_level=4, strategy=0, threads=1):
    """Batch pmd deflate; returns (out, out_off, out_len, status)."""
    n = len(lens)
    cap = np.array([upper_bound(int(x)) + 16 for x in lens], dtype=np.uint32)
    out_off = np.zeros(n, dtype=np.uint64)
    if n:
        out_off[1:] = np.cumsum(cap[:-1].astype(np.uint64))
    out = np.zeros(int(cap.astype(np.uint64).sum()) + 1, dtype=np.uint8)
    out_len = np.zeros(n, dtype=np.uint32)
    status = np.zeros(n, dtype=np.int32)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    lib().bzo_pmd_deflate_batch(level, wbits, mem_level, strategy, _p(data), _p(off), _p(lens),
                                n, _p(out), _p(out_off), _p(cap), _p(out_len), _p(status), threads)
    return out, out_off, out_len, status


def inflate_batch(data: np.ndarray, off: np.ndarray, lens: np.ndarray, out_cap: np.ndarray,
                  wbits=15, raw=False, threads=1):
    """Batch pmd inflate; returns (out, out_off, out_len, status)."""
    n = len(lens)
    out_cap = np.ascontiguousarray(out_cap, dtype=np.uint32)
    out_off = np.zeros(n, dtype=np.uint64)
    if n:
        out_off[1:] = np.cumsum(out_cap[:-1].astype(np.uint64))
    out = np.zeros(int(out_cap.astype(np.uint64).sum()) + 1, dtype=np.uint8)
    out_len = np.zeros(n, dtype=np.uint32)
    status = np.zeros(n, dtype=np.int32)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    lib().bzo_pmd_inflate_batch(wbits, 1 if raw else 0, _p(data), _p(off), _p(lens), n, _p(out),
                                _p(out_off), _p(out_cap), _p(out_len), _p(status), threads)
    return out, out_off, out_len, status


def ref_pmd_deflate(data: bytes, level=6, wbits=15, mem_level=4, strategy=0, mode=0):
    R = ref()
    if R is None:
        return None
    cap = upper_bound(len(data)) + 64
    out = ctypes.create_string_buffer(cap)
    src = ctypes.create_string_buffer(data, len(data)) if data else None
    n = R.zref_deflate(level, wbits, mem_level, strategy, mode, src, len(data), out, cap)
    if n < 0:
        raise RuntimeError("reference zlib deflate failed")
    return out.raw[:n]


class Inflater:
    """Streaming zlib::inflate_stream restatement (inflate_stream.hpp:63-213)."""

    def __init__(self, wbits=15):
        self.L = lib()
        self.z = self.L.bzo_inflate_new()
        self.reset(wbits)

    def reset(self, wbits=15):
        r = self.L.bzo_inflate_reset(self.z, wbits)
        if r:
            raise ValueError("windowBits out of range")

    def write(self, zs: ZParams, flush: str) -> int:
        return self.L.bzo_inflate_write(self.z, ctypes.byref(zs), FLUSH[flush])

    def __del__(self):
        try:
            self.L.bzo_inflate_free(self.z)
        except Exception:
            pass


class Deflater:
    """Streaming zlib::deflate_stream restatement (deflate_stream.hpp:59-369)."""

    def __init__(self, level=6, wbits=15, mem_level=9, strategy=0):
        self.L = lib()
        self.z = self.L.bzo_deflate_new()
        if self.L.bzo_deflate_reset_params(self.z, level, wbits, mem_level, strategy):
            raise ValueError("invalid deflate parameters")

    def reset(self):
        self.L.bzo_deflate_reset(self.z)

    def write(self, zs: ZParams, flush: str) -> int:
        return self.L.bzo_deflate_write(self.z, ctypes.byref(zs), FLUSH[flush])

    def __del__(self):
        try:
            self.L.bzo_deflate_free(self.z)
        except Exception:
            pass


# ---------------------------------------------------------------- frame passes

def mask(data: bytes, key: int, phase: int = 0) -> bytes:
    """mask_inplace (websocket/detail/mask.ipp:38-59) with the frame key
    (little-endian from the wire) rotated by `phase` bytes already masked."""
    data = bytes(data)
    buf = ctypes.create_string_buffer(data, max(len(data), 1))
    lib().bzo_mask(buf, len(data), key & 0xFFFFFFFF, phase & 3)
    return buf.raw[:len(data)]


def frame_write(payload: bytes, op: int, rsv1: bool, keys=None, frame_max: int = 4096) -> bytes:
    """A message's frames on the wire (frame.hpp:134-175 headers, the
    write.hpp:463-545 frame loop): frames of at most frame_max payload bytes,
    opcode and RSV1 on the first, FIN on the last, frame f masked with keys[f]
    (None = unmasked)."""
    payload = bytes(payload)
    L = lib()
    masked = keys is not None
    size = L.bzo_frame_wire_size(len(payload), frame_max, int(masked))
    out = ctypes.create_string_buffer(max(size, 1))
    kp = None
    if masked:
        kp = (ctypes.c_uint32 * max(len(keys), 1))(*[k & 0xFFFFFFFF for k in keys])
    w = L.bzo_frame_write(out, payload, len(payload), op, int(bool(rsv1)), kp, frame_max)
    assert w == size
    return out.raw[:w]


def utf8_check(data: bytes) -> int:
    """0 valid, 1 write() ok but finish() fails, 2 write() fails (utf8_checker.ipp)."""
    data = bytes(data)
    return lib().bzo_utf8_check(data, len(data))


class _U8(ctypes.Structure):
    _fields_ = [("need", ctypes.c_size_t), ("have", ctypes.c_size_t), ("cp", ctypes.c_uint8 * 4)]


class Utf8Checker:
    """Streaming utf8_checker (websocket/detail/utf8_checker.hpp:29-86)."""

    def __init__(self):
        self._s = _U8()
        lib().bzo_utf8_reset(ctypes.byref(self._s))

    def write(self, data) -> bool:
        data = bytes(data)
        return bool(lib().bzo_utf8_write(ctypes.byref(self._s), data, len(data)))

    def finish(self) -> bool:
        return bool(lib().bzo_utf8_finish(ctypes.byref(self._s)))

    def reset(self):
        lib().bzo_utf8_reset(ctypes.byref(self._s))


# ------------------------------------------------------------ context takeover

def pmd_deflate_stream(msgs, level=6, wbits=15, mem_level=4, strategy=0):
    """One connection without no_context_takeover: one deflater for every
    message, never reset (impl_base.hpp:85-166).  Returns the payloads."""
    L = lib()
    z = L.bzo_deflate_new()
    try:
        if L.bzo_deflate_reset_params(z, level, wbits, mem_level, strategy):
            raise ValueError("invalid deflate parameters")
        out = []
        for m in msgs:
            m = bytes(m)
            cap = upper_bound(len(m)) + 64
            buf = ctypes.create_string_buffer(cap)
            src = ctypes.create_string_buffer(m, len(m)) if m else None
            n = L.bzo_pmd_deflate_msg(z, src, len(m), buf, cap)
            if n < 0:
                raise RuntimeError(f"deflate failed: {ERRORS.get(-n, -n)}")
            out.append(buf.raw[:n])
        return out
    finally:
        L.bzo_deflate_free(z)


def pmd_inflate_stream(payloads, cap: int = 1 << 20, wbits=15):
    """One connection's messages through one inflater that keeps its window
    (inflate_stream::clear() is a no-op, inflate_stream.ipp:49-53).  Returns
    [(status, output)]."""
    L = lib()
    z = L.bzo_inflate_new()
    try:
        if L.bzo_inflate_reset(z, wbits):
            raise ValueError("windowBits out of range")
        res = []
        for p in payloads:
            p = bytes(p)
            out = ctypes.create_string_buffer(max(cap, 1))
            got = ctypes.c_size_t(0)
            src = ctypes.create_string_buffer(p, len(p)) if p else None
            st = L.bzo_pmd_inflate_msg(z, src, len(p), out, cap, ctypes.byref(got), 0)
            res.append((st, out.raw[:got.value]))
        return res
    finally:
        L.bzo_inflate_free(z)


def ref_batch(inflate: bool, data, off, lens, out_cap, level=6, wbits=15, mem_level=4, threads=1):
    """The reference's zlib 1.3.1 over a batch (CPU baseline / calibration):
    inflate = payload + 00 00 FF FF with Z_SYNC_FLUSH, deflate = pmd framing.
    Returns (out, out_off, out_len) or None when libzref.so is absent."""
    R = ref()
    if R is None:
        return None
    n = len(lens)
    out_cap = np.ascontiguousarray(out_cap, dtype=np.uint32)
    out_off = np.zeros(n, dtype=np.uint64)
    if n:
        out_off[1:] = np.cumsum(out_cap[:-1].astype(np.uint64))
    out = np.zeros(int(out_cap.astype(np.uint64).sum()) + 1, dtype=np.uint8)
    out_len = np.zeros(n, dtype=np.uint32)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    R.zref_batch(1 if inflate else 0, level, wbits, mem_level, _p(data), _p(off), _p(lens), n, _p(out),
                 _p(out_off), _p(out_cap), _p(out_len), threads)
    return out, out_off, out_len


def time_batch(impl: str, inflate: bool, data, off, lens, out_cap, threads=1, reps=3, level=6, wbits=15,
               mem_level=4):
    """Median wall seconds of one batch call on the host cores, outputs
    preallocated outside the timed region.  impl: "port" (this C restatement
    of Beast's zlib), "reference" (the reference's zlib 1.3.1, oracle/_ref) or
    "system" (the image's zlib, oracle/libzsys.so).
    Returns (seconds, out_len) or None when the implementation is absent."""
    import time
    n = len(lens)
    out_cap = np.ascontiguousarray(out_cap, dtype=np.uint32)
    out_off = np.zeros(n, dtype=np.uint64)
    if n:
        out_off[1:] = np.cumsum(out_cap[:-1].astype(np.uint64))
    out = np.ones(int(out_cap.astype(np.uint64).sum()) + 1, dtype=np.uint8)   # touched: no page faults timed
    out_len = np.zeros(n, dtype=np.uint32)
    status = np.zeros(n, dtype=np.int32)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    if impl in ("reference", "system"):
        R = ref() if impl == "reference" else zsys()
        if R is None:
            return None
        call = lambda: R.zref_batch(1 if inflate else 0, level, wbits, mem_level, _p(data), _p(off), _p(lens), n,  # noqa: E731
                                    _p(out), _p(out_off), _p(out_cap), _p(out_len), threads)
    elif inflate:
        L = lib()
        call = lambda: L.bzo_pmd_inflate_batch(wbits, 0, _p(data), _p(off), _p(lens), n, _p(out), _p(out_off),  # noqa: E731
                                               _p(out_cap), _p(out_len), _p(status), threads)
    else:
        L = lib()
        call = lambda: L.bzo_pmd_deflate_batch(level, wbits, mem_level, 0, _p(data), _p(off), _p(lens), n,  # noqa: E731
                                               _p(out), _p(out_off), _p(out_cap), _p(out_len), _p(status), threads)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        call()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2], out_len.copy()
