"""Where a per-stream inflate call's time goes: the prof build's per-phase
cycle counters of zstream_write_kernel (pmd_zstream.hip, -DBPMD_PROF) over
configs[0]'s call pattern (1 KiB JSON messages, context takeover, the
facade's rd_buf slices + 4-byte tail; scripts/facade_latency.py).
    BPMD_LIB=beast_amd/libbeast_pmd_prof.so python scripts/diag_zstream.py [messages]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import synth  # noqa: E402
from tests import test_gpu_stream as S  # noqa: E402
from scripts.diag_deflate import NAMES as DNAMES  # noqa: E402

NAMES = ["entry (state in)", "block header", "table builds", "inflate_fast", "window load", "match copies",
         "done + state out", "whole call", "input staging"]
COUNTS = ["copies", "fast tokens", "output bytes", "stagings", "calls", "input bytes"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    L = S._lib()
    L.bpmd_diag_zstream_counters.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    zo, zi = S._mk(L, True, 8), S._mk(L, False)
    data, off, ln = synth.make_batch("json", [size] * n, seed=0x5EED0001)
    msgs = [bytes(data[int(off[i]):int(off[i]) + size]) for i in range(n)]
    L.bpmd_diag_deflate_counters.argtypes = [ctypes.c_void_p, ctypes.c_int]
    c = (ctypes.c_ulonglong * 32)()
    dc = (ctypes.c_ulonglong * 32)()
    for i, m in enumerate(msgs):
        if i == 8:
            L.bpmd_diag_zstream_counters(c, 1)
            L.bpmd_diag_deflate_counters(dc, 1)
        p = S.ws_deflate_message(L, zo, m)
        assert S.ws_inflate_message(L, zi, p) == m, i
    L.bpmd_diag_zstream_counters(c, 0)
    L.bpmd_diag_deflate_counters(dc, 0)
    k = n - 8
    calls = max(1, c[13])
    print(f"{k} messages of {size} B, {c[13]} calls; per message: {c[14] / k:.0f} input bytes, {c[11] / k:.0f} output bytes, "
          f"{c[10] / k:.0f} fast-loop tokens, {c[9] / k:.0f} match copies, {c[12] / k:.1f} input stagings")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:18s} {c[i] / k:10.0f} cycles per message ({c[i] / calls:9.0f} per call)")
    if c[21]:   # the wave-parallel inflate_fast
        print(f"  pfast: {c[21] / k:.1f} windows and {c[22] / k:.0f} tokens per message, {c[20] / k:.0f} cycles "
              f"({c[20] / max(1, c[22]):.0f} per token): staging {c[15] / k:.0f}, candidates {c[16] / k:.0f}, "
              f"chain {c[17] / k:.0f}, output {c[18] / k:.0f}")
        print(f"  outside inflate_fast and the header: {(c[7] - c[20] - c[3] - c[1] - c[0] - c[6]) / k:.0f} cycles per message")
    if c[19]:   # the laps build (-DBPMD_ZSTREAM_LAPS): inside inflate_fast, per token
        lap = c[19] / max(1, c[10])
        print(f"  laps build, cycles per fast-loop token (one lap = {lap:.0f}, not subtracted):")
        for i, nm in ((15, "refill + lookup"), (16, "literal store"), (17, "length + distance decode"),
                      (23, "match copies"), (18, "loop tail")):
            print(f"    {nm:26s} {c[i] / max(1, c[10]):8.0f}")
    if c[27] + c[28] + c[29] + c[30]:   # switch trips by mode (nested laps included)
        print(f"  by mode: type {c[27] / k:.0f}, stored {c[28] / k:.0f}, dynamic header {c[29] / k:.0f}, "
              f"LEN..LIT {c[30] / k:.0f}, other {c[31] / k:.0f} cycles per message; "
              f"{c[24] / k:.1f} slow-path symbols, {c[25] / k:.1f} code-length symbols in hdr_par windows, "
              f"{c[26] / k:.1f} block headers")
    if c[9]:
        print(f"  cycles per match copy {c[5] / c[9]:.0f}; per fast-loop token {c[3] / max(1, c[10]):.0f}")
    print("deflate (chunk kernel phases, per message):")
    for i in sorted(DNAMES):
        print(f"  {DNAMES[i]:>28}: {dc[i] / k:12.0f}")
    L.bpmd_stream_destroy(zo)
    L.bpmd_stream_destroy(zi)


if __name__ == "__main__":
    main()
