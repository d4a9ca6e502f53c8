"""Per-call latency of the per-stream facade (bpmd_{deflate,inflate}_stream_*,
behind the drop-in zlib headers) on configs[0]'s shape: 1 KiB JSON messages,
one never-reset deflater and inflater (context takeover), websocket::stream's
call pattern (tests/test_gpu_stream.py ws_deflate_message / ws_inflate_message).
Prints per-message host times; run under rocprofv3 --kernel-trace for the
kernels each message launches.
    python scripts/facade_latency.py [messages]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import synth  # noqa: E402
from tests import test_gpu_stream as S  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    busy = os.environ.get("BPMD_LAT_BUSY")   # a spin kernel on a side stream meanwhile (clock ramp check)
    if busy:
        import torch
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            for _ in range(int(busy)):
                torch.cuda._sleep(1 << 30)
    L = S._lib()
    zo, zi = S._mk(L, True, 8), S._mk(L, False)
    data, off, ln = synth.make_batch("json", [1024] * n, seed=0x5EED0001)
    msgs = [bytes(data[int(off[i]):int(off[i]) + 1024]) for i in range(n)]
    td = ti = 0.0
    for i, m in enumerate(msgs):
        t0 = time.perf_counter()
        p = S.ws_deflate_message(L, zo, m)
        t1 = time.perf_counter()
        back = S.ws_inflate_message(L, zi, p)
        t2 = time.perf_counter()
        assert back == m, i
        if i >= 8:
            td += t1 - t0
            ti += t2 - t1
    k = n - 8
    print(f"{'busy ' if busy else ''}facade per message: deflate {td / k * 1e6:.1f} us, inflate {ti / k * 1e6:.1f} us "
          f"(ws_deflate_message: none/block/sync writes; ws_inflate_message: rd_buf slices + the 4-byte tail)")
    L.bpmd_stream_destroy(zo)
    L.bpmd_stream_destroy(zi)


if __name__ == "__main__":
    main()
