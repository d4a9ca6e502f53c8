"""Event counts of the per-stream inflater on C1's call pattern, from the host
build of the kernel's own source (tests/model/zstream_host.py with
-DBPMD_ZS_HOST_COUNT): how many symbols the slow path decodes per message,
how many inflate_fast tokens, block headers, calls.  Payloads from the
oracle's Beast deflate_stream (context takeover, level 6, memLevel 4), read
as websocket::stream does (rd_buf slices, then the 4-byte tail).
    ZS_HOST_FLAGS=-DBPMD_ZS_HOST_COUNT python scripts/zstream_host_counts.py [messages] [size]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ZS_HOST_FLAGS", "-DBPMD_ZS_HOST_COUNT")
from tests import zstream_cases as Z  # noqa: E402
from tests.model import zstream_host as H  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    msgs = Z.msgs_of("json", [size] * n, seed=0x5EED0001)
    pays = O.pmd_deflate_stream(msgs, 6, 15, 4)
    inf = H.HostInflater()
    cnt = (ctypes.c_ulonglong * 32).in_dll(inf.L, "zs_host_counts")
    calls = 0
    for i, p in enumerate(pays):
        if i == 8:
            for j in range(32):
                cnt[j] = 0
            calls = 0
        for chunk in ([p[k:k + 1536] for k in range(0, len(p), 1536)] or [b""]) + [Z.EB]:
            src = ctypes.create_string_buffer(chunk, max(1, len(chunk)))
            buf = ctypes.create_string_buffer(4096)
            zs = Z.ZParams(ctypes.addressof(src), len(chunk), 0, ctypes.addressof(buf), 4096, 0, 0)
            inf.write(zs, Z.SYNC)
            calls += 1
    k = n - 8
    print(f"{k} messages of {size} B, {calls / k:.1f} calls per message; per message: "
          f"{cnt[10] / k:.1f} serial inflate_fast tokens, {cnt[22] / k:.1f} parallel ones in {cnt[21] / k:.1f} windows, "
          f"{cnt[24] / k:.1f} slow-path symbol decodes, {cnt[25] / k:.1f} code-length symbols in parallel windows, {cnt[26] / k:.1f} block headers, {cnt[9] / k:.1f} copies, "
          f"{cnt[12] / k:.1f} stagings")


if __name__ == "__main__":
    main()
