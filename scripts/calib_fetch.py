"""FETCH_SIZE calibration for bench.py's roofline.traffic: reads 2 GiB (past
the 256 MiB Infinity Cache) once in each access pattern of
bpmd_diag_read_pattern.  Run under rocprofv3 --pmc FETCH_SIZE; the known
byte count divided by the counter gives the pattern's correction factor
(scripts/profile.sh writes it to profiles/<tag>_fetch_calib.csv)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from beast_amd import pmd  # noqa: E402


def main():
    L = pmd.lib()
    L.bpmd_diag_read_pattern.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p]
    nbytes = 2 << 30
    buf = torch.ones(nbytes, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    for mode in (0, 1):
        for _ in range(2):
            assert L.bpmd_diag_read_pattern(ctypes.c_void_p(buf.data_ptr()), nbytes, mode,
                                            ctypes.c_void_p(sink.data_ptr()), None) == 0
        torch.cuda.synchronize()
    print(f"read {nbytes} bytes per launch; launches: mode 0 x2, mode 1 x2")


if __name__ == "__main__":
    main()
