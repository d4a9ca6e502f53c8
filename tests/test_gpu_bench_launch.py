"""GPU: `python bench.py --gpus 2` without a launcher starts two ranks
(torch.distributed.run as a child process) and reports n_gpus == 2.  The box
has one GPU and RCCL refuses two ranks on one device, so the rehearsal runs
the ranks' collectives over gloo (BPMD_BENCH_BACKEND=gloo), both ranks on
cuda:0, on a small C2 batch."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_2_launches_two_ranks():
    env = dict(os.environ, BPMD_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--msgs", "4096", "--no-mixed", "--no-cpu-baseline", "--no-deflate", "--no-frame"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 prints the one line
    line = lines[0]
    assert line["n_gpus"] == 2 and line["parity_ok"]
    assert "dp2" in line["config"]["parallelism"]
