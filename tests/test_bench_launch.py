"""bench.py --gpus N: the launcher starts N ranks (one process per GPU) as a
child process, and a rank refuses a WORLD_SIZE that is not N.  CPU tests: the
command, the mismatch rule, and a real 2-rank torch.distributed.run over a
probe script (gloo) that reports what each rank saw.  The GPU rehearsal of
the bench itself is tests/test_gpu_bench_launch.py."""
import json
import os
import subprocess
import sys
import types


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launch_cmd_is_torchrun_on_loopback():
    cmd = bench.launch_cmd(["--gpus", "4", "--steps", "5"], 4, 29555, python="py")
    assert cmd[:3] == ["py", "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "5"]


def test_world_size_mismatch_is_refused(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.maybe_launch(types.SimpleNamespace(gpus=4), []) == 2
    assert bench.maybe_launch(types.SimpleNamespace(gpus=2), []) is None


def test_single_gpu_runs_in_process(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.maybe_launch(types.SimpleNamespace(gpus=1), []) is None


PROBE = r"""
import json, os, sys
import torch.distributed as dist
dist.init_process_group("gloo")
import torch
t = torch.tensor([int(os.environ["RANK"])])
dist.all_reduce(t)
# one file per rank: the ranks share the launcher's stdout, whose lines can interleave
with open(os.path.join(os.environ["PROBE_DIR"], "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({"rank": int(os.environ["RANK"]), "world": int(os.environ["WORLD_SIZE"]),
               "sum": int(t), "argv": sys.argv[1:]}, f)
dist.destroy_process_group()
"""


def test_launcher_starts_two_gloo_ranks(tmp_path, monkeypatch):
    probe = tmp_path / "probe.py"
    probe.write_text(PROBE)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("PROBE_DIR", str(tmp_path))
    cmd = bench.launch_cmd(["--gpus", "2"], 2, bench._free_port(), script=str(probe))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.load(open(tmp_path / f"rank{k}.json")) for k in range(2)]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["sum"] == 1 and x["argv"] == ["--gpus", "2"] for x in lines)
