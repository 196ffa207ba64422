"""bench.py's multi-GPU entry: `python bench.py --gpus N` with no WORLD_SIZE starts torch.distributed.run
as ONE child (one rank per GPU) before any GPU call and passes rank 0's JSON line through."""
import json
import os
import subprocess
import sys

import bench


def test_launcher_command_for_two_ranks():
    cmd, env = bench.launcher_cmd(["--gpus", "2", "--steps", "3"], 2, 29517)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29517"
    assert cmd[-4:] == [os.path.abspath(bench.__file__), "--gpus", "2", "--steps", "3"][-4:]
    assert os.path.abspath(bench.__file__) in cmd
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["MASTER_ADDR"] == "127.0.0.1"


def test_launcher_runs_one_process_per_rank(tmp_path):
    """The same command over a stand-in script (CPU: no GPU is touched): two ranks start with the
    rendezvous environment and rank 0's line reaches the parent's stdout."""
    probe = tmp_path / "probe.py"
    probe.write_text("import json, os\n"
                     "r = int(os.environ['RANK'])\n"
                     "print(json.dumps({'rank': r, 'world': int(os.environ['WORLD_SIZE'])}) if r == 0 else '', "
                     "flush=True)\n")
    cmd, env = bench.launcher_cmd(["--gpus", "2"], 2, 0, script=str(probe))
    cmd[cmd.index("--master-port") + 1] = "0"
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert lines == [{"rank": 0, "world": 2}]
