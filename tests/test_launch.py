"""`bench.py --gpus N` starts its own N ranks when no launcher did (nldsc_amd/launch.py), and refuses a rank count
or a device count that does not match --gpus — checked on CPU: the launch mechanism with a gloo stand-in for the
bench body, and bench.py's own checks, which run before anything touches a GPU."""
import json
import os
import subprocess
import sys

from conftest import REPO

RANK_SCRIPT = r'''
import json, os, sys
sys.path.insert(0, {repo!r})
from nldsc_amd.launch import ranks_or_spawn
gpus = int(sys.argv[sys.argv.index("--gpus") + 1])
rc = ranks_or_spawn(os.path.abspath(__file__), sys.argv[1:], gpus, "gloo")
if rc is not None:
    sys.exit(rc)
import torch
import torch.distributed as dist
world = int(os.environ.get("WORLD_SIZE", "1"))
if world > 1:
    dist.init_process_group("gloo")
x = torch.tensor([float(int(os.environ.get("RANK", "0")) + 1)])
if world > 1:
    dist.all_reduce(x)
    assert dist.get_world_size() == gpus
if int(os.environ.get("RANK", "0")) == 0:
    print(json.dumps({{"n_gpus": world, "rank_sum": x.item()}}), flush=True)
if world > 1:
    dist.destroy_process_group()
'''


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_gpus_n_spawns_n_ranks_and_relays_rank0_line(tmp_path):
    script = tmp_path / "ranks.py"
    script.write_text(RANK_SCRIPT.format(repo=REPO))
    p = subprocess.run([sys.executable, str(script), "--gpus", "3"], env=_env(), capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # exactly rank 0's line
    d = json.loads(lines[0])
    assert d == {"n_gpus": 3, "rank_sum": 6.0}


def test_gpus_1_runs_in_process(tmp_path):
    script = tmp_path / "ranks.py"
    script.write_text(RANK_SCRIPT.format(repo=REPO))
    p = subprocess.run([sys.executable, str(script), "--gpus", "1"], env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0 and json.loads(p.stdout.strip().splitlines()[-1])["n_gpus"] == 1, p.stderr[-2000:]


def test_bench_refuses_world_size_other_than_gpus():
    env = dict(_env(), WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3", "--no-cpu", "--no-file"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr, p.stderr[-2000:]


def test_bench_rccl_needs_one_device_per_rank():
    """With the RCCL backend, --gpus N needs N visible devices (here: none); the check runs before any GPU call."""
    import torch
    if torch.cuda.device_count() >= 2:
        return  # a multi-GPU host: nothing to refuse
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--no-cpu", "--no-file"],
                       env=_env(), capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "HIP devices visible" in p.stderr, p.stderr[-2000:]
