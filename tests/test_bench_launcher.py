"""bench.py --gpus N starts its own rank processes (CPU; no GPU call is made).

The driver may run `python bench.py --gpus 8` with no launcher around it. bench.py then
starts N ranks through torch.distributed.run before torch or libbhrt is imported, so the
parent never initialises HIP (no process that touched the GPU ever starts another program).
BHRT_BENCH_DRYRUN=1 makes every rank print its environment and stop before its first GPU
call, and the parent report whether it ever mapped libamdhip64 or imported torch.
"""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _run(*args, env_extra=None):
    env = dict(os.environ, BHRT_BENCH_DRYRUN="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                       capture_output=True, text=True, timeout=240)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p, lines


def test_gpus_2_launches_two_ranks_from_a_gpu_free_parent():
    p, lines = _run("--gpus", "2", "--steps", "1", "--warmup", "0")
    assert p.returncode == 0, p.stderr[-3000:]
    ranks = [x for x in lines if "rank" in x]
    launcher = [x for x in lines if x.get("launcher")]
    assert sorted(x["rank"] for x in ranks) == [0, 1]
    assert sorted(x["local_rank"] for x in ranks) == [0, 1]
    assert sorted(x["device"] for x in ranks) == [0, 1]  # one GPU per rank
    assert all(x["world_size"] == 2 and x["master_addr"] == "127.0.0.1" for x in ranks)
    assert len({x["master_port"] for x in ranks}) == 1
    assert launcher == [{"launcher": True, "rc": 0, "hip_loaded": False,
                         "torch_imported": False}]


def test_gpus_1_runs_in_process():
    p, lines = _run("--gpus", "1")
    assert p.returncode == 0, p.stderr[-3000:]
    assert lines == [{"rank": 0, "local_rank": 0, "world_size": 1, "master_addr": None,
                      "master_port": None, "device": 0}]


def test_rehearsal_maps_every_rank_to_gpu_0():
    p, lines = _run("--gpus", "2", env_extra={"BHRT_BENCH_SHARE_DEVICE": "1"})
    assert p.returncode == 0, p.stderr[-3000:]
    assert sorted(x["device"] for x in lines if "rank" in x) == [0, 0]


def test_a_launcher_environment_is_respected():
    """Under an outer launcher (WORLD_SIZE set) bench.py does not launch again."""
    p, lines = _run("--gpus", "2", env_extra={"WORLD_SIZE": "2", "RANK": "1",
                                              "LOCAL_RANK": "1"})
    assert p.returncode == 0, p.stderr[-3000:]
    assert lines == [{"rank": 1, "local_rank": 1, "world_size": 2, "master_addr": None,
                      "master_port": None, "device": 1}]


def test_a_failing_rank_fails_the_launch():
    """--gpus 2 with a mismatching outer world size exits non-zero in each rank; the parent
    returns the launcher's non-zero code."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--streams", "3"],
                       env={k: v for k, v in os.environ.items()
                            if k not in ("WORLD_SIZE", "BHRT_BENCH_DRYRUN")},
                       capture_output=True, text=True, timeout=240)
    assert p.returncode != 0
