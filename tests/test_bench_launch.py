"""bench.py's multi-GPU plumbing on CPU: --gpus N self-launches N ranks (one
process per GPU) before any GPU call, each rank reads RANK / WORLD_SIZE /
LOCAL_RANK, and the shares are configs 4/5 (64 GiB in whole 300-B blocks,
1024 images) split without gaps."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_self_launch_runs_n_ranks():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--launch-check"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["local_rank"] == x["rank"] for x in lines)
    by = {x["rank"]: x for x in lines}
    assert by[0]["lz4_shard"][0] == 0 and by[1]["lz4_shard"][1] == 64 << 30
    assert by[0]["lz4_shard"][1] == by[1]["lz4_shard"][0]
    assert by[0]["lz4_shard"][1] % 300 == 0
    assert by[0]["jpeg_images"] == [0, 512] and by[1]["jpeg_images"] == [512, 1024]
    assert all(x["scaling"] == "strong" for x in lines)


def test_no_self_launch_under_a_launcher_or_for_one_gpu():
    class A:
        gpus = 8
    assert bench.maybe_self_launch(A, [], env={"WORLD_SIZE": "8"}) is None
    A.gpus = 1
    assert bench.maybe_self_launch(A, [], env={}) is None


def test_dist_rehearsal_self_launches_one_rank():
    """--dist at one GPU: the N > 1 code path as one launcher rank (the RCCL
    rehearsal tests/test_gpu_rccl.py runs on the box); sharded workloads."""
    class A:
        gpus = 1
        dist = True
        lz4_bytes_per_rank = 1 << 30
        jpeg_images_per_rank = 1
        lz4_total_bytes = 0
        jpeg_total_images = 0
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--dist",
                        "--launch-check"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["world"] == 1 and lines[0]["scaling"] == "strong"
    assert lines[0]["lz4_shard"] == [0, 64 << 30]
    assert bench.workloads(1, A) == (64 << 30, 1024, "strong")


def test_launcher_command_is_one_node_loopback():
    cmd = bench.launcher_cmd(4, ["--gpus", "4", "--steps", "3"], 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert "--nnodes=1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "3"]


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_workload_shares_cover(world):
    class A:
        lz4_bytes_per_rank = 1 << 30
        jpeg_images_per_rank = 1
        lz4_total_bytes = 0
        jpeg_total_images = 0
    lz4_total, imgs, scaling = bench.workloads(world, A)
    if world == 1:
        assert (lz4_total, imgs, scaling) == (1 << 30, 1, "weak")
    else:
        assert (lz4_total, imgs, scaling) == (64 << 30, 1024, "strong")
    prev = 0
    for r in range(world):
        i0, i1 = bench.image_share(imgs, world, r)
        assert i0 == prev and i1 >= i0
        prev = i1
    assert prev == imgs
    assert bench.rank_env({"WORLD_SIZE": str(world), "RANK": "0", "LOCAL_RANK": "0"}) == \
        (world, 0, 0)


def test_cpu_cores_positive():
    assert bench.host_cpu_cores() >= 1


def test_phase_watchdog_ends_a_stuck_rank():
    """bench.phase(): a rank whose phase outlives its limit (a collective that
    never completes on the first 8-GPU run) dumps every thread's stack and
    exits non-zero with the phase named, instead of sitting until the
    driver's limit kills the run silently."""
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "bench.phase('lz4 gather', 3, 2); time.sleep(60)" % REPO)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=50)
    assert r.returncode != 0
    assert "rank 3: phase lz4 gather" in r.stderr
    assert "Timeout" in r.stderr and "time.sleep" not in r.stdout     # faulthandler's dump


def test_phase_watchdog_is_rearmed_per_phase():
    """Each phase() call replaces the previous deadline: a run whose phases
    each finish in time is not killed however long the whole run takes."""
    code = ("import faulthandler, sys, time; sys.path.insert(0, %r); import bench\n"
            "for k in range(4):\n"
            "    bench.phase('p%%d' %% k, 0, 2); time.sleep(1)\n"
            "faulthandler.cancel_dump_traceback_later(); print('done')" % REPO)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=50)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip() == "done"
