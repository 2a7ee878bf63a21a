"""The multi-GPU path over RCCL (backend "nccl") at world size 1, on the one
GPU of the box: a fresh child process with the env a torch.distributed.run
rank gets (bench.py's launcher), dist.init_process_group("nccl",
device_id=...), the HIP segment compressor, the length all_gather on device
tensors (all_gather_into_tensor) and the gather assembly -- the framed
stream checked against the oracle.  The P2P leg of the gatherv (batched
isend/irecv between ranks) needs two GPUs: RCCL refuses two ranks on one
device, so it first runs on the driver's 8-GPU node.
Reference: the thread-per-block split of Algorithms/parallel/LZ4/LZ4.c:742
lifted to ranks (lz4jpeg/dist.py)."""
import hashlib
import json
import os
import socket
import subprocess
import sys

import pytest

import golden_inputs

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "lz4-jpeg_amd")

CHILD = r"""
import hashlib, json, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from lz4jpeg import dist as ldist
from lz4jpeg import lz4
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
try:
    assert dist.get_backend() == "nccl"
    data = open(sys.argv[2], "rb").read()
    n = len(data)
    world, rank = dist.get_world_size(), dist.get_rank()
    lo, hi = ldist.shard_bytes(n, world, rank)
    local = torch.from_numpy(np.frombuffer(data[lo:hi], dtype=np.uint8).copy()).to(dev)
    comp = lz4.Compressor()
    # a device-tensor all_gather_into_tensor and all_reduce straight over RCCL
    x = torch.tensor([12345 + rank], dtype=torch.int64, device=dev)
    g = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(g, x)
    r = torch.tensor([2.5], dtype=torch.float64, device=dev)
    dist.all_reduce(r, op=dist.ReduceOp.MAX)
    dist.barrier()
    full = ldist.compress_sharded(local, n, ldist.hip_segment_compressor(comp, final_shard=hi == n))
    torch.cuda.synchronize()
    comp.close()
    out = full.cpu().numpy().tobytes()
    print(json.dumps({"backend": dist.get_backend(), "world": world, "gathered": g.tolist(),
                      "reduced": float(r.item()), "len": len(out),
                      "md5": hashlib.md5(out).hexdigest()}), flush=True)
finally:
    dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_env():
    env = dict(os.environ)
    env.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONPATH"] = PKG + os.pathsep + env.get("PYTHONPATH", "")
    return env


def test_rccl_world1_segment_compress_and_gather(gpu, oracle, tmp_path):
    text = golden_inputs.lz4_input("metamorphosis_spaces")
    data = bytes(text[:300 * 1000 + 77])
    src = tmp_path / "in.bin"
    src.write_bytes(data)
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    res = subprocess.run([sys.executable, "-u", str(script), PKG, str(src)], env=_rank_env(),
                         capture_output=True, text=True, timeout=180)
    assert res.returncode == 0, res.stderr[-3000:]
    got = json.loads(res.stdout.strip().splitlines()[-1])
    expect = oracle.lz4_compress(data)
    assert got["backend"] == "nccl" and got["world"] == 1
    assert got["gathered"] == [12345] and got["reduced"] == 2.5
    assert got["len"] == len(expect)
    assert got["md5"] == hashlib.md5(expect).hexdigest()


def test_bench_distributed_path_at_world1(gpu):
    """bench.py's N > 1 code path (RCCL group, sharded workloads, length
    all_gather, gather on rank 0, max/sum over ranks) as one rank under the
    same launcher the driver uses, on small workloads."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--dist", "--lz4-total-bytes", str(16 << 20),
           "--jpeg-total-images", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    line = json.loads([l for l in res.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["scaling"] == "strong"
    assert line["config"]["workload"].endswith("_text_sharded_rccl_gather")
    assert line["lz4_gather_ok"] is True and line["value"] > 0
    assert line["lz4_decode"]["roundtrip_ok"] is True
    assert line["jpeg"]["value"] > 0
    # the fail-fast additions: per-rank times, the gather's piece size, the
    # phases each rank announces (its watchdog is armed per phase)
    pr = line["per_rank"]
    assert len(pr["call_ms"]) == 1 and pr["call_ms"][0] > 0 and len(pr["step_ms"]) == 1
    assert line["lz4_gather_chunk_bytes"] == 1 << 30
    for ph in ("init_process_group", "lz4 warm-up", "lz4 timed steps", "lz4 gather", "jpeg"):
        assert f"rank 0: phase {ph}" in res.stderr, ph
