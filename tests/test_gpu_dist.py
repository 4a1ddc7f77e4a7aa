"""Multi-rank rehearsal on the one-GPU box: N ranks, all on cuda:0,
gloo for the collectives — the process topology, weight broadcast, sharding and gather
that the 8-GPU RCCL run uses, with the wavs checked.

* ``dist.vocode_sharded`` under world size 2: C3 (V1 [64, 80, 1024]) and C5 (the reference
  SAM-BERT acoustic model's 32 ragged utterances) — each gathered wav BITWISE equal to the
  single-process forward of the whole batch (tests/tools/dist_world2_check.py).
* ``bench.py --gpus 2 --dist-backend gloo`` with no launcher: bench.py starts the 2 ranks
  itself and rank 0 reports ``n_gpus: 2`` (world size observed = 2, per-rank step times).

Ranks are child processes started with torch.distributed.run (never exec'd in place).
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _last_json(stdout):
    for line in reversed(stdout.strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError("no JSON line in:\n" + stdout[-2000:])


def test_world2_vocode_sharded_bitwise(dev):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "tools", "dist_world2_check.py")]
    r = subprocess.run(["timeout", "-k", "10", "240"] + cmd, cwd=ROOT, capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    res = _last_json(r.stdout)
    print("\n" + json.dumps(res, indent=1))
    assert res["world"] == 2
    assert set(res["checks"]) == {"C3_v1_64x80x1024/f16x3", "C5_sambert_b32/f16x3",
                                  "C5_sambert_b32/fp32"}
    for name, chk in res["checks"].items():
        assert chk["bitwise_vs_single_process"], name
        assert sum(chk["per_rank_items"]) == chk["items"] and min(chk["per_rank_items"]) > 0
        if "max_err_vs_reference_wav" in chk:
            assert chk["max_err_vs_reference_wav"] < 1e-4, name


def test_nccl_world1_vocode_sharded_bitwise(dev):
    """The RCCL branch on the one-GPU box: one rank under
    torch.distributed.run, backend nccl, device_id set — the weight broadcast and
    vocode_sharded's batch broadcast (src=0) on device buffers, each wav bitwise the
    single-process forward.  Point-to-point sends need two GPUs: left to the 8-GPU run."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "tools", "dist_world2_check.py")]
    env = dict(os.environ, HFG_DIST_BACKEND="nccl")
    r = subprocess.run(["timeout", "-k", "10", "240"] + cmd, cwd=ROOT, capture_output=True,
                       text=True, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    res = _last_json(r.stdout)
    print("\n" + json.dumps(res, indent=1))
    assert res["world"] == 1 and res["backend"] == "nccl"
    assert res["weights_on"].startswith("cuda")
    assert set(res["checks"]) == {"C3_v1_64x80x1024/f16x3", "C5_sambert_b32/f16x3",
                                  "C5_sambert_b32/fp32"}
    for name, chk in res["checks"].items():
        assert chk["bitwise_vs_single_process"], name
        if "max_err_vs_reference_wav" in chk:
            assert chk["max_err_vs_reference_wav"] < 1e-4, name


def test_bench_gpus1_nccl(dev):
    """bench.py --dist-backend nccl --force-dist at N = 1: the bench's RCCL branch
    (init_process_group("nccl", device_id=...), the flat weight broadcast on the GPU) runs
    and reports world size 1."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dist-backend", "nccl", "--force-dist",
           "--steps", "2", "--warmup", "1", "--no-extra", "--no-cpu-baseline", "--no-pmc", "--also"]
    r = subprocess.run(["timeout", "-k", "10", "300"] + cmd, cwd=ROOT, capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    print("\n" + json.dumps({k: line.get(k) for k in ("n_gpus", "value", "world_size_observed",
                                                       "dist_backend", "launch")}))
    assert line["n_gpus"] == 1 and line["world_size_observed"] == 1
    assert line["dist_backend"] == "nccl"


def test_bench_gpus2_self_launch(dev):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--steps", "2", "--warmup", "1", "--no-extra", "--no-cpu-baseline", "--no-pmc",
           "--also"]
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(["timeout", "-k", "10", "300"] + cmd, cwd=ROOT, capture_output=True,
                       text=True, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    print("\n" + json.dumps({k: line[k] for k in ("n_gpus", "value", "value_per_gpu",
                                                   "per_rank_ms_per_step", "world_size_observed",
                                                   "launch")}))
    assert line["n_gpus"] == 2 and line["world_size_observed"] == 2
    assert line["launch"] == "self-launched torch.distributed.run"
    assert len(line["per_rank_ms_per_step"]) == 2
    assert line["config"]["global_batch"] == 16
    assert abs(line["value_per_gpu"] * 2 - line["value"]) < 1e-6 * line["value"]
