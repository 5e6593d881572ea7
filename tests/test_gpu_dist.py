"""The multi-GPU path with the product: bench.py launched by torch.distributed.run with two
ranks, each running its own 8 sequences through lego_amd.Batch on the HIP library, the trajectories
all-gathered to rank 0 and the step time max-reduced over ranks.  On a one-GPU box both ranks share
cuda:0 and the collectives run over gloo (RCCL over xGMI is the driver's 8-GPU run).  Rank 0's gathered
poses must equal one process running the same 16 sequences.  The C5 dataset mode (--config c5: sequences
sharded over the ranks, every scan's odometry recorded on the device and gathered) is run the same way
at a reduced size and checked against one process and the oracle.  (tests/test_dist_shard_arith_cpu.py
checks only the shard / gather arithmetic, on the oracle.)"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-alt-order", "--roofline-streams", "0",
          "--roofline-reps", "2", "--threads", "4"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


def test_torchrun_two_ranks_match_single_process(gpu, tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    p2, p1 = str(tmp_path / "poses2.npy"), str(tmp_path / "poses1.npy")
    cmd2 = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
            "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2",
            "--dist-backend", "gloo", "--streams", "8", "--dump-poses", p2, "--no-c5"] + COMMON
    r2 = subprocess.run(cmd2, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, universal_newlines=True, env=env,
                        timeout=300, cwd=REPO)
    assert r2.returncode == 0, r2.stdout[-3000:]
    d2 = _json_line(r2.stdout)
    assert d2["n_gpus"] == 2 and d2["trajectories_gathered"] == 16 and d2["scaling"] == "weak"
    assert d2["value"] > 0 and d2["config"]["streams_per_gpu"] == 8
    cmd1 = [sys.executable, os.path.join(REPO, "bench.py"), "--streams", "16", "--dump-poses", p1, "--no-c5"] + COMMON
    r1 = subprocess.run(cmd1, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, universal_newlines=True, env=env,
                        timeout=300, cwd=REPO)
    assert r1.returncode == 0, r1.stdout[-3000:]
    d1 = _json_line(r1.stdout)
    assert d1["n_gpus"] == 1 and d1["trajectories_gathered"] == 16
    a2, a1 = np.load(p2), np.load(p1)
    assert a2.shape == a1.shape == (16, 12)
    assert np.array_equal(a2.view(np.int32), a1.view(np.int32)), np.abs(a2 - a1).max()


def test_torchrun_c5_two_ranks_match_single_process_and_oracle(gpu, tmp_path):
    """--config c5 at 5 sequences x 6 scans: rank 0 holds sequences 0-2, rank 1 sequences 3-4 (padded
    gather); the gathered per-scan odometry equals one process's bit for bit and the oracle's within 1e-4."""
    import helpers as Hs
    import lego_amd as L
    import oracle as O
    from lego_amd import _abi as A
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    small = ["--config", "c5", "--c5-sequences", "5", "--c5-scans", "6"]
    p2, p1 = str(tmp_path / "c5_2.npy"), str(tmp_path / "c5_1.npy")
    cmd2 = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
            "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2",
            "--dist-backend", "gloo", "--streams", "4", "--dump-c5", p2] + small + COMMON
    r2 = subprocess.run(cmd2, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, universal_newlines=True, env=env,
                        timeout=300, cwd=REPO)
    assert r2.returncode == 0, r2.stdout[-3000:]
    d2 = _json_line(r2.stdout)
    assert d2["n_gpus"] == 2 and d2["scaling"] == "strong" and d2["c5"]["sequences_per_rank"] == 3
    assert d2["c3"]["scaling"] == "weak" and d2["value"] == d2["c5"]["value"] > 0
    cmd1 = [sys.executable, os.path.join(REPO, "bench.py"), "--streams", "4", "--dump-c5", p1] + small + COMMON
    r1 = subprocess.run(cmd1, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, universal_newlines=True, env=env,
                        timeout=300, cwd=REPO)
    assert r1.returncode == 0, r1.stdout[-3000:]
    d1 = _json_line(r1.stdout)
    assert d1["n_gpus"] == 1 and d1["c5"]["sequences_per_rank"] == 5
    a2, a1 = np.load(p2), np.load(p1)
    assert a2.shape == a1.shape == (5, 6, 12)
    assert np.array_equal(a2.view(np.int32), a1.view(np.int32)), np.abs(a2 - a1).max()
    params = L.params_vlp16()
    cfg = A.synth_cfg("vlp16")
    for s in range(5):
        orc = O.Oracle(params)
        for k in range(6):
            orc.cloud_handler(A.synth_scan(cfg, 100000 + s, k))
            fr = orc.feature_association()
            np.testing.assert_allclose(a1[s, k, :6], fr["transform_cur"], atol=Hs.TF_TOL, rtol=0)
            np.testing.assert_allclose(a1[s, k, 6:], fr["transform_sum"], atol=Hs.TF_TOL, rtol=0)
