"""Shard / gather ARITHMETIC only (world-size-2 gloo, CPU): sequences are sharded across ranks with no
collective on the data path; the only exchange is the final all-gather of per-sequence trajectories to
rank 0.  The oracle stands in for each rank's device here; tests/test_gpu_dist.py runs the product path
(bench.py under torch.distributed.run, lego_amd.Batch on the HIP library)."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

import make_golden as MG
from lego_amd import _abi as A


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def shard(rank, world, n_seq):
    """Sequence ids owned by a rank (contiguous blocks, as bench.py assigns them)."""
    per = n_seq // world
    return list(range(rank * per, rank * per + per))


def run_sequences(seqs, nscans):
    import oracle as O
    import torch
    params = MG.params_for("vlp16")
    cfg = A.synth_cfg("vlp16")
    out = []
    for s in seqs:
        orc = O.Oracle(params)
        for k in range(nscans):
            orc.cloud_handler(A.synth_scan(cfg, s, k))
            fa = orc.feature_association()
        out.append(np.concatenate([[s], fa["transform_cur"], fa["transform_sum"]]).astype(np.float64))
    return torch.tensor(np.stack(out))


def _worker(rank, world, port, nseq, nscans, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    mine = run_sequences(shard(rank, world, nseq), nscans)
    gathered = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    if rank == 0:
        q.put(torch.cat(gathered).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_and_gather_arithmetic_with_oracle_ranks():
    world, nseq, nscans = 2, 4, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nseq, nscans, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = run_sequences(list(range(nseq)), nscans).numpy()
    assert got.shape == (nseq, 13)
    np.testing.assert_array_equal(got[:, 0], np.arange(nseq))
    # each rank processed its shard independently: identical to a single-process run
    np.testing.assert_array_equal(got, ref)
