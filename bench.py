#!/usr/bin/env python3
"""Throughput benchmark: scans/s of LeGO-LOAM-BOR's per-scan path (project + segment + features + LM)
on synthetic VLP-16 sweeps, one process per GPU.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--streams S] [--kind vlp16|hdl64]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W

A step advances every one of the S independent sequences ("streams") on a GPU by one scan: one
launch per stage for all of them (lego_batch_step).  Inputs of all W+K steps are generated on the
host, uploaded, and resident in HBM before the timed region.  Each rank owns its own S sequences
(weak scaling, no collective on the data path); after timing, the per-stream trajectories are
all-gathered to rank 0 (RCCL), the only collective.  Rank 0 prints one JSON line.

The measured path runs PCL VoxelGrid with voxel_tie_order = 0: libstdc++ std::sort's permutation of
equal leaf indices, bit-identical to the GCC-built reference (--voxel-tie-order 1: each voxel's points
summed in point order, std::stable_sort's).  At N = 1 the other order is measured too on the same
inputs and reported as "other_voxel_tie_order" (--no-alt-order skips it).

The roofline pair's durations are reported twice: launched back to back (roofline.launch_ms, the
kernels' own time) and inside the timed pipeline, where the previous scan's LM shares the CUs
(roofline.in_pipeline: events around the two stages of every step of a third pass over the same
steps, lego_batch_set_probe).

The roofline pair (k_project + k_fa_prep4) is also timed at --roofline-streams scans per launch (2048:
a working set far above the 256 MiB Infinity Cache) and reported beside the S-stream figure.

BASELINE's configs:  --config c3 (default) is the headline: S streams per GPU, weak scaling.  Every line
also carries "c5": BASELINE config C5, the 20k-scan synthetic dataset (80 sequences x 250 scans) sharded
by sequence over the N ranks (80 / N sequences each, strong scaling), every scan of it timed; --config
c5 makes that the headline value (--c5-sequences / --c5-scans shrink it for tests; --no-c5 skips it).
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lego-loam-bor_amd"))

METRIC = "scans/sec (project+segment+features+LM) on VLP-16 sweeps, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--streams", type=int, default=256, help="independent sequences per GPU")
    ap.add_argument("--kind", default="vlp16", choices=["vlp16", "hdl64"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (rank 0)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--roofline-reps", type=int, default=20,
                    help="back-to-back k_project + k_fa_prep4 pairs timed for the roofline")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="threads of the all-cores CPU variant (one sequence per thread; the box's CPU share)")
    ap.add_argument("--threads", type=int, default=16, help="host threads for input generation")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL over xGMI) or gloo (test rehearsal)")
    ap.add_argument("--groups", type=int, default=1, help="stream slices launched on separate HIP streams")
    ap.add_argument("--wide", type=int, default=-1, choices=[-1, 0, 1, 2],
                    help="projection / segmentation layout (lego_batch_set_wide): -1 automatic")
    ap.add_argument("--lag", type=int, default=None, choices=[0, 1, 2],
                    help="pipeline depth (lego_batch_set_lag): 1 = a step runs the previous scan's LM, 2 = the one "
                         "before; default automatic (DESIGN §4)")
    ap.add_argument("--voxel-tie-order", type=int, default=0, choices=[0, 1],
                    help="lego_params.voxel_tie_order of the measured path: 0 = libstdc++ std::sort order, "
                         "bit-identical to the GCC-built reference; 1 = VoxelGrid sums each voxel in point order "
                         "(stable). At N=1 the other order is measured too and reported beside the value.")
    ap.add_argument("--no-alt-order", action="store_true",
                    help="skip measuring the other voxel_tie_order on the same inputs (N = 1)")
    ap.add_argument("--fp-mode", type=int, default=0, choices=[0, 1],
                    help="lego_params.fp_mode: libm overload model of the reference build (0 = float overloads, "
                         "GCC >= 6; 1 = double, the Indigo / Kinetic toolchains)")
    ap.add_argument("--roofline-streams", type=int, default=2048,
                    help="also time the roofline pair at this many scans per launch (0: skip)")
    ap.add_argument("--dump-poses", default="", help="rank 0: write the gathered trajectories (.npy) here")
    ap.add_argument("--config", default="c3", choices=["c3", "c5"],
                    help="headline workload: c3 = S streams per GPU (weak scaling); c5 = the 20k-scan dataset "
                         "sharded over the ranks (strong scaling)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 measurement (config c3)")
    ap.add_argument("--c5-sequences", type=int, default=80, help="C5: sequences in the dataset")
    ap.add_argument("--c5-scans", type=int, default=250, help="C5: scans per sequence")
    ap.add_argument("--dump-c5", default="", help="rank 0: write C5's gathered per-scan odometry (.npy) here")
    return ap.parse_args()


def cpu_baseline(params, cfg, pts, counts, budget_s):
    """The CPU oracle (oracle/, a restatement of the reference's path; 'port') on the SAME inputs,
    one thread, sequence by sequence, until the time budget is spent.  Scan 0 of each sequence (no
    LM) is run but not counted, matching the GPU timed region which starts after warm-up."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    nsteps, S = counts.shape
    t_sum, n_scans, n_seq = 0.0, 0, 0
    t_start = time.time()
    for s in range(S):
        orc = O.Oracle(params)
        for k in range(nsteps):
            p = pts[k, s, :counts[k, s]]
            t0 = time.perf_counter()
            orc.cloud_handler(p)
            orc.feature_association()
            dt = time.perf_counter() - t0
            if k > 0:
                t_sum += dt
                n_scans += 1
        n_seq += 1
        if time.time() - t_start > budget_s:
            break
    return {"value": round(n_scans / t_sum, 2), "unit": "scans/s", "cores": 1, "kind": "port",
            "sample": "%d sequences x %d scans (scan 0 excluded) of the benchmark's own inputs, single thread, "
                      "host %s" % (n_seq, nsteps - 1, cpu_model()),
            "ms_per_scan": round(1e3 * t_sum / max(n_scans, 1), 3)}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_baseline_threads(params, cfg, pts, counts, budget_s, threads):
    """The same oracle throughput with one sequence per host thread (SURVEY 8(d)'s all-cores variant):
    `threads` Python threads, each running whole sequences through its own oracle instance (the ctypes
    calls release the GIL), until the time budget is spent; scans of all threads / wall time."""
    import threading
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    nsteps, S = counts.shape
    lock = threading.Lock()
    state = {"next": 0, "scans": 0}
    t_start = time.time()

    def worker():
        while True:
            with lock:
                s = state["next"]
                if s >= S or time.time() - t_start > budget_s:
                    return
                state["next"] += 1
            orc = O.Oracle(params)
            n = 0
            for k in range(nsteps):
                orc.cloud_handler(pts[k, s, :counts[k, s]])
                orc.feature_association()
                n += 1
            with lock:
                state["scans"] += n
    ts = [threading.Thread(target=worker) for _ in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    wall = time.time() - t_start
    return {"value": round(state["scans"] / wall, 1), "unit": "scans/s", "cores": threads, "kind": "port",
            "sample": "%d sequences x %d scans, one sequence per thread, %d threads, host %s" % (
                state["next"], nsteps, threads, cpu_model())}


def pmc_traffic(args, S, kernels):
    """HBM bytes per launch of `kernels` from the committed rocprofv3 PMC summary of this workload
    (profiles/*_pmc.json, written by tools/pmc_summarize.py from separate FETCH_SIZE / WRITE_SIZE
    passes); None when no summary matches the workload."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc*.json"))):  # r03i_pmc.json, r03i_pmc_2048.json
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        by_base = {k.split("<")[0]: v for k, v in d.get("kernels", {}).items()}  # k_pw_scatter<4> -> k_pw_scatter
        # each entry of `kernels` names one kernel slot as "a|b": the first of its alternatives present
        pick = [next((a for a in k.split("|") if a in by_base), None) for k in kernels]
        if d.get("streams") == S and d.get("workload") == args.kind and all(pick):
            best = (f, [by_base[k] for k in pick])
    if best is None:
        return None, None
    return int(sum(v["hbm_bytes"] for v in best[1])), os.path.relpath(best[0], REPO)


def configure_batch(b, order, lag=None, wide=-1, groups=1):
    """The schedule every measured batch runs (and tests/test_gpu_bench_config.py pins against the
    oracle): `groups` stream slices, pipeline depth `lag` (None: lego_batch_set_lag's automatic choice,
    DESIGN §4), projection / segmentation layout `wide` (-1: lego_batch_set_wide's automatic choice).
    Returns the lag in effect."""
    b.set_groups(groups)
    b.set_lag(-1 if lag is None else lag)
    b.set_wide(wide)
    return b.lag()


def roofline_kernels(wide):
    """The projection + smoothness kernels the roofline pair times: k_project + k_fa_prep4 in the LDS
    layout, k_pw_scatter + k_pw_columns + k_fa_prep4 in the wide layout."""
    return ("k_pw_scatter", "k_pw_columns", "k_fa_prep4") if wide else ("k_project", "k_fa_prep4")


def roofline_at(args, L, A, mk_params, cfg, dev_index, stream):
    """The roofline pair (k_project + k_fa_prep4) at args.roofline_streams scans per launch (SURVEY §8(d):
    >= 2048 VLP-16 scans, ~2.7 GB, far above the 256 MiB Infinity Cache): a batch of that many sequences
    runs two steps (so k_fa_prep4 has its inputs), then R back-to-back pairs are timed between hipEvents,
    the projections alternating between the two steps' inputs.  Sequences 10^6 + s (not the timed
    region's)."""
    import torch
    Sb = args.roofline_streams
    params = mk_params(voxel_tie_order=args.voxel_tie_order, fp_mode=args.fp_mode)
    V, H = params.num_vertical_scans, params.num_horizontal_scans
    cap = V * H
    seqs = np.repeat(np.arange(10 ** 6, 10 ** 6 + Sb, dtype=np.int32)[None, :], 2, 0).reshape(-1)
    scans = np.repeat(np.arange(2, dtype=np.int32)[:, None], Sb, 1).reshape(-1)
    pts, cnt = A.synth_batch(cfg, seqs, scans, nthreads=args.threads)
    d_pts = torch.from_numpy(pts).to(torch.device("cuda", dev_index))
    del pts
    d_off = torch.from_numpy((np.arange(2 * Sb, dtype=np.int64) * cap).reshape(2, Sb)).to(d_pts.device)
    d_cnt = torch.from_numpy(cnt.reshape(2, Sb).astype(np.int32)).to(d_pts.device)
    b = L.Batch(params, Sb, cap, device=dev_index)
    configure_batch(b, args.voxel_tie_order, args.lag, args.wide)
    wide_b = b.wide() == 1
    for k in range(2):
        b.step(d_pts.data_ptr(), d_off[k].data_ptr(), d_cnt[k].data_ptr(), stream.cuda_stream)
    b.flush()
    torch.cuda.synchronize()
    m_sum = float(b.counts()[:, 0].astype(np.float64).sum())
    ms = b.time_hbm_stages(d_pts.data_ptr(), d_off[1].data_ptr(), d_cnt[1].data_ptr(), d_off[0].data_ptr(),
                           d_cnt[0].data_ptr(), reps=args.roofline_reps, stream=stream.cuda_stream)
    n_mean = float(cnt.reshape(2, Sb)[1].mean())
    b_tot = Sb * (16.0 * n_mean + 20.0 * cap) + 22.0 * m_sum
    b.close()
    del d_pts
    torch.cuda.empty_cache()
    achieved = b_tot / (ms * 1e-3) / 1e9
    traffic, src = pmc_traffic(args, Sb, roofline_kernels(wide_b))
    return {"streams": Sb, "kernels": "+".join(roofline_kernels(wide_b)), "bytes_per_launch": int(b_tot), "launch_ms": round(ms, 4), "achieved": round(achieved, 1),
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src,
            "note": "%d scans per launch: working set %.2f GB, above the 256 MiB Infinity Cache" % (Sb, b_tot / 1e9)}


C5_SEQ0 = 100000  # C5's sequence ids: a dataset of its own, apart from C3's 0 .. S * N - 1


def run_c5(args, L, A, mk_params, cfg, rank, world, dev_index, stream, dist, coll_dev):
    """BASELINE config C5: the synthetic dataset of --c5-sequences x --c5-scans VLP-16 scans (80 x 250 =
    20k), sequences sharded over the ranks in contiguous blocks (no collective on the data path).  Each
    rank runs its sequences as the streams of one batch, every scan of the dataset in the timed region
    (inputs resident in HBM before it; barrier + sync on both sides, max over ranks), the per-scan
    odometry recorded on the device (lego_batch_set_trajectory) and all-gathered to rank 0 afterwards,
    the path's only collective.  Returns (summary dict, gathered odometry [sequences, scans, 12] or
    None off rank 0)."""
    import torch
    n_seq, K = args.c5_sequences, args.c5_scans
    per = (n_seq + world - 1) // world  # the gather's padded shard size
    lo, hi = min(rank * per, n_seq), min((rank + 1) * per, n_seq)
    S = hi - lo
    params = mk_params(voxel_tie_order=args.voxel_tie_order, fp_mode=args.fp_mode)
    cap = params.num_vertical_scans * params.num_horizontal_scans
    dev = torch.device("cuda", dev_index)
    el, t_gen, lag, wide = 0.0, 0.0, None, None
    traj = torch.zeros((per, K, 12), dtype=torch.float32, device=dev)
    if S > 0:
        t0 = time.time()
        seqs = np.repeat(np.arange(C5_SEQ0 + lo, C5_SEQ0 + hi, dtype=np.int32)[None, :], K, 0).reshape(-1)
        scans = np.repeat(np.arange(K, dtype=np.int32)[:, None], S, 1).reshape(-1)
        pts, cnt = A.synth_batch(cfg, seqs, scans, nthreads=args.threads)
        t_gen = time.time() - t0
        d_pts = torch.from_numpy(pts).to(dev)
        del pts
        d_off = torch.from_numpy((np.arange(K * S, dtype=np.int64) * cap).reshape(K, S)).to(dev)
        d_cnt = torch.from_numpy(cnt.reshape(K, S).astype(np.int32)).to(dev)
        b = L.Batch(params, S, cap, device=dev_index)
        lag = configure_batch(b, args.voxel_tie_order, args.lag, args.wide, args.groups)
        wide = int(b.wide())
        b.set_trajectory(traj.data_ptr(), K)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if S > 0:
        for k in range(K):
            b.step(d_pts.data_ptr(), d_off[k].data_ptr(), d_cnt[k].data_ptr(), stream.cuda_stream)
        b.flush()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    status = 0
    if S > 0:
        status = int(np.bitwise_or.reduce(b.poses()[1]))
        b.close()
        del d_pts
        torch.cuda.empty_cache()
    out = traj.to(coll_dev)
    if world > 1:
        parts = [torch.empty_like(out) for _ in range(world)]
        dist.all_gather(parts, out)
        out = torch.cat(parts)
    gathered = out[:n_seq].cpu().numpy() if rank == 0 else None
    summary = {"workload": "C5: synthetic %s dataset, %d sequences x %d scans = %d scans, sharded by sequence "
                           "over %d rank(s) (%d sequences a rank), every scan timed"
                           % (args.kind.upper(), n_seq, K, n_seq * K, world, per),
               "value": round(n_seq * K / el, 1), "unit": "scans/s", "n_gpus": world, "elapsed_s": round(el, 4),
               "ms_per_step": round(1e3 * el / K, 3), "scaling": "strong", "sequences": n_seq,
               "scans_per_sequence": K, "sequences_per_rank": per, "lag": lag, "wide": wide,
               "lm_status_bits_rank0": status, "input_gen_s": round(t_gen, 2)}
    return summary, gathered


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import lego_amd as L
    from lego_amd import _abi as A

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    local_dev = local % max(ndev, 1)  # == local on a full node; lets a 1-GPU box rehearse N>1 with gloo
    torch.cuda.set_device(local_dev)  # before the process group: RCCL's barrier and collectives use this device
    if world > 1:
        dist.init_process_group(args.dist_backend)
    dev = torch.device("cuda", local_dev)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")

    mk_params = L.params_vlp16 if args.kind == "vlp16" else L.params_hdl64
    params = mk_params(voxel_tie_order=args.voxel_tie_order, fp_mode=args.fp_mode)
    cfg = A.synth_cfg(args.kind)
    V, H = params.num_vertical_scans, params.num_horizontal_scans
    cap = V * H
    S, W, K = args.streams, args.warmup, args.steps
    nsteps = W + K

    # ---- inputs: rank r owns sequences r*S .. r*S+S-1, scans 0 .. W+K-1 ----------------------------
    t0 = time.time()
    seqs = np.repeat(np.arange(rank * S, rank * S + S, dtype=np.int32)[None, :], nsteps, 0).reshape(-1)
    scans = np.repeat(np.arange(nsteps, dtype=np.int32)[:, None], S, 1).reshape(-1)
    host_pts, host_cnt = A.synth_batch(cfg, seqs, scans, nthreads=args.threads)  # [nsteps*S, cap, 4]
    host_pts = host_pts.reshape(nsteps, S, cap, 4)
    host_cnt = host_cnt.reshape(nsteps, S)
    t_gen = time.time() - t0
    d_pts = torch.from_numpy(host_pts).to(dev)
    offs = (np.arange(nsteps * S, dtype=np.int64) * cap).reshape(nsteps, S)
    d_off = torch.from_numpy(offs).to(dev)
    d_cnt = torch.from_numpy(host_cnt.astype(np.int32)).to(dev)
    batch = L.Batch(params, S, cap, device=local_dev)
    lag = configure_batch(batch, args.voxel_tie_order, args.lag, args.wide, args.groups)
    wide_pw = batch.wide() == 1  # the projection's kernels: k_pw_scatter + k_pw_columns (else k_project)
    stream = torch.cuda.current_stream(dev)

    def step(k, b=None):
        (b or batch).step(d_pts.data_ptr(), d_off[k].data_ptr(), d_cnt[k].data_ptr(), stream.cuda_stream)

    def timed(b):
        """W untimed warm-up steps, then exactly K timed steps between barrier + sync; max over ranks.
        The pipeline is drained (flush) at the end of the warm-up and inside the timed region, so the
        timed region runs exactly K scans' work per stream, the last scan's LM and publish included."""
        for k in range(W):
            step(k, b)
        b.flush()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(W, W + K):
            step(k, b)
        b.flush()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    elapsed = timed(batch)
    poses, status = batch.poses()
    # trajectory gather: the path's only collective
    traj = torch.from_numpy(poses).to(coll_dev)
    if world > 1:
        gathered = [torch.empty_like(traj) for _ in range(world)]
        dist.all_gather(gathered, traj)
        traj_all = torch.cat(gathered)
    else:
        traj_all = traj
    total_scans = S * K * world
    value = total_scans / elapsed
    alt = None
    if world == 1 and not args.no_alt_order:  # the other VoxelGrid tie order, same inputs
        alt_order = 1 - args.voxel_tie_order
        params_alt = mk_params(voxel_tie_order=alt_order, fp_mode=args.fp_mode)
        batch_alt = L.Batch(params_alt, S, cap, device=local_dev)
        configure_batch(batch_alt, alt_order, args.lag, args.wide, args.groups)
        el_alt = timed(batch_alt)
        batch_alt.close()
        alt = {"voxel_tie_order": alt_order, "value": round(total_scans / el_alt, 1),
               "ms_per_step": round(1e3 * el_alt / K, 3)}

    # ---- the roofline pair inside the pipeline: the same steps again with events around k_project and
    # k_fa_prep4 of every step (lego_batch_set_probe; not the timed pass, whose value stays event-free)
    probe = None
    if args.groups == 1 and lag >= 1:
        batch.reset()
        batch.set_probe(True)
        timed(batch)
        p_ms, f_ms, p_steps = batch.probe_times()
        batch.set_probe(False)
        probe = (p_ms, f_ms, p_steps)

    # ---- per-stage kernel times (hipEvents on the launch stream), re-running the timed steps ------
    batch.reset()
    batch.set_timing(True)
    stage = np.zeros(6)
    for k in range(W + K):
        step(k)
        if k >= W:
            stage += np.array(batch.stage_times())
        if k == W + K - 1:
            m_last = batch.counts()[:, 0].astype(np.float64)  # segmented-cloud sizes M of the last step
    stage /= K
    batch.set_timing(False)
    # the roofline pair (k_project + k_fa_prep4) launched back to back on the last step's inputs: the
    # kernels' own durations, without the per-stage event gaps (which stages_ms keeps)
    k_last = W + K - 1
    k_alt = k_last - 1 if k_last > 0 else k_last  # alternate inputs: no launch re-reads its predecessor's
    pair_ms = batch.time_hbm_stages(d_pts.data_ptr(), d_off[k_last].data_ptr(), d_cnt[k_last].data_ptr(),
                                    d_off[k_alt].data_ptr(), d_cnt[k_alt].data_ptr(),
                                    reps=args.roofline_reps, stream=stream.cuda_stream)
    voxel_ms = batch.time_voxel(reps=10, stream=stream.cuda_stream)  # the VoxelGrid stage alone
    n_mean = float(host_cnt[W:].mean())
    # Algorithmic bytes, per launch of S scans:
    #   projection  B_proj = 16 N + 20 V H  (read x,y,z,i of every point; write range + cloud cell of every cell)
    #   smoothness  B_smooth = 22 M         (read range + colInd; write curvature, picked, label, sort key/index)
    b_proj = S * (16.0 * n_mean + 20.0 * cap)
    b_smooth = 22.0 * float(m_last.sum())
    t_ms = pair_ms  # k_project + k_fa_prep4
    achieved = (b_proj + b_smooth) / (t_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(args, S, roofline_kernels(wide_pw))
    pk = "+".join(roofline_kernels(wide_pw)[:-1])  # the projection's kernel(s)
    big = roofline_at(args, L, A, mk_params, cfg, local_dev, stream) if world == 1 and args.roofline_streams > 0 else None
    roofline = {"kernel": "%s+k_fa_prep4 (projection+smoothness)" % pk, "bound": "hbm",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "bytes_per_launch": int(b_proj + b_smooth), "launch_ms": round(t_ms, 4),
                "launch_ms_source": "%d back-to-back %s + k_fa_prep4 pairs between two hipEvents on the "
                                    "launch stream (projection inputs alternating between the last two steps')"
                                    % (args.roofline_reps, pk),
                "launch_ms_stage_events": round(stage[0] + stage[2], 4),
                "frac_stage_events": round((b_proj + b_smooth) / ((stage[0] + stage[2]) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "per_kernel": {pk: {"bytes": int(b_proj), "ms": round(stage[0], 4),
                                             "GBps": round(b_proj / (stage[0] * 1e-3) / 1e9, 1)},
                               "k_fa_prep4": {"bytes": int(b_smooth), "ms": round(stage[2], 4),
                                             "GBps": round(b_smooth / (stage[2] * 1e-3) / 1e9, 1)}},
                "traffic_source": traffic_src,
                "in_pipeline": None if probe is None else {
                    "launch_ms": round(probe[0] + probe[1], 4), "project_ms": round(probe[0], 4),
                    "fa_prep_ms": round(probe[1], 4), "steps": probe[2],
                    "achieved": round((b_proj + b_smooth) / ((probe[0] + probe[1]) * 1e-3) / 1e9, 1),
                    "frac": round((b_proj + b_smooth) / ((probe[0] + probe[1]) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "source": "events around the projection and smoothness stages of every step of the "
                              "overlap schedule (the previous scan's LM on the CUs), a pass over the timed steps"},
                "note": ("%d scans per launch: working set below the 256 MiB Infinity Cache (cache-assisted)" % S
                         if b_proj + b_smooth < 256 * 2**20 else
                         "%d scans per launch: working set above the 256 MiB Infinity Cache" % S),
                "at_roofline_streams": big}

    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "scans/s", "n_gpus": world, "steps": K, "warmup": W,
        "ms_per_step": round(1e3 * elapsed / K, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "%s: batched synthetic %s sweeps, %d independent sequences per GPU x 1 scan per step"
                               % ("C3" if args.kind == "vlp16" else "C4", args.kind.upper(), S),
                   "V": V, "H": H, "points_per_scan": round(n_mean, 1), "streams_per_gpu": S,
                   "parallelism": "sequence-sharded x%d" % world, "stream_groups": args.groups, "lag": lag,
                   "voxel_tie_order": args.voxel_tie_order, "fp_mode": args.fp_mode, "wide": int(batch.wide())},
        "roofline": roofline,
        "stages_ms": {"project": round(stage[0], 4), "segment": round(stage[1], 4), "fa_prep": round(stage[2], 4),
                      "extract": round(stage[3], 4), "concat_publish": round(stage[4], 4),
                      "lm": round(stage[5], 4), "voxel_alone": round(voxel_ms, 4)},
        "other_voxel_tie_order": alt,
        "lm_status_bits": int(np.bitwise_or.reduce(status)),
        "trajectories_gathered": int(traj_all.shape[0]),
        "input_gen_s": round(t_gen, 2),
    }
    if args.config == "c5" or not args.no_c5:
        del d_pts
        torch.cuda.empty_cache()
        c5, c5_traj = run_c5(args, L, A, mk_params, cfg, rank, world, local_dev, stream, dist, coll_dev)
        if rank == 0 and args.dump_c5:
            np.save(args.dump_c5, c5_traj)
        if args.config == "c5":  # the headline is C5; C3's line moves under "c3"
            out["c3"] = {k: out[k] for k in ("value", "ms_per_step", "scaling", "config")}
            out["value"], out["ms_per_step"], out["scaling"] = c5["value"], c5["ms_per_step"], "strong"
            out["config"] = dict(out["config"], workload=c5["workload"], streams_per_gpu=c5["sequences_per_rank"],
                                 lag=c5["lag"], wide=c5["wide"])
        out["c5"] = c5
    if world == 1 and not args.no_cpu_baseline:  # N = 1 only; the reference's own VoxelGrid order (std::sort)
        params_ref = mk_params(voxel_tie_order=0, fp_mode=args.fp_mode)
        out["cpu_baseline"] = cpu_baseline(params_ref, cfg, host_pts, host_cnt, args.cpu_seconds)
        out["speedup_vs_cpu_1thread"] = round(value / out["cpu_baseline"]["value"], 1)
        if args.cpu_threads > 1:
            out["cpu_baseline_threads"] = cpu_baseline_threads(params_ref, cfg, host_pts, host_cnt, args.cpu_seconds,
                                                               args.cpu_threads)
    if rank == 0:
        if args.dump_poses:
            np.save(args.dump_poses, traj_all.cpu().numpy())
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
