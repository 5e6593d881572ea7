"""Measure the scan-to-map LM (include/lego_s2m.h): problems/s on one GPU vs the CPU oracle.

Problems come from the product path itself: S synthetic VLP-16 sequences run through lego_amd.Batch
(lag 0) for K scans; the AssociationOut records of each sequence (corner / surf / outlier Last
clouds, transformSum) build its scan-to-map problem for scan K-1 (lego_amd.mapping.build_problem:
the previous up-to-10 scans as the surrounding map, the reference's VoxelGrid leaves).  All S
problems run in one lego_s2m_run launch; the timed region is R launches on device-resident inputs,
bracketed by hipEvents on the launch stream.  The CPU baseline runs the oracle (oracle/s2m_oracle.cpp,
single thread) on a sample of the same problems, which also gives the parity figure.  The map-side
preparation (lego_map_transform / lego_map_voxel through lego_amd.mapping.prepare_gpu) is timed too.

  python tools/bench_s2m.py [--streams 256] [--scans 8] [--reps 20] [--cpu-sample 16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "lego-loam-bor_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--scans", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=16)
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import torch
    import lego_amd as LA
    from lego_amd import _abi as A
    from lego_amd import mapping as M
    from test_gpu_s2m import _device_io

    S, K = args.streams, args.scans
    p = LA.params_vlp16()
    cfg = A.synth_cfg("vlp16")
    t0 = time.time()
    cap = 40000
    pts = np.zeros((K, S, cap, 4), np.float32)
    cnt = np.zeros((K, S), np.int32)
    for k in range(K):
        for s in range(S):
            x = A.synth_scan(cfg, 100 + s, k)
            pts[k, s, :len(x)] = x
            cnt[k, s] = len(x)
    b = LA.Batch(p, S, cap)
    b.set_lag(0)
    d_pts = torch.from_numpy(pts.reshape(K, S * cap, 4)).cuda()
    offs = torch.from_numpy((np.arange(S, dtype=np.int64) * cap)).cuda()
    frames = [[] for _ in range(S)]
    for k in range(K):
        d_cnt = torch.from_numpy(cnt[k]).cuda()
        b.step(d_pts[k].data_ptr(), offs.data_ptr(), d_cnt.data_ptr(), torch.cuda.current_stream().cuda_stream)
        b.sync()
        for s in range(S):
            frames[s].append(b.read(s)[1])
    b.close()
    problems = [M.build_problem(frames[s], K - 1) for s in range(S)]
    t_gen = time.time() - t0
    sizes = {n: float(np.mean([len(pr[n]) for pr in problems])) for n in ("corner", "surf", "corner_map", "surf_map")}
    max_map = max(max(len(pr["corner_map"]), len(pr["surf_map"]), len(pr["corner"]) + len(pr["surf"])) for pr in problems)

    m = LA.ScanToMap(max_problems=S, max_map_points=max_map, device=0)
    io, keep, tr, dg, info = _device_io(problems, torch)
    tr0 = tr.clone()
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        tr.copy_(tr0)
        m.run(S, io, stream.cuda_stream)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    total = 0.0
    for _ in range(args.reps):
        tr.copy_(tr0)  # every launch solves the same problems from their initial guesses
        dg.zero_()
        ev0.record(stream)
        m.run(S, io, stream.cuda_stream)
        ev1.record(stream)
        ev1.synchronize()
        total += ev0.elapsed_time(ev1)
    ms = total / args.reps
    t_gpu, dg_gpu, info_gpu = tr.cpu().numpy(), dg.cpu().numpy(), info.cpu().numpy()

    # map-side preparation on the GPU (lego_map_transform + lego_map_voxel, mapping.prepare_gpu): the
    # same problems assembled from the sequences' records, timed end to end (host uploads of the key
    # frames, the kernels, one read of the VoxelGrid counts)
    m.close()
    m = LA.ScanToMap(max_problems=S, max_map_points=max(max_map, 8 * 12000 + 4000), device=0)
    seqs = [frames[s] for s in range(S)]
    M.prepare_gpu(m, seqs, K - 1)  # warm-up (allocates the VoxelGrid scratch)
    torch.cuda.synchronize()
    prep, prep_dev_ms = [], []
    for _ in range(3):
        t1 = time.time()
        evs = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        pio, pkeep, ptr, pdg, pinfo, _v = M.prepare_gpu(m, seqs, K - 1, events=evs)
        torch.cuda.synchronize()
        prep.append(time.time() - t1)
        prep_dev_ms.append(evs[0].elapsed_time(evs[1]))
    prep_ms = 1e3 * min(prep)
    prep_d = min(prep_dev_ms)
    m.run(S, pio, stream.cuda_stream)
    torch.cuda.synchronize()
    prep_dev = float(np.abs(ptr.cpu().numpy() - t_gpu).max())  # GPU-prepared (stable VoxelGrid) vs numpy-prepared
    m.close()

    # CPU oracle on a sample of the same problems (single thread): baseline and parity
    import oracle as O
    n_cpu = min(args.cpu_sample, S)
    dev = []
    t1 = time.time()
    for i in range(n_cpu):
        pr = problems[i]
        t_ref, _, info_ref = O.scan2map(pr["corner"], pr["surf"], pr["corner_map"], pr["surf_map"], pr["transform"])
        dev.append(float(np.abs(t_ref - t_gpu[i]).max()))
    cpu_s = (time.time() - t1) / n_cpu
    # the map-side preparation on the CPU: the oracle's transformPointCloud + VoxelGrid (stable order)
    t1 = time.time()
    for i in range(n_cpu):
        cparts, sparts, (c, s_, o) = M._parts(frames[i], K - 1, 10)
        vg = lambda x, leaf: O.voxel_grid(x, leaf, stable=True)[0]  # noqa: E731
        vg(np.concatenate([O.transform_cloud(x, t) for x, t in cparts]), 0.2)
        vg(np.concatenate([O.transform_cloud(x, t) for x, t in sparts]), 0.4)
        vg(c, 0.2)
        vg(np.concatenate([vg(s_, 0.4), vg(o, 0.4)]), 0.4)
    cpu_prep_s = (time.time() - t1) / n_cpu
    out = {
        "metric": "scan-to-map problems/s (MapOptimization::scan2MapOptimization, <= 10 LM iterations each)",
        "value": round(S / (ms * 1e-3), 1), "unit": "problems/s", "n_gpus": 1, "ms_per_launch": round(ms, 4),
        "problems_per_launch": S, "reps": args.reps, "dtype": "f32 (normal equations f64)",
        "data": "synthetic VLP-16 sequences through lego_amd.Batch; maps of the previous <= 10 scans",
        "mean_sizes": sizes, "iterations_mean": float(info_gpu[:, 1].mean()),
        "correspondences_mean": float(info_gpu[:, 2].mean()),
        "status_or": int(np.bitwise_or.reduce(info_gpu[:, 3])), "degenerate": int(dg_gpu.sum()),
        "cpu_baseline": {"value": round(1.0 / cpu_s, 1), "unit": "problems/s", "cores": 1, "kind": "port",
                         "sample": "%d of the same problems, oracle/s2m_oracle.cpp (grid kNN-5), single thread" % n_cpu},
        "parity": {"max_abs_transform_diff": max(dev), "tolerance": 1e-4, "sample": n_cpu},
        "input_gen_s": round(t_gen, 1),
        "map_prep": {"device_ms": round(prep_d, 3), "problems_per_s": round(S / (prep_d * 1e-3), 1),
                     "end_to_end_ms": round(prep_ms, 3),
                     "note": "lego_map_transform + lego_map_voxel for all problems (two of each, one count read in "
                             "between), hipEvents around the device work; end_to_end adds the Python assembly and "
                             "host upload of the key frames (mapping.prepare_gpu)",
                     "max_abs_transform_diff_vs_numpy_prepared": prep_dev,
                     "cpu_baseline": {"value": round(1.0 / cpu_prep_s, 1), "unit": "problems/s", "cores": 1,
                                      "kind": "port", "sample": "the same %d problems: oracle transform_cloud + "
                                      "voxel_grid (stable), single thread" % n_cpu}},
    }
    line = json.dumps(out)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
