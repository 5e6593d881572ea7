"""The mapping loop (lego_amd.mapping.MapSequence around the GPU operations) against the same loop
around the oracle's operations.

MapOptimization::run (mapOptmization.cpp:1521-1570, loop closure off) consumes every
mapping_frequency_divider-th AssociationOut (featureAssociation.cpp:1431-1448): transformAssociateToMap,
extractSurroundingKeyFrames, downsampleCurrentScan, scan2MapOptimization, transformUpdate and
saveKeyFramesAndFactor.  Here several sequences run through it in lock step, batched on the GPU
(mapping_step_gpu) and one by one on the oracle; the per-cycle optimised pose must agree within
1e-4 and the key-frame bookkeeping must be identical.
"""
import numpy as np
import pytest

import oracle as O
from lego_amd import _abi as A
from lego_amd import mapping as M

pytestmark = pytest.mark.gpu

LEGO_ST_EMITTED = 0x080


def _emitted(seq, n_scans):
    import lego_amd as LA
    orc = O.Oracle(LA.params_vlp16())
    cfg = A.synth_cfg("vlp16")
    out = []
    for k in range(n_scans):
        orc.cloud_handler(A.synth_scan(cfg, seq, k))
        a = orc.feature_association()
        if a["status"] & LEGO_ST_EMITTED:
            out.append(a)
    return out


def mapping_step_oracle(seqs, assocs, voxel_tie_order=0):
    """One mapping cycle around the oracle's operations; VoxelGrid in the given tie order (0: PCL's
    std::sort permutation, the reference's; 1: std::stable_sort's)."""
    res = []
    for sq, a in zip(seqs, assocs):
        cparts, sparts, (c, s, o), t0 = sq.begin(a)
        vg = lambda x, leaf: O.voxel_grid(x, leaf, stable=voxel_tie_order == 1)[0]  # noqa: E731
        cat = lambda xs: np.concatenate(xs) if xs else np.zeros((0, 4), np.float32)  # noqa: E731
        cm = vg(cat([O.transform_cloud(x, t) for x, t in cparts]), 0.2)
        sm = vg(cat([O.transform_cloud(x, t) for x, t in sparts]), 0.4)
        cds, sds, ods = vg(c, 0.2), vg(s, 0.4), vg(o, 0.4)
        surf = vg(np.concatenate([sds, ods]), 0.4)
        t, dg, info = O.scan2map(cds, surf, cm, sm, t0, sq.degenerate)
        sq.end(t, dg, info, (cds, sds, ods))
        res.append((t, dg, info))
    return res


@pytest.mark.parametrize("order", [0, 1])
def test_mapping_loop_matches_oracle(gpu, order):
    import lego_amd as LA
    streams = [_emitted(seq, 31) for seq in (3, 6, 8)]
    n = min(len(s) for s in streams)
    assert n >= 5
    s2m = LA.ScanToMap(max_problems=len(streams), max_map_points=150000, device=gpu)
    s2m.set_voxel_tie_order(order)
    g = [M.MapSequence() for _ in streams]
    r = [M.MapSequence(associate=O.associate_to_map, odometry=O.odometry_to_transform) for _ in streams]
    ran = 0
    for k in range(n):
        out_g = M.mapping_step_gpu(s2m, g, [s[k] for s in streams])
        out_r = mapping_step_oracle(r, [s[k] for s in streams], order)
        for p, ((tg, dgg, ig), (tr, dgr, ir)) in enumerate(zip(out_g, out_r)):
            assert np.abs(tg - tr).max() <= 1e-4, (k, p, tg, tr)
            assert dgg == dgr and ig[0] == ir[0] and ig[1] == ir[1], (k, p, ig, ir)
            ran += int(ig[0] == 1)
        for a, b in zip(g, r):
            assert a.existing == b.existing and len(a.key_pos) == len(b.key_pos)
            assert np.abs(a.t_aft - b.t_aft).max() <= 1e-4
    s2m.close()
    assert ran >= (n - 1) * len(streams)  # every cycle after the first has a map
    assert all(len(sq.key_pos) >= 3 for sq in g)
