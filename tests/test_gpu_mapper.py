"""The native mapping thread (lego_mapper_*, Mapper) against MapSequence around the oracle's operations.

lego_mapper_step is MapOptimization::run's loop body (mapOptmization.cpp:1521-1570, loop closure off)
with the host logic in C++ and the key frames' clouds in device memory; MapSequence +
mapping_step_oracle is the same loop in Python over the CPU restatements.  Bar: north_star's 1e-4 on
transformAftMapped; measured bit-identical (the device's sinf / cosf restate the host glibc's and the
normal equations are summed in the oracle's order), so the test asserts identical bits every cycle,
identical LM gate / iteration / correspondence counts and identical key poses.
"""
import numpy as np
import pytest

import oracle as O
from lego_amd import mapping as M
from test_gpu_mapping_loop import _emitted, mapping_step_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seq,max_map,max_key,order", [(3, 150000, 4_000_000, 0), (8, 150000, 4_000_000, 0),
                                                        (3, 1500, 2000, 0), (3, 150000, 4_000_000, 1),
                                                        (8, 150000, 4_000_000, 1)])
def test_mapper_matches_oracle_loop(gpu, seq, max_map, max_key, order):
    """Both VoxelGrid tie orders (0: PCL's std::sort permutation, the reference's; 1: stable), each
    against the oracle's VoxelGrid in the same order.  (3, 1500, 2000): initial capacities far below the
    sequence's raw map, scan clouds and key-frame store, so every buffer of the mapper grows on demand
    (the reference has no such limits) and the results stay identical."""
    import lego_amd as LA
    stream = _emitted(seq, 61)
    assert len(stream) >= 5
    mp = LA.Mapper(max_map_points=max_map, max_key_points=max_key, device=gpu, voxel_tie_order=order)
    r = M.MapSequence(associate=O.associate_to_map, odometry=O.odometry_to_transform)
    ran = 0
    for k, a in enumerate(stream):
        tg, ig = mp.step(a["corner_last"], a["surf_last"], a["outlier_last"],
                             M.odometry_to_transform(a["odom_orientation"], a["odom_position"]))
        (_, _, ir), = mapping_step_oracle([r], [a], order)
        assert np.array_equal(tg.view(np.int32), r.t_aft.view(np.int32)), (k, tg, r.t_aft)
        assert np.array_equal(ig, ir), (k, ig, ir)
        ran += int(ig[0] == 1)
    kp = mp.key_poses()
    assert kp.shape == (len(r.key_pose6), 6)
    assert np.array_equal(kp.view(np.int32), np.array(r.key_pose6, np.float32).view(np.int32))
    mp.close()
    assert ran >= len(stream) - 1
    assert len(kp) >= 3


def test_mapper_rejects_bad_args(gpu):
    import lego_amd as LA
    with pytest.raises(LA.LegoError):
        LA.Mapper(max_map_points=0, device=gpu)
    with pytest.raises(LA.LegoError):
        LA.Mapper(max_map_points=1000, max_key_points=0, device=gpu)
    mp = LA.Mapper(max_map_points=1000, max_key_points=10000, device=gpu)
    assert mp.key_poses().shape == (0, 6)
    mp.close()
