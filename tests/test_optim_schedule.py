"""CPU checks of the optimizer's host logic (training.multistep_lr_table, the gradient
bucket's loss slots under a world-size-2 gloo all-reduce).  The device kernels are checked
against torch.optim in tests/test_gpu_optim.py.

Reference: set_param_for_training_gnn.py:51-56 (MultiStepLR), training.py:40-45, 79-85
(skip_batch on a NaN total loss)."""
import bisect
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


@pytest.mark.parametrize('milestones', [[3, 7], [0, 2], [-1, 2], [2, 2, 5], [3, 3], [], [0],
                                        [int(0.5 * 200000 - 150000), int(0.8 * 200000 - 150000)]])
def test_multistep_lr_table_equals_torch_scheduler(milestones):
    from graph_neural_network_for_radar_perception_amd.training import multistep_lr_table
    base = 0.005
    ms, lrs = multistep_lr_table(base, milestones, 0.1)
    p = torch.nn.Parameter(torch.zeros(1))
    o = torch.optim.SGD([p], lr=base, momentum=0.9)
    s = torch.optim.lr_scheduler.MultiStepLR(o, milestones=milestones, gamma=0.1)
    for k in range(12 + max([m for m in milestones if m < 100] or [0])):
        assert lrs[bisect.bisect_right(ms, k)] == o.param_groups[0]['lr'], (milestones, k)
        o.step()
        s.step()


def test_reference_milestones_formula():
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.training import reference_milestones
    cfg = default_config()
    assert reference_milestones(cfg) == [100000, 160000]                # yml: 200 000 iterations
    assert reference_milestones(cfg, 120000) == [-20000, 40000]         # resumed past the first


def test_too_many_milestones_refused():
    from graph_neural_network_for_radar_perception_amd.training import multistep_lr_table
    with pytest.raises(ValueError):
        multistep_lr_table(0.1, list(range(17)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _bucket_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    dist.init_process_group('gloo')
    from graph_neural_network_for_radar_perception_amd.training import (N_LOSS_SLOTS,
                                                                          allreduce_gradients)
    n = 10
    bucket = torch.zeros(n + N_LOSS_SLOTS)
    bucket[:n] = torch.arange(n, dtype=torch.float32) * (rank + 1)
    losses = torch.tensor([0.5, 0.25, 0.125, 1.0]) * (rank + 1)
    if rank == 1:
        losses[2] = float('nan')            # rank 1's corrupted batch
    bucket[n:] = losses
    scale = allreduce_gradients(bucket, world)
    np.savez(os.path.join(out_dir, f'b{rank}.npz'), bucket=bucket.numpy(), scale=scale)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_loss_slots_carry_nan_to_every_rank_gloo(tmp_path):
    """The trainer's one all-reduce bucket = gradients then the four losses
    (TrainEngine.flat_bucket): after the reduction every rank holds the same summed losses,
    NaN where any rank's was -- the input rg_sgd_step_sched's skip test reads, so all ranks
    decide alike; the gradients are summed as before."""
    world = 2
    mp.spawn(_bucket_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    b = [np.load(tmp_path / f'b{r}.npz') for r in range(world)]
    np.testing.assert_array_equal(b[0]['bucket'], b[1]['bucket'])
    np.testing.assert_array_equal(b[0]['bucket'][:10], np.arange(10, dtype=np.float32) * 3)
    slots = b[0]['bucket'][10:]
    assert np.isnan(slots[2]) and np.isfinite(slots[[0, 1, 3]]).all()
    total = np.float32(slots[0]) + np.float32(slots[1]) + np.float32(slots[2]) + np.float32(slots[3])
    assert np.isnan(total)
    assert float(b[0]['scale']) == 0.5
