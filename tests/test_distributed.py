"""World-size-2 gloo rehearsal of bench.py's multi-GPU path on the CPU.

bench.py shards FRAMES across ranks (weak scaling): each rank owns
its own frames, builds and runs them with no data-path collective, and only the timing
(max over ranks) and the frame count (sum over ranks) are reduced.  These tests run the
same helpers under two gloo processes and check (1) the shards are disjoint and cover
the single-process frame set, (2) the reductions are the max / sum, and (3) the per-rank
graphs (oracle restatement, CPU) concatenate to the single-process result, i.e. the
sharding needs no exchange step.  On a GPU box, test_frame_sharding_two_ranks_hip_pipeline
runs the same sharding with the product HIP pipeline on every rank.
"""
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


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, frames, nodes, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank), RG_BENCH_BACKEND='gloo')
    import bench
    from graph_neural_network_for_radar_perception_amd import synthetic
    from oracle import graph_features_ref as gref
    w, r, _ = bench.setup_dist()
    assert (w, r) == (world, rank)
    seeds = bench.rank_frame_seeds(rank, frames, synthetic.SEED0)
    n_edges = []
    for s in seeds:
        fr = synthetic.make_frame(nodes, s)
        adj = gref.compute_adjacency_information(fr, 25.0, 8)
        n_edges.append(adj['adj_list'].shape[1])
    bench.barrier(w)
    t_max = bench.max_over_ranks(float(rank + 1), w)
    total = bench.sum_over_ranks(float(len(seeds)), w)
    np.savez(os.path.join(out_dir, f'rank{rank}.npz'), seeds=np.array(seeds),
             n_edges=np.array(n_edges), t_max=t_max, total=total)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_frame_sharding_two_ranks_gloo(tmp_path):
    world, frames, nodes = 2, 3, 120
    mp.spawn(_worker, args=(world, _free_port(), frames, nodes, str(tmp_path)), nprocs=world,
             join=True)
    from graph_neural_network_for_radar_perception_amd import synthetic
    from oracle import graph_features_ref as gref
    res = [np.load(tmp_path / f'rank{r}.npz') for r in range(world)]
    seeds = np.concatenate([x['seeds'] for x in res])
    assert len(set(seeds.tolist())) == world * frames            # disjoint shards
    for x in res:
        assert float(x['t_max']) == float(world)                 # max over ranks
        assert float(x['total']) == float(world * frames)        # whole-job frame count
    # single process over the union of the shards == concatenation of the ranks' work
    want = []
    for s in seeds:
        adj = gref.compute_adjacency_information(synthetic.make_frame(nodes, int(s)), 25.0, 8)
        want.append(adj['adj_list'].shape[1])
    np.testing.assert_array_equal(np.concatenate([x['n_edges'] for x in res]), want)


def test_rank_seeds_weak_scaling():
    import bench
    a = bench.rank_frame_seeds(0, 64, 7)
    b = bench.rank_frame_seeds(1, 64, 7)
    assert len(a) == len(b) == 64 and not set(a) & set(b)
    assert bench.rank_frame_seeds(0, 64, 7) == a                 # deterministic per rank


def _ddp_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    dist.init_process_group('gloo')
    from graph_neural_network_for_radar_perception_amd.training import (allreduce_gradients,
                                                                          broadcast_parameters)
    g = torch.arange(10, dtype=torch.float32) * (rank + 1)
    scale = allreduce_gradients(g, world)
    p = torch.full((4,), float(rank))
    broadcast_parameters(p, world)
    np.savez(os.path.join(out_dir, f'ddp{rank}.npz'), g=g.numpy(), scale=scale, p=p.numpy())
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gradient_allreduce_two_ranks_gloo(tmp_path):
    """BASELINE config 4's data-parallel sync (training.allreduce_gradients /
    broadcast_parameters): one flat bucket summed over ranks, averaged by the SGD step's
    grad_scale = 1/world; every rank starts from rank 0's weights."""
    world = 2
    mp.spawn(_ddp_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = np.arange(10, dtype=np.float32) * 3
    for r in range(world):
        d = np.load(tmp_path / f'ddp{r}.npz')
        np.testing.assert_array_equal(d['g'], want)
        assert float(d['scale']) == 0.5
        np.testing.assert_array_equal(d['p'], np.zeros(4, np.float32))


def _hip_worker(rank, world, port, frames, nodes, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank), RG_BENCH_BACKEND='gloo')
    import bench
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.graph_features import FrameBatch
    from graph_neural_network_for_radar_perception_amd.pipeline import RadarGNNPipeline
    w, r, _ = bench.setup_dist()           # one process per "GPU" (both share cuda:0 here)
    dev = torch.device('cuda', torch.cuda.current_device())
    cfg = default_config()
    model = bench.make_model(cfg, dev, bench.model_state(cfg, 'trained'))
    seeds = bench.rank_frame_seeds(rank, frames, synthetic.SEED0)
    fr = [synthetic.make_frame(nodes, s) for s in seeds]
    cl = [synthetic.cluster_lists(nodes) for _ in seeds]
    batch = FrameBatch.from_frames(fr, cl, device=dev)
    with torch.no_grad():
        gb, out = RadarGNNPipeline(model, cfg, 'fp32').step(batch)
    torch.cuda.synchronize()
    bench.barrier(w)
    total = bench.sum_over_ranks(float(len(seeds)), w)
    np.savez(os.path.join(out_dir, f'hip{rank}.npz'), seeds=np.array(seeds),
             node_cls=out.node_cls.cpu().numpy(), node_reg=out.node_reg.cpu().numpy(),
             n_edges=int(gb.n_edges_dev.item()), total=total)
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_frame_sharding_two_ranks_hip_pipeline(tmp_path, cuda_device):
    """bench.py's multi-rank path with the PRODUCT pipeline on every rank: two processes
    (gloo for the bookkeeping collectives, both on the one card of the test box), each
    building and running its own frames through the HIP graph build + fp32 forward.  The
    ranks' outputs, concatenated, equal one process running all frames: frame sharding
    needs no data-path exchange, and the batched union is exact per frame."""
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.graph_features import FrameBatch
    from graph_neural_network_for_radar_perception_amd.pipeline import RadarGNNPipeline
    import bench
    world, frames, nodes = 2, 3, 700
    mp.spawn(_hip_worker, args=(world, _free_port(), frames, nodes, str(tmp_path)),
             nprocs=world, join=True)
    res = [np.load(tmp_path / f'hip{r}.npz') for r in range(world)]
    seeds = np.concatenate([x['seeds'] for x in res])
    assert len(set(seeds.tolist())) == world * frames
    assert all(float(x['total']) == world * frames for x in res)
    dev = cuda_device
    cfg = default_config()
    model = bench.make_model(cfg, dev, bench.model_state(cfg, 'trained'))
    fr = [synthetic.make_frame(nodes, int(s)) for s in seeds]
    cl = [synthetic.cluster_lists(nodes) for _ in seeds]
    with torch.no_grad():
        gb, out = RadarGNNPipeline(model, cfg, 'fp32').step(FrameBatch.from_frames(fr, cl, device=dev))
    assert int(gb.n_edges_dev.item()) == sum(int(x['n_edges']) for x in res)
    np.testing.assert_array_equal(np.concatenate([x['node_cls'] for x in res]),
                                  out.node_cls.cpu().numpy())
    np.testing.assert_array_equal(np.concatenate([x['node_reg'] for x in res]),
                                  out.node_reg.cpu().numpy())


def _run_bench(args, timeout=240):
    import json
    import subprocess
    env = dict(os.environ, RG_BENCH_BACKEND='gloo')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py')] + args, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout       # rank 0 alone prints the line
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_gpus2_launches_two_ranks(cuda_device):
    """`python bench.py --gpus 2` (no launcher in the environment) starts two ranks itself:
    the line reports n_gpus 2 and the value counts both ranks' frames (weak scaling; gloo
    for the timing collectives so both ranks can share the test box's one card), and rank 0
    adds the CPU baseline after the timed region while the other rank waits."""
    line = _run_bench(['--gpus', '2', '--steps', '2', '--warmup', '1', '--frames', '4',
                       '--nodes', '1000', '--cpu-frames', '1', '--no-extra'])
    assert line['n_gpus'] == 2
    # multi-rank lines carry the CPU baseline too (rank 0, after the timed region)
    cb = line['cpu_baseline']
    assert cb['kind'] == 'port' and cb['value'] > 0 and cb['cores'] >= 1
    assert cb['forward_1thread_ms'] > 0 and 'median of 5 frames' in cb['sample']
    assert line['config']['frames_per_rank_timed'] == [8, 8]
    assert line['config']['backend'] == 'gloo'
    # value = frames of all ranks / max-over-ranks elapsed = 16 / (steps * ms_per_step)
    assert abs(line['value'] - 16.0 / (2 * line['ms_per_step'] * 1e-3)) <= 0.01 * line['value']


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_c3_eight_ranks_512_frames(tmp_path, cuda_device):
    """BASELINE config 3's workload through the product path: `bench.py --config c3 --gpus 8`
    = 8 ranks x 64 frames of C2's shape (3000 nodes, k = 32, L = 6, bf16) = 512 frames per
    step, frame-parallel with no collective in the step (the reference loops its frames
    independently, gnn_detector.py:443-452).  The 8 ranks share the test box's one card
    (gloo for the bookkeeping collectives); the driver's 8-GPU node runs the same launcher
    with one card per rank over RCCL.  Each rank saves the outputs of 2 of its frames
    (--save-outputs); they are checked here against the oracle at the bf16 bound."""
    from graph_neural_network_for_radar_perception_amd import synthetic
    from graph_neural_network_for_radar_perception_amd.config import default_config
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    from oracle import gnn_forward_ref, graph_features_ref as gref
    from test_gpu_parity import GRID_MAX_R, argmax_flips, assert_bf16_close
    import bench
    world = 8
    line = _run_bench(['--config', 'c3', '--gpus', str(world), '--steps', '2', '--warmup', '1',
                       '--cpu-frames', '1', '--save-outputs', str(tmp_path), '--save-frames', '2'],
                      timeout=800)
    assert line['n_gpus'] == world
    assert line['config']['frames_per_rank_timed'] == [128] * world    # 64 frames x 2 steps
    assert line['config']['frames_per_gpu'] == 64 and line['config']['layers'] == 6
    assert '512 frames frame-parallel over 8 GPU(s)' in line['config']['workload']
    assert abs(line['value'] - 1024.0 / (2 * line['ms_per_step'] * 1e-3)) <= 0.01 * line['value']
    cb = line['cpu_baseline']
    assert cb['kind'] == 'port' and cb['value'] > 0
    # every rank's saved frames against the oracle (the bench's own seeded random init)
    cfg = default_config(graph_convolution_stem_channels=[64] * 6, k_number_nearest_points=32)
    sd = bench.model_state(cfg, 'random')
    m = Model_Training(cfg, 'cpu')
    m.load_state_dict(sd, strict=True)
    pred = m.pred.eval()
    keys = ('node_cls', 'node_reg', 'link_cls', 'obj_cls')
    seen = set()
    for r in range(world):
        d = np.load(tmp_path / f'rank{r}.npz')
        seeds = [int(s) for s in d['seeds']]
        assert seeds == bench.rank_frame_seeds(r, 64, synthetic.SEED0)[:2]
        seen.update(seeds)
        N = int(d['nodes'])
        clusters = synthetic.cluster_lists(N)
        ncl = len(clusters)
        for f, s in enumerate(seeds):
            g = gref.build_frame_graph(synthetic.make_frame(N, s), 25.0, 32, GRID_MAX_R)
            with torch.no_grad():
                ref = gnn_forward_ref.forward(sd, cfg, torch.from_numpy(g['node_features']),
                                              torch.from_numpy(g['edge_features']),
                                              torch.from_numpy(g['edge_index']), None,
                                              [torch.from_numpy(c) for c in clusters])
            sel = (d['pair_src'] >= f * N) & (d['pair_src'] < (f + 1) * N)
            got = (d['node_cls'][f * N:(f + 1) * N], d['node_reg'][f * N:(f + 1) * N],
                   d['link_cls'][sel], d['obj_cls'][f * ncl:(f + 1) * ncl])
            for key, gt, rf in zip(keys, got, ref):
                assert gt.shape == tuple(rf.shape), (r, f, key)
                worst, _ = assert_bf16_close(pred, key, gt, rf.numpy(), min_agree=None)
                if key != 'node_reg':
                    fl, tie = argmax_flips(gt, rf.numpy())
                    assert not (fl & ~tie).any(), (r, f, key)
                print(f'rank {r} frame {f} {key}: worst {worst:.3f} of the bf16 bound')
    assert len(seen) == 2 * world     # disjoint shards


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_c4_gpus2_allreduce_path(cuda_device):
    """`bench.py --config c4 --gpus 2`: data-parallel training through the launcher path,
    the flat-gradient all-reduce (training.allreduce_gradients) on every step."""
    line = _run_bench(['--config', 'c4', '--gpus', '2', '--steps', '2', '--warmup', '1',
                       '--frames', '2', '--nodes', '500', '--no-cpu-baseline'])
    assert line['n_gpus'] == 2
    assert line['config']['frames_per_rank_timed'] == [4, 4]
    assert all(np.isfinite(line['last_losses']))


def _world_check_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank), RG_BENCH_BACKEND='gloo')
    import bench
    try:
        bench.setup_dist(world + 1)
        ok = False
    except SystemExit:
        ok = True
    w, r, _ = bench.setup_dist(world)
    counts = bench.per_rank_counts(10 * (rank + 1), w)
    np.savez(os.path.join(out_dir, f'wc{rank}.npz'), ok=ok, counts=np.array(counts))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_setup_dist_checks_world_and_gathers_counts(tmp_path):
    """--gpus N under a launcher that started a different number of ranks is refused; the
    per-rank frame counts of the line are gathered in rank order."""
    world = 2
    mp.spawn(_world_check_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
             join=True)
    for r in range(world):
        d = np.load(tmp_path / f'wc{r}.npz')
        assert bool(d['ok'])
        np.testing.assert_array_equal(d['counts'], [10, 20])


_RCCL_PROBE = r'''
import os, sys, json
import torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from graph_neural_network_for_radar_perception_amd import training
torch.cuda.set_device(0)
dist.init_process_group('nccl', world_size=1, rank=0)
assert dist.get_backend() == 'nccl'
# the training step's one flat-gradient bucket (training.allreduce_gradients) and the
# construction-time broadcast, on device tensors through RCCL
flat = torch.linspace(-1.0, 1.0, 463144, device='cuda')
ref = flat.clone()
dist.all_reduce(flat, op=dist.ReduceOp.SUM)
training.broadcast_parameters(flat, 1)
dist.broadcast(flat, 0)
# bench.py's timing reductions (max / sum over ranks of a device scalar) and its barrier
t = torch.tensor([3.5], dtype=torch.float64, device='cuda')
dist.all_reduce(t, op=dist.ReduceOp.MAX)
dist.barrier()
torch.cuda.synchronize()
print(json.dumps({'equal': bool(torch.equal(flat, ref)), 'max': float(t.item()),
                  'rccl': torch.cuda.nccl.version() if hasattr(torch.cuda, 'nccl') else None}))
dist.destroy_process_group()
'''


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_rccl_collectives_on_device(cuda_device):
    """The RCCL ('nccl' backend) branch of the multi-GPU path on the hardware: a one-rank
    process group initialises on the MI355X and the collectives the data path uses -- the
    flat-gradient all-reduce of training.allreduce_gradients, the parameter broadcast, the
    bench's max-over-ranks and barrier -- run on device tensors (sum / max over one rank is
    the identity).  Multi-rank RCCL needs one card per rank (the driver's 8-GPU run)."""
    import json
    import subprocess
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()),
               WORLD_SIZE='1', RANK='0', LOCAL_RANK='0')
    r = subprocess.run([sys.executable, '-c', _RCCL_PROBE, REPO], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{')][-1])
    assert out['equal'] and out['max'] == 3.5, out
