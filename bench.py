"""Benchmark: radar frames/s of the MI355X-native hot path (BASELINE.json metric).

One step = one batch of synthetic RadarScenes-shaped frames, raw measurements
already resident in HBM, through the whole hot path: kNN graph build + ball
query, node / edge input features, node and edge encoders, L message-passing
layers, the four task heads (graph_features.py:58-164 + gnn_detector.py:141-201).

Default workload = the metric's own configuration **M** (SURVEY.md §8(d)): 64 frames
x 3000 nodes per GPU, the yml graph (k = 10, eps^2 = 25 -> E ~ 37.8k edges per frame),
L = 7, **fp32** compute (the reference precision; parity 1e-4), the trained
checkpoint's weights (`1718175257362`, committed as the `w/*` arrays of
tests/golden/model_trained_N50.npz -- nothing is read from the reference at run time).
The same run also times BASELINE config 2 (64 x 3000, k = 32, L = 6, bf16) as the extra
key ``c2_bf16``.
Multi-GPU (torchrun, one process per GPU): every rank owns its own 64 frames
(frame-parallel, weak scaling, no collective in the timed region; barrier +
max-over-ranks timing only).

``--config c5``: BASELINE config 5 (dense-scene stress): one frame of 20,000 nodes per GPU,
pure radius graph (compute_ball_query semantics, eps^2 = 2.5 -> E ~ 400k), L = 7, fp16
operands (v_mfma_f32_32x32x16_f16, f32 accumulation) as the config names.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from graph_neural_network_for_radar_perception_amd import synthetic  # noqa: E402
from graph_neural_network_for_radar_perception_amd.config import default_config  # noqa: E402

METRIC = json.load(open(os.path.join(REPO, 'BASELINE.json')))['metric']
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MFMA_PEAK_TFLOPS = {'bf16': 2500.0, 'fp16': 2500.0, 'fp32': 157.3}   # dense MFMA peaks (same doc)


# workloads; k is unused by the pure radius graph
PRESETS = {
    # the metric's configuration (BASELINE.json metric "N~3k nodes, E~30k edges"; yml k = 10,
    # L = 7, configuration_radarscenes_gnn.yml:14,58), fp32, trained weights, two batches in
    # flight (the next step's graph build beside this forward: +2.9 %)
    'm': dict(frames=64, nodes=3000, k=10, layers=7, graph='knn', eps2=25.0, cpu_frames=5,
              cpu_warm=2, dtype='fp32', weights='trained', streams=2),
    'c2': dict(frames=64, nodes=3000, k=32, layers=6, graph='knn', eps2=25.0, cpu_frames=5,
               cpu_warm=2, dtype='bf16', weights='random', streams=2),
    # BASELINE config 3: 512 frames of C2's shape frame-parallel over 8 GPUs, forward only --
    # 64 frames per rank (weak scaling: --gpus 8 processes 512), no collective in the step
    'c3': dict(frames=64, nodes=3000, k=32, layers=6, graph='knn', eps2=25.0, cpu_frames=5,
               cpu_warm=2, dtype='bf16', weights='random', streams=2),
    # one 20 000-node frame per step leaves the persistent kernels a few tiles per wave: the
    # in-flight batches (three) run on streams of their own, so consecutive forwards overlap,
    # each conv launch on 1536 waves (+15 % and +8 %, profiles/r05_concurrent_ab.log,
    # r05_conv_waves_ab.log)
    'c5': dict(frames=1, nodes=20000, k=10, layers=7, graph='radius', eps2=2.5, cpu_frames=1,
               cpu_warm=1, dtype='fp16', weights='random', streams=3, concurrent=1),
    # the same dense frames batched 8 per step (3.2 M edges per step): the throughput form of
    # config 5 -- a 20 000-node frame alone leaves the persistent kernels ~1 block per wave
    'c5b': dict(frames=8, nodes=20000, k=10, layers=7, graph='radius', eps2=2.5, cpu_frames=1,
                cpu_warm=1, dtype='fp16', weights='random', streams=2),
    # training (yml: k = 10, L = 7), 8 frames per GPU, DDP gradient all-reduce over RCCL
    'c4': dict(frames=8, nodes=3000, k=10, layers=7, graph='knn', eps2=25.0, cpu_frames=1,
               cpu_warm=1),
    # cluster-level classifier GNN (configuration_radarscenes_classifier.yml):
    # 'frames' = samples per GPU, 'nodes' = objects per sample (2..24 measurements each),
    # L = 5 layers of C = 128, complete graph per object
    'cls': dict(frames=64, nodes=200, k=0, layers=5, graph='objects', eps2=0.0, cpu_frames=4,
                cpu_warm=1),
    # real-data front-end: 'frames' = windows per GPU of 10 scans
    # (configuration_radarscenes_gnn.yml:12), 'nodes' = mean measurements per scan
    'frontend': dict(frames=64, nodes=160, k=0, layers=10, graph='scans', eps2=0.0,
                     cpu_frames=16, cpu_warm=2),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=3)
    p.add_argument('--config', default='m', choices=sorted(PRESETS),
                   help='m: the metric configuration (default; fp32, trained weights); '
                        'c2: BASELINE config 2 (bf16); c3: config 3 (C2 frames, 64 per GPU, '
                        'frame-parallel over --gpus, forward only); '
                        'c5: config 5 radius-graph stress (one frame per step); c5b: its frames '
                        'batched 8 per step; '
                        'c4: config 4 training step (forward + backward + SGD, DDP); '
                        'cls: the cluster-level classifier GNN (SURVEY 8(f) rank 4); '
                        'frontend: the real-data front-end (SURVEY 8(f) rank 3)')
    p.add_argument('--frames', type=int, default=None, help='frames per GPU')
    p.add_argument('--nodes', type=int, default=None)
    p.add_argument('--k', type=int, default=None)
    p.add_argument('--layers', type=int, default=None)
    p.add_argument('--dtype', default=None, choices=['bf16', 'fp16', 'fp32'],
                   help='compute dtype (default: the preset\'s -- fp32 for m / c4 / cls, '
                        'bf16 for c2, fp16 for c5)')
    p.add_argument('--weights', default=None, choices=['trained', 'random'],
                   help='trained: the checkpoint committed in tests/golden (L = 7 only)')
    p.add_argument('--no-extra', action='store_true',
                   help='m: skip the extra BASELINE config 2 (bf16) measurement')
    p.add_argument('--cpu-frames', type=int, default=None,
                   help='CPU baseline sample (timed frames)')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--fine-events', action='store_true',
                   help='time every launch with its own HIP event pair (adds ~10 us of stream '
                        'gap per pair to the timed steps)')
    p.add_argument('--seed', type=int, default=synthetic.SEED0)
    p.add_argument('--save-outputs', default=None, metavar='DIR',
                   help='inference configs: every rank writes the four outputs of its first '
                        '--save-frames frames of the last timed step (and their seeds) to '
                        'DIR/rank<r>.npz, for a parity check against the oracle outside the '
                        'bench (tests/test_distributed.py)')
    p.add_argument('--save-frames', type=int, default=2)
    p.add_argument('--streams', type=int, default=None,
                   help='inference configs: batches in flight -- 2 builds step i\'s graph on a '
                        'side stream while step i-1\'s forward runs (pipeline.PipelinedSteps); '
                        '1: build and forward back to back on one stream (default: the preset\'s, '
                        '2 for every inference preset)')
    p.add_argument('--ransac', type=int, default=0,
                   help='frontend config: 1 adds the RANSAC stationary rejection (numpy\'s global '
                        'generator seeded once with --seed; the host draws the consensus sets)')
    p.add_argument('--conv-waves', type=int, default=None,
                   help='16-bit conv static schedule (small graphs): waves per launch, a '
                        'multiple of 64 (default 2048, 1536 with --concurrent 1)')
    p.add_argument('--concurrent', type=int, default=None,
                   help='with --streams > 1: 1 runs each in-flight batch\'s build AND forward on '
                        'a stream of its own, so consecutive forwards overlap too '
                        '(PipelinedSteps(concurrent=True); default: the preset\'s, else 0)')
    a = p.parse_args()
    for key, v in PRESETS[a.config].items():
        if getattr(a, key, None) is None:
            setattr(a, key, v)
    if a.dtype is None:
        a.dtype = {'c2': 'bf16', 'c3': 'bf16', 'c5': 'fp16', 'c5b': 'fp16'}.get(a.config, 'fp32')
    if a.weights is None:
        a.weights = 'random'
    if a.streams is None:
        a.streams = 1
    if a.concurrent is None:
        a.concurrent = 0
    return a


def conv_waves_of(args):
    """The 16-bit conv's static-schedule wave count this run uses on small graphs (None:
    fp32, or the dynamic schedule)."""
    if args.dtype not in ('bf16', 'fp16'):
        return None
    from graph_neural_network_for_radar_perception_amd import engine as _eng
    from graph_neural_network_for_radar_perception_amd import pipeline as _pl
    if args.conv_waves:
        return args.conv_waves
    return (_pl.CONCURRENT_CONV_WAVES if args.concurrent and args.streams > 1
            else _eng.DeviceGraph.CONV_WAVES)


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` run directly (no WORLD_SIZE from a launcher): start N child
    processes of this same script, one per GPU (RANK = LOCAL_RANK = i, WORLD_SIZE = N,
    rendezvous on 127.0.0.1), and return the worst exit code.  Called before this process
    makes any HIP call; the children are new processes (no exec of a GPU process).  Rank 0
    prints the JSON line to the inherited stdout."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    procs = []
    for i in range(n):
        env = dict(os.environ, RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    # a rank that fails would leave the others waiting in a collective: stop them
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.kill()
            for p in procs:
                p.wait()
            return bad[0]
        if all(c == 0 for c in codes):
            return 0
        time.sleep(0.2)


def setup_dist(expect_world=None):
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if expect_world is not None and world != expect_world:
        raise SystemExit(f'bench.py --gpus {expect_world} but WORLD_SIZE={world}: run it '
                         f'directly (it starts the ranks itself) or under torch.distributed.run '
                         f'with --nproc-per-node {expect_world}')
    if torch.cuda.is_available():
        # one GPU per rank; modulo the visible count only so that a rehearsal of the
        # multi-rank logic can share one card (RG_BENCH_BACKEND=gloo)
        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
    if world > 1:
        backend = os.environ.get('RG_BENCH_BACKEND') or ('nccl' if torch.cuda.is_available()
                                                          else 'gloo')
        # rank 0 times the CPU baseline after the timed region while the others wait in a
        # barrier: the timeout covers its worst case (--cpu-frames of a dense frame) with room
        import datetime
        dist.init_process_group(backend, timeout=datetime.timedelta(minutes=60))
    return world, rank, local


def _reduce_device():
    """RCCL reduces device tensors; gloo host tensors."""
    return 'cuda' if dist.get_backend() == 'nccl' else 'cpu'


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_reduce_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_reduce_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def per_rank_counts(x: int, world: int):
    """Every rank's count (rank order), e.g. the frames each rank processed."""
    if world == 1:
        return [int(x)]
    t = torch.tensor([float(x)], dtype=torch.float64, device=_reduce_device())
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [int(v.item()) for v in out]


def rank_frame_seeds(rank: int, frames: int, seed0: int):
    """Frames owned by a rank (weak scaling): seeds seed0 + rank*frames + f."""
    return [seed0 + rank * frames + f for f in range(frames)]


def scatter_aggregate_bench(gb, E, N, steps):
    """The north-star scatter-aggregate kernel on its own: rg_segment_reduce_ordered (PyG aggr
    'add', gnn_blocks.py:57/106 -> scatter_add_ at edge_index[1]) over the step's
    destination-major CSR with its longest-first segment order (rg_segment_order, computed
    once per graph like the CSR itself and reused by every layer; its own time is reported as
    `order_ms`), messages E x 64 already in HBM (synthetic values).  It is the aggregation of
    the unfused paths (max / mean aggregation, residual projections, shapes the fused kernels
    do not take); the default steps fuse it into the conv kernels.  Algorithmic bytes per
    launch: E*C*s_msg + N*C*s_out + (N+1)*4 (+ N*4 for the order).  Timed with
    HIP events on the stream it runs on (torch's current stream: engine launches there)."""
    from graph_neural_network_for_radar_perception_amd import engine
    C = 64
    out = {}
    seg = gb.graph.seg_ptr
    order = engine.segment_order(seg, N)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        engine.segment_order(seg, N)
    b.record()
    torch.cuda.synchronize()
    out['order_ms'] = round(a.elapsed_time(b) / steps, 4)
    for name, tdt, s in (('bf16', torch.bfloat16, 2), ('fp32', torch.float32, 4)):
        msg = torch.randn((E, C), device=seg.device).to(tdt)
        agg = torch.empty((N, C), dtype=tdt, device=seg.device)
        for _ in range(2):
            engine.segment_reduce_ordered(msg, seg, order, N, 'add', agg)
        # one event pair around `steps` back-to-back launches (a pair per launch adds its
        # own stream gap to every timed launch), avg = span / steps
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(steps):
            engine.segment_reduce_ordered(msg, seg, order, N, 'add', agg)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / steps
        nbytes = E * C * s + N * C * s + (N + 1) * 4 + N * 4
        gbs = nbytes / (ms * 1e-3) / 1e9
        out[name] = {'avg_ms': round(ms, 4), 'bytes_per_launch': nbytes,
                     'achieved_gbs': round(gbs, 1), 'hbm_frac': round(gbs / HBM_PEAK_GBS, 4)}
        del msg, agg
    return out


TRAINED_FIXTURE = os.path.join(REPO, 'tests', 'golden', 'model_trained_N50.npz')


def model_state(cfg, weights: str) -> dict:
    """CPU state_dict of Model_Training: the trained checkpoint (the `w/*` arrays of the
    committed fixture, written by tests/golden/make_golden.py from the reference's
    model_weights/gnn/1718175257362) or the seeded random init of the yml architecture."""
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    torch.manual_seed(1234)
    m = Model_Training(cfg, 'cpu')
    if weights == 'trained':
        d = np.load(TRAINED_FIXTURE)
        sd = {k[2:]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith('w/')}
        m.load_state_dict(sd, strict=True)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def make_model(cfg, device, sd):
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    m = Model_Training(cfg, 'cpu')
    m.load_state_dict(sd, strict=True)
    return m.to(device).pred.eval().requires_grad_(False)


def _cgroup_cpu_limit():
    """CPUs granted by the cgroup CPU quota (cgroup v2 cpu.max / v1 cfs files), or None."""
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            return max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    try:
        q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
        per = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
        if q > 0:
            return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return None


def host_threads() -> int:
    """Every host core this process may use: the CPUs in its affinity
    mask, capped by the cgroup CPU quota when one is set (more threads than the quota
    only time-slice the same CPU time)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    lim = _cgroup_cpu_limit()
    return min(n, lim) if lim else n


T_START = time.perf_counter()


def log(msg: str):
    """Progress line on stderr (a long silent phase looks hung to the GPU harness)."""
    print(f'[bench {time.perf_counter() - T_START:7.1f}s] {msg}', file=sys.stderr, flush=True)


class EventList(list):
    """(name, event) pairs; coarse: engine.forward_batched records one pair around the
    whole conv stack ('conv_stack') instead of one per launch."""

    def __init__(self, coarse: bool = False):
        super().__init__()
        self.coarse = coarse


def clock_probe(dev, n_mfma: int = 65536, blocks: int = 256) -> dict:
    """The shader clock the chip holds now (rg_clock_probe, csrc/clock_probe.hip): every wave
    runs a dependent chain of n_mfma v_mfma_f32_32x32x16_bf16 (32 cycles each on its SIMD,
    MI355X_MICROARCH.md) stamped with s_memtime / s_memrealtime.  mhz = median over
    workgroups of shader cycles / wall-clock ticks x the tick rate; mhz_fixed_work = the
    chain's known cycle count / the launch's HIP-event time (a cross-check)."""
    import ctypes
    from graph_neural_network_for_radar_perception_amd import _native as nat
    out = torch.zeros(2 * blocks, dtype=torch.int64, device=dev)
    sink = torch.empty(4 * blocks, dtype=torch.float32, device=dev)
    khz = ctypes.c_int(0)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    nat.check(nat.lib().rg_clock_probe(blocks, n_mfma, out.data_ptr(), sink.data_ptr(),
                                       ctypes.byref(khz), nat.stream_ptr(dev)), 'rg_clock_probe')
    b.record()
    torch.cuda.synchronize()
    o = out.view(blocks, 2).cpu().double()
    ratio = float((o[:, 0] / o[:, 1].clamp(min=1)).median())
    ms = a.elapsed_time(b)
    return {'mhz': round(ratio * khz.value / 1e3, 1), 'wall_clock_khz': khz.value,
            'mhz_fixed_work': round(n_mfma * 32 / (ms * 1e-3) / 1e6, 1), 'probe_ms': round(ms, 4)}


def clock_record(before: dict, after: dict) -> dict:
    return {'mhz_before': before['mhz'], 'mhz_after': after['mhz'],
            'mhz_fixed_work_before': before['mhz_fixed_work'],
            'mhz_fixed_work_after': after['mhz_fixed_work'],
            'method': 'rg_clock_probe right before and right after the timed region: 256 '
                      'workgroups x 4 waves, each a dependent chain of 65536 '
                      'v_mfma_f32_32x32x16_bf16 on register operands; mhz = median s_memtime / '
                      's_memrealtime x wall-clock rate; mhz_fixed_work = 32 cycles x 65536 / the '
                      'probe\'s HIP-event time; kernels[*].kcycles = avg_ms x mean(mhz)'}


def add_cycles(kern: dict, roof: dict, clock: dict):
    """Per-kernel cycles at the measured clock (ms x MHz = thousands of cycles)."""
    mhz = 0.5 * (clock['mhz_before'] + clock['mhz_after'])
    for rec in kern.values():
        if 'avg_ms' in rec:
            rec['kcycles'] = round(rec['avg_ms'] * mhz, 1)
    if 'avg_ms' in roof:
        roof['kcycles'] = round(roof['avg_ms'] * mhz, 1)
        if roof.get('avg_ms_isolated'):
            roof['kcycles_isolated'] = round(roof['avg_ms_isolated'] * mhz, 1)


def event_durations(events):
    """(name:start, name:end) event pairs -> {name: [ms, ...]}"""
    out, open_ = {}, {}
    for name, ev in events:
        base, which = name.rsplit(':', 1)
        if which == 'start':
            open_[base] = ev
        else:
            out.setdefault(base, []).append(open_.pop(base).elapsed_time(ev))
    return out


def pmc_traffic(args, kernel_substr):
    """HBM bytes per launch of the roofline kernel from the newest committed PMC table
    (profiles/rNN_pmc_traffic.json, written by scripts/pmc_traffic.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this same command), or None when
    no table was collected for this workload.  kernel_substr: a name substring, or
    [(substring, weight), ...] summed (every part must be in the table)."""
    parts = [(kernel_substr, 1.0)] if isinstance(kernel_substr, str) else list(kernel_substr)
    import glob
    want = {'frames': args.frames, 'nodes': args.nodes, 'k': args.k, 'layers': args.layers,
            'dtype': args.dtype}
    if args.graph != 'knn':
        want.update(graph=args.graph, eps2=args.eps2)
    for path in sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_pmc_traffic.json')),
                       reverse=True):
        doc = json.load(open(path))
        if doc.get('workload') != want:
            continue
        total, found = 0.0, 0
        for sub, w in parts:
            for name, rec in doc['kernels'].items():
                if sub in name:
                    total += w * float(rec['traffic_bytes'])
                    found += 1
                    break
        if found == len(parts):
            return total, os.path.relpath(path, REPO)
    return None, None


def graph_desc(args) -> str:
    if args.graph == 'radius':
        return f'radius graph eps^2={args.eps2}'
    return f'k={args.k}'


def _cpu_model() -> str:
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def cpu_baseline(args, cfg, sd):
    """The oracle (numpy dense graph build + op-for-op torch fp32 forward, i.e. the
    reference's own CPU algorithm) on a bounded sample of the same workload, same
    weights (2 warm-up frames, median of the timed frames, graph build
    and forward reported separately, on every host core, plus a 1-thread forward)."""
    from oracle import gnn_forward_ref, graph_features_ref as gref
    threads = host_threads()
    warm = args.cpu_warm
    frames = [synthetic.make_frame(args.nodes, args.seed + 10**6 + i)
              for i in range(args.cpu_frames + warm)]
    gmax = float(np.sqrt(np.float64(cfg.max_x ** 2 + cfg.max_y ** 2)))

    def one(fr):
        t0 = time.perf_counter()
        if args.graph == 'radius':
            g = gref.build_frame_graph_radius(fr, args.eps2, gmax)
        else:
            g = gref.build_frame_graph(fr, cfg.ball_query_eps_square,
                                       cfg.k_number_nearest_points, gmax)
        t1 = time.perf_counter()
        cl = [torch.from_numpy(c) for c in synthetic.cluster_lists(args.nodes)]
        with torch.no_grad():
            gnn_forward_ref.forward(sd, cfg, torch.from_numpy(g['node_features']),
                                    torch.from_numpy(g['edge_features']),
                                    torch.from_numpy(g['edge_index']),
                                    None if g['adj_matrix'] is None else
                                    torch.from_numpy(g['adj_matrix']), cl)
        return t1 - t0, time.perf_counter() - t1

    torch.set_num_threads(threads)
    tb, tf = [], []
    for i, fr in enumerate(frames):
        b_, f_ = one(fr)
        log(f'cpu baseline frame {i}: build {b_ * 1e3:.0f} ms, forward {f_ * 1e3:.0f} ms '
            f'({threads} threads)')
        if i >= warm:
            tb.append(b_)
            tf.append(f_)
    build_ms = float(np.median(tb)) * 1e3
    fwd_ms = float(np.median(tf)) * 1e3
    total_ms = float(np.median(np.array(tb) + np.array(tf))) * 1e3
    f1, n1 = None, 0
    if args.graph == 'knn':  # (a 1-thread pass over a 20k-node frame would take minutes)
        # median over >= 5 frames (the reference's CPU path per frame), the
        # first frame of the sample warming the 1-thread pools
        torch.set_num_threads(1)
        one(frames[0])
        t1 = [one(frames[i % len(frames)])[1] for i in range(1, 6)]
        f1, n1 = float(np.median(t1)), len(t1)
        torch.set_num_threads(threads)
    return {'value': round(1e3 / total_ms, 4), 'unit': 'frames/s', 'cores': threads, 'kind': 'port',
            'graph_build_ms': round(build_ms, 1), 'forward_ms': round(fwd_ms, 1),
            'forward_only_frames_per_s': round(1e3 / fwd_ms, 4),
            'forward_1thread_ms': None if f1 is None else round(f1 * 1e3, 1),
            'forward_1thread_frames_per_s': None if f1 is None else round(1.0 / f1, 4),
            'cpu_model': _cpu_model(), 'os_cpu_count': os.cpu_count(),
            'affinity_cpus': len(os.sched_getaffinity(0)), 'cgroup_cpu_limit': _cgroup_cpu_limit(),
            'sample': f'{len(tb)} frame(s) of {args.nodes} nodes, {graph_desc(args)}, '
                      f'L={args.layers} after {warm} warm-up frame(s): oracle graph build (dense '
                      f'numpy, graph_features.py) + torch-fp32 forward (gnn_detector.py), median '
                      f'{total_ms:.0f} ms/frame at torch threads={threads}'
                      + (f'; the forward also timed on 1 thread (median of {n1} frames after '
                         f'1 warm-up)' if f1 else '')}


def batch_labels(frames, gb, cfg, device):
    """Synthetic labels of a batch on its device-built graph (synthetic.batch_labels)."""
    rp = gb.row_ptr.cpu().numpy().astype(np.int64)
    col = gb.col[:int(rp[-1])].cpu().numpy().astype(np.int64)
    lab, clusters = synthetic.batch_labels(frames, rp, col, cfg.num_classes)
    lab = {k: torch.from_numpy(v).to(device) for k, v in lab.items()}
    lab['class_weights'] = torch.tensor(cfg.class_weights_dyn, dtype=torch.float32, device=device)
    return lab, clusters


def cpu_train_baseline(args, cfg):
    """The oracle's training step (torch fp32 forward + autograd backward of
    Model_Training + Loss_Graph, i.e. the reference's CPU algorithm) on a bounded sample:
    args.cpu_frames single-frame steps after args.cpu_warm warm-up frames."""
    from oracle import graph_features_ref as gref, train_ref
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    threads = host_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(1234)
    sd = {k: v.detach() for k, v in Model_Training(cfg, 'cpu').state_dict().items()}
    gmax = float(np.sqrt(np.float64(cfg.max_x ** 2 + cfg.max_y ** 2)))
    times = []
    for i in range(args.cpu_warm + args.cpu_frames):
        fr = synthetic.make_frame(args.nodes, args.seed + 10**6 + i)
        t0 = time.perf_counter()
        g = gref.build_frame_graph(fr, cfg.ball_query_eps_square, cfg.k_number_nearest_points, gmax)
        lb = synthetic.make_labels(fr, g['edge_index'], cfg.num_classes, i)
        f = {'node_features': torch.from_numpy(g['node_features']),
             'edge_features': torch.from_numpy(g['edge_features']),
             'edge_index': torch.from_numpy(g['edge_index']),
             'node_class': torch.from_numpy(lb['node_class']),
             'node_offsets': torch.from_numpy(lb['node_offsets']),
             'edge_class': torch.from_numpy(lb['edge_class']),
             'cluster_node_idx': [torch.from_numpy(c) for c in lb['cluster_node_idx']],
             'cluster_labels': torch.from_numpy(lb['cluster_labels'])}
        train_ref.training_grads(sd, cfg, [f])
        if i >= args.cpu_warm:
            times.append(time.perf_counter() - t0)
    ms = float(np.median(times)) * 1e3
    return {'value': round(1e3 / ms, 4), 'unit': 'frames/s', 'cores': threads, 'kind': 'port',
            'step_ms_per_frame': round(ms, 1), 'cpu_model': _cpu_model(),
            'sample': f'{len(times)} single-frame training step(s) of {args.nodes} nodes, k={args.k}, '
                      f'L={args.layers} after {args.cpu_warm} warm-up: oracle graph build + '
                      'labels + torch-fp32 forward + Loss_Graph + autograd backward, '
                      f'torch threads={threads} (SGD update excluded)'}


def train_main(args, world, rank, local):
    """BASELINE config 4: one data-parallel training iteration per step."""
    from graph_neural_network_for_radar_perception_amd.gnn_detector import Model_Training
    from graph_neural_network_for_radar_perception_amd.graph_features import (FrameBatch,
                                                                                build_graph_batch)
    from graph_neural_network_for_radar_perception_amd.training import RadarGNNTrainer
    dev = torch.device('cuda', torch.cuda.current_device())  # set from LOCAL_RANK in setup_dist
    cfg = default_config(graph_convolution_stem_channels=[64] * args.layers,
                         k_number_nearest_points=args.k)
    torch.manual_seed(1234)
    model = Model_Training(cfg, dev).to(dev).train()
    seeds = rank_frame_seeds(rank, args.frames, args.seed)
    frames = [synthetic.make_frame(args.nodes, s) for s in seeds]
    batch0 = FrameBatch.from_frames(frames, device=dev)
    labels, clusters = batch_labels(frames, build_graph_batch(batch0, cfg), cfg, dev)
    batch = FrameBatch.from_frames(frames, clusters, device=dev)
    trainer = RadarGNNTrainer(model, cfg, world)
    for _ in range(args.warmup):
        losses, acc, gb = trainer.step(batch, labels)
    torch.cuda.synchronize()
    E = int(gb.n_edges_dev.item())
    clk0 = clock_probe(dev)
    barrier(world)
    torch.cuda.synchronize()
    events = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        losses, acc, gb = trainer.step(batch, labels, events=events)
    torch.cuda.synchronize()
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    clock = clock_record(clk0, clock_probe(dev))
    frames_total = sum_over_ranks(args.frames * args.steps, world)
    rank_frames = per_rank_counts(args.frames * args.steps, world)
    durs = event_durations(events)
    # roofline of the forward tape (the step's largest phase: the f32 row-MLP chain kernel
    # writing every layer's pre-norm / activation rows): the model's forward flops in the
    # form the training forward computes them (message MLP over all 192 inputs per edge,
    # SURVEY §8(d)) on the f32 MFMA peak (v_mfma_f32_16x16x4_f32); the backward beside it
    # at twice those flops (dX and dW per layer)
    N = args.frames * args.nodes
    U = int(gb.graph.n_pairs_dev.item())
    Fw = (84992.0 * N + 118272.0 * E + args.layers * (65536.0 * E + 16384.0 * N) + 99456.0 * N
          + 33024.0 * U + 9088.0 * (N / 5))
    fwd_ms = float(np.mean(durs['train_forward']))
    bwd_ms = float(np.mean(durs['train_backward']))
    roof = {'kernel': 'training forward tape (rg_mlp_chain f32 with save_pre / save_out, '
                      'gnn_detector.py:428-478 + loss.py:37-76)',
            'bound': 'mfma', 'achieved': round(Fw / (fwd_ms * 1e-3) / 1e12, 2),
            'peak': MFMA_PEAK_TFLOPS['fp32'], 'unit': 'TFLOP/s',
            'frac': round(Fw / (fwd_ms * 1e-3) / 1e12 / MFMA_PEAK_TFLOPS['fp32'], 4),
            'traffic': None, 'avg_ms': round(fwd_ms, 4), 'flops_per_launch': Fw,
            'timing': 'HIP events on the launch stream around the forward of every timed step',
            'backward_ms': round(bwd_ms, 4),
            'backward_tflops': round(2 * Fw / (bwd_ms * 1e-3) / 1e12, 2)}
    line = {
        'metric': 'radar frames/sec training (BASELINE config 4: yml k=10, L=7, batch 8/GPU, '
                  'SGD momentum 0.9, DDP gradient all-reduce over RCCL)',
        'value': round(frames_total / elapsed, 2), 'unit': 'frames/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'fp32',
        'data': 'synthetic RadarScenes-shaped frames + synthetic labels (SURVEY.md §8(d)), '
                'random-init weights of the yml architecture',
        'config': {'workload': f'BASELINE config 4: {args.frames} frames x {args.nodes} nodes per '
                               f'GPU, k={args.k}, L={args.layers}; step = graph build + features + '
                               'forward tape + Loss_Graph + backward + all-reduce + SGD',
                   'frames_per_gpu': args.frames, 'nodes_per_frame': args.nodes, 'k': args.k,
                   'layers': args.layers, 'edges_per_gpu': E,
                   'parallelism': f'data-parallel x{world} (one flat-gradient all-reduce per step)',
                   'frames_per_rank_timed': rank_frames,
                   'backend': dist.get_backend() if world > 1 else None},
        'last_losses': [round(float(x), 5) for x in losses.cpu()],
        'applied_steps': trainer.opt.applied_steps(),
        'roofline': roof,
        'clock': clock,
    }
    add_cycles({}, roof, clock)
    if rank == 0 and not args.no_cpu_baseline:  # after the timed region, every world size
        line['cpu_baseline'] = cpu_train_baseline(args, cfg)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()  # the other ranks wait for rank 0's CPU baseline
        dist.destroy_process_group()


def cpu_classifier_baseline(args, cfg, sd):
    """The oracle (numpy compute_edge_index + op-for-op torch fp32 classifier forward, the
    reference's CPU algorithm) on a bounded sample: args.cpu_frames samples after
    args.cpu_warm warm-up samples, median per sample."""
    from oracle import classifier_ref
    threads = host_threads()
    torch.set_num_threads(threads)
    times = []
    for i in range(args.cpu_warm + args.cpu_frames):
        smp = synthetic.make_objects(args.nodes, args.seed + 10**6 + i)
        t0 = time.perf_counter()
        ei = classifier_ref.compute_edge_index(smp['object_size'].tolist())
        with torch.no_grad():
            classifier_ref.forward(sd, cfg, torch.from_numpy(smp['node_features']),
                                   torch.from_numpy(ei), torch.from_numpy(smp['object_size']))
        if i >= args.cpu_warm:
            times.append(time.perf_counter() - t0)
    ms = float(np.median(times)) * 1e3
    return {'value': round(args.nodes * 1e3 / ms, 2), 'unit': 'objects/s', 'cores': threads,
            'kind': 'port', 'ms_per_sample': round(ms, 1), 'cpu_model': _cpu_model(),
            'sample': f'{len(times)} sample(s) of {args.nodes} objects after {args.cpu_warm} '
                      'warm-up: oracle compute_edge_index (numpy block_diag + nonzero) + '
                      f'torch-fp32 classifier forward, median, torch threads={threads}'}


def cls_main(args, world, rank, local):
    """Cluster-level classifier GNN: one step = the batch's graph
    (complete graph per object, from the object sizes) + pooling ranges + encoder + L
    conv blocks + max-pool + stem/head, over `frames` samples of `nodes` objects."""
    from graph_neural_network_for_radar_perception_amd.classifier import Model_Training
    from graph_neural_network_for_radar_perception_amd.classifier import engine as ce
    from graph_neural_network_for_radar_perception_amd.config import default_classifier_config
    dev = torch.device('cuda', torch.cuda.current_device())  # set from LOCAL_RANK in setup_dist
    cfg = default_classifier_config(classifier_graph_convolution_stem_channels=[128] * args.layers)
    torch.manual_seed(1234)
    model = Model_Training(cfg)
    sd_cpu = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(dev).eval().requires_grad_(False)
    seeds = rank_frame_seeds(rank, args.frames, args.seed)
    smps = [synthetic.make_objects(args.nodes, s) for s in seeds]
    nf = torch.from_numpy(np.concatenate([s['node_features'] for s in smps])).to(dev)
    sizes = np.concatenate([s['object_size'] for s in smps])
    osz = torch.from_numpy(sizes).to(dev)
    nodes = [int(s['object_size'].sum()) for s in smps]
    sobj = torch.tensor(np.arange(0, args.frames + 1) * args.nodes, dtype=torch.int32).to(dev)
    nbase = torch.tensor(np.cumsum([0] + nodes[:-1]), dtype=torch.int32).to(dev)
    N = int(sum(nodes))
    E = int((sizes * (sizes - 1)).sum())

    def step(events=None):
        g = ce.object_graph(osz, N, E)
        b, e = ce.object_row_ranges(osz, sobj, nbase, args.frames)
        return ce.forward_graph(model.pred, nf, g, b, e, args.dtype, events)

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        events = []
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(events)
        torch.cuda.synchronize()
        barrier(world)
        elapsed = max_over_ranks(time.perf_counter() - t0, world)
    durs = event_durations(events)
    objs_total = sum_over_ranks(args.frames * args.nodes * args.steps, world)
    s = 2 if args.dtype == 'bf16' else 4
    C = 128
    kern = {k: {'avg_ms': round(float(np.mean(v)), 4), 'launches_per_step': len(v) // args.steps}
            for k, v in durs.items()}
    ms = float(np.mean(durs['message_chain']))
    flops = 2.0 * (2 * C * C + C * C) * E        # msg MLP 256 -> 128 -> 128 per edge
    tf = flops / (ms * 1e-3) / 1e12
    peak = MFMA_PEAK_TFLOPS[args.dtype]
    kern['message_chain'].update(flops_per_launch=flops, algorithmic_tflops=round(tf, 2))
    agg_ms = float(np.mean(durs['segment_reduce']))
    agg_bytes = E * C * s + N * C * s + (N + 1) * 4
    agg_gbs = agg_bytes / (agg_ms * 1e-3) / 1e9
    kern['segment_reduce'].update(bytes_per_launch=agg_bytes, algorithmic_gbs=round(agg_gbs, 1),
                                  hbm_frac=round(agg_gbs / HBM_PEAK_GBS, 4))
    line = {
        'metric': 'classifier objects/sec (cluster-level classifier GNN, SURVEY §8(f) rank 4)',
        'value': round(objs_total / elapsed, 1), 'unit': 'objects/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': args.dtype,
        'data': 'synthetic object samples (synthetic.make_objects: 2..24 measurements per '
                'object), random-init weights of the classifier yml architecture',
        'config': {'workload': f'classifier: {args.frames} samples x {args.nodes} objects per GPU, '
                               f'L={args.layers} (C=128); step = complete-graph build + pooling '
                               'ranges + encoder + message passing + max-pool + head',
                   'samples_per_gpu': args.frames, 'objects_per_sample': args.nodes,
                   'nodes_per_gpu': N, 'edges_per_gpu': E, 'layers': args.layers,
                   'parallelism': f'sample-parallel x{world} (no collective in the step)'},
        'roofline': {'kernel': 'message_chain (rg_mlp_chain GATHER3, classifier/blocks.py:84-85)',
                     'bound': 'mfma', 'achieved': round(tf, 2), 'peak': peak, 'unit': 'TFLOP/s',
                     'frac': round(tf / peak, 4), 'traffic': None},
        'kernels': kern,
    }
    if rank == 0 and not args.no_cpu_baseline:  # after the timed region, every world size
        line['cpu_baseline'] = cpu_classifier_baseline(args, cfg, sd_cpu)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()  # the other ranks wait for rank 0's CPU baseline
        dist.destroy_process_group()


def frontend_main(args, world, rank, local):
    """Real-data front-end: a batch of windows of 10 radar scans in
    HBM -> stationary gate, ego compensation, ground truth, grid + moving selection ->
    the dynamic frames (frame_ptr) the graph build takes.  One step = the batch; the
    step synchronises once (the selected count), as the reference's boolean indexing."""
    from graph_neural_network_for_radar_perception_amd import frontend
    dev = torch.device('cuda', torch.cuda.current_device())
    seeds = rank_frame_seeds(rank, args.frames, args.seed)
    wins = [synthetic.make_scan_window(s, n_scans=args.layers, mean_meas=args.nodes)
            for s in seeds]
    batch = frontend.scan_window_batch(wins, dev)
    n_meas = batch.n_meas

    def step(events=None):
        if events is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            events.append(('sync:start', ev))
        d = frontend.extract_and_sync_radar_data(batch, reject_outlier_by_ransac=bool(args.ransac))
        if events is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            events.append(('sync:end', ev))
        gt = frontend.compute_ground_truth(d)
        return frontend.select_dynamic(d, gt)

    np.random.seed(args.seed)   # the RANSAC draws (meas_selection.py:128)
    for _ in range(args.warmup):
        dd, _ = step()
    torch.cuda.synchronize()
    n_dyn = int(dd['frame_ptr'][-1].item())
    events = []
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(events)
    torch.cuda.synchronize()
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    durs = event_durations(events)
    total = sum_over_ranks(args.frames * args.steps, world)
    ms = float(np.mean(durs['sync']))
    nbytes = n_meas * (5 * 4 + 4 * 4 + 1)   # 5 f32 fields in, px py vx vy out, flag
    gbs = nbytes / (ms * 1e-3) / 1e9
    line = {
        'metric': 'radar windows/sec through the real-data front-end (SURVEY §8(f) rank 3)',
        'value': round(total / elapsed, 1), 'unit': 'windows/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(elapsed / args.steps * 1e3, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32/f64',
        'data': 'synthetic RadarScenes-shaped scan windows (synthetic.make_scan_window)',
        'config': {'workload': f'frontend: {args.frames} windows x {args.layers} scans x '
                               f'~{args.nodes} measurements per GPU; step = sync (gate, ego '
                               'compensation' + (', RANSAC: host draws + device fits' if args.ransac
                                                 else '') + ') + labels + grid/moving selection',
                   'ransac': bool(args.ransac),
                   'windows_per_gpu': args.frames, 'measurements_per_gpu': n_meas,
                   'dynamic_per_gpu': n_dyn,
                   'parallelism': f'window-parallel x{world} (no collective in the step)'},
        'roofline': {'kernel': 'frontend_sync_kernel (rg_frontend_sync)', 'bound': 'hbm',
                     'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(gbs / HBM_PEAK_GBS, 4), 'traffic': None,
                     'avg_ms': round(ms, 4), 'bytes_per_launch': nbytes},
    }
    if rank == 0 and not args.no_cpu_baseline:  # after the timed region, every world size
        from oracle import frontend_ref  # the CPU baseline leg only
        sample = wins[:args.cpu_frames]
        t = time.perf_counter()
        for w in sample:
            w2 = dict(w)
            w2['track_key'] = frontend._host_track_keys(w)
            full = frontend_ref.sync_window(w2, reject_outlier_by_ransac=bool(args.ransac))
            frontend_ref.select_dynamic(full, frontend_ref.ground_truth(full, w2['track_key']))
        dt = time.perf_counter() - t
        line['cpu_baseline'] = {'value': round(len(sample) / dt, 1), 'unit': 'windows/s',
                                'cores': 1, 'kind': 'port',
                                'sample': f'{len(sample)} windows through the numpy oracle '
                                          '(oracle/frontend_ref.py), one thread'}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()  # the other ranks wait for rank 0's CPU baseline
        dist.destroy_process_group()


def workload_name(args) -> str:
    head = {'m': 'M (the metric configuration, SURVEY §8(d))',
            'c2': 'BASELINE config 2', 'c5': 'BASELINE config 5',
            'c5b': 'BASELINE config 5 frames batched',
            'c3': f'BASELINE config 3 ({args.frames * max(args.gpus, 1)} frames frame-parallel '
                  f'over {max(args.gpus, 1)} GPU(s), forward only, no collective in the step)'
            }.get(args.config, args.config)
    return (f'{head}: {args.frames} frame(s) x {args.nodes} nodes per GPU, {graph_desc(args)}, '
            f'L={args.layers}, {args.dtype}, {args.weights} weights; step = graph build + '
            'node/edge features + encoders + message passing + 4 heads')


def save_rank_outputs(args, rank, seeds, gb, out):
    """This rank's outputs of its first args.save_frames frames (the last timed step):
    node_cls / node_reg rows, the link pairs (global node ids) whose source lies in those
    frames with their logits, and the frames' cluster logits -- plus the frame seeds, so a
    checker can rebuild the same frames and run the oracle on them (the bench itself never
    touches oracle/ outside its CPU-baseline leg)."""
    F = min(args.save_frames, args.frames)
    N = args.nodes
    ncl = len(synthetic.cluster_lists(N))
    U = int(gb.graph.n_pairs_dev.item())
    ps = gb.graph.pair_src[:U].cpu().numpy()
    pd = gb.graph.pair_dst[:U].cpu().numpy()
    sel = ps < F * N
    os.makedirs(args.save_outputs, exist_ok=True)
    np.savez(os.path.join(args.save_outputs, f'rank{rank}.npz'),
             seeds=np.asarray(seeds[:F]), nodes=N, k=args.k, eps2=args.eps2,
             layers=args.layers, dtype=args.dtype,
             node_cls=out.node_cls[:F * N].float().cpu().numpy(),
             node_reg=out.node_reg[:F * N].float().cpu().numpy(),
             pair_src=ps[sel], pair_dst=pd[sel],
             link_cls=out.link_cls[:U].float().cpu().numpy()[sel],
             obj_cls=out.obj_cls[:F * ncl].float().cpu().numpy())
    log(f'rank {rank}: outputs of {F} frame(s) saved to {args.save_outputs}')


def gnn_measure(args, world, dev, cfg, sd, scatter=True):
    """Warm up, then time args.steps full steps (barrier + synchronize on both sides,
    max over ranks), then the forward alone; per-kernel HIP-event durations and the
    roofline of the conv layer kernel."""
    from graph_neural_network_for_radar_perception_amd.graph_features import FrameBatch
    from graph_neural_network_for_radar_perception_amd.pipeline import (PipelinedSteps,
                                                                         RadarGNNPipeline)
    from graph_neural_network_for_radar_perception_amd import _native as nat
    rank = dist.get_rank() if world > 1 else 0
    mode = nat.GRAPH_RADIUS if args.graph == 'radius' else nat.GRAPH_KNN
    model = make_model(cfg, dev, sd)
    seeds = rank_frame_seeds(rank, args.frames, args.seed)
    frames = [synthetic.make_frame(args.nodes, s) for s in seeds]
    clusters = [synthetic.cluster_lists(args.nodes) for _ in seeds]
    batch = FrameBatch.from_frames(frames, clusters, device=dev)
    if args.streams > 1:
        stepper = PipelinedSteps(model, cfg, args.dtype, mode=mode, eps2=args.eps2,
                                 depth=args.streams, concurrent=bool(args.concurrent),
                                 conv_waves=args.conv_waves)
    else:
        stepper = RadarGNNPipeline(model, cfg, args.dtype, mode=mode, eps2=args.eps2,
                                   conv_waves=args.conv_waves)
    log(f'{args.config}: {args.frames} frames generated; warm-up')

    with torch.no_grad():
        # every in-flight pipeline warms once (its workspaces, a radius graph's capacity)
        for _ in range(max(args.warmup, args.streams)):
            gb, out = stepper.step(batch)
        torch.cuda.synchronize()
        pipe = stepper.pipes[(stepper.i - 1) % stepper.depth] if args.streams > 1 else stepper
        E = int(gb.n_edges_dev.item())
        log(f'{args.config}: warm-up done, E = {E}; timing {args.steps} steps')
        # ---- timed region: K full steps -----------------------------------------
        # coarse events: one pair around the edge encoder and one around the conv stack
        # per step (a pair per launch cost ~10 us of stream gap each); --fine-events
        # times every launch
        events = EventList(coarse=not args.fine_events)
        clk0 = clock_probe(dev)
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            gb, out = stepper.step(batch, events=events)
        torch.cuda.synchronize()
        barrier(world)
        elapsed = max_over_ranks(time.perf_counter() - t0, world)
        clock = clock_record(clk0, clock_probe(dev))
        if args.streams > 1:
            pipe = stepper.pipes[(stepper.i - 1) % stepper.depth]
        if args.save_outputs:
            save_rank_outputs(args, rank, seeds, gb, out)
        durs = event_durations(events)
        if 'conv_stack' in durs:  # per-layer launch time = span / layers
            durs['conv_fused'] = [ms / args.layers for ms in durs.pop('conv_stack')]
        # ---- forward only (graph + features already built) -----------------------
        barrier(world)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ev_iso = EventList(coarse=True)
        for _ in range(args.steps):
            pipe.forward(batch, gb, ev_iso)
        torch.cuda.synchronize()
        barrier(world)
        fwd_elapsed = max_over_ranks(time.perf_counter() - t1, world)
        # the conv stack without a concurrent graph build (the timed steps overlap step i's
        # build with step i-1's forward when --streams > 1)
        iso = event_durations(ev_iso).get('conv_stack')
        iso_ms = float(np.mean(iso)) / args.layers if iso else None
        sc = (scatter_aggregate_bench(gb, E, args.frames * args.nodes, max(args.steps, 5))
              if scatter else None)

    frames_total = sum_over_ranks(args.frames * args.steps, world)
    rank_frames = per_rank_counts(args.frames * args.steps, world)
    N = args.frames * args.nodes
    s = 2 if args.dtype in ('bf16', 'fp16') else 4
    C = 64
    kern = {}
    for name, ms in durs.items():
        kern[name] = {'avg_ms': round(float(np.mean(ms)), 4), 'launches_per_step':
                      len(ms) // args.steps}
    peak_tf = MFMA_PEAK_TFLOPS[args.dtype]
    ref_tf = None
    conv_exec, conv_peak = 1.0, MFMA_PEAK_TFLOPS[args.dtype]
    if 'conv_fused' in durs:
        # fused conv layer: gather x_i, x_j, e -> msg MLP -> segment sum -> update MLP.
        # Roofline flops = the dense work the kernel's algorithm needs:
        #  fp32 (rg_conv_layer_f32): msg0 factorised, W_xi x_i + W_xj x_j once per NODE
        #    (P | Q, 64 -> 256), per edge W_e e (64 -> 128) + msg1 (128 -> 64), per node the
        #    update (128 -> 64): 32768 E + 49152 N
        #  bf16 (rg_conv_layer_fused): per node P = W_xi x_i, per edge W_[xj,e] (128 -> 128)
        #    + msg1, per node the update: 49152 E + 32768 N
        # The reference form (SURVEY §8(d), msg0 over all 192 inputs per edge: 65536 E +
        # 16384 N) is reported beside it as reference_form_tflops.
        #  fp32 x3 (rg_conv_layer_x3, the default): one layer = W_e e + msg1 per edge, the
        #    update per node, and the NEXT layer's P | Q per node (the first layer's P | Q
        #    is rg_conv_proj_x3): timed as one span over the whole stack (proj + L layers),
        #    so per layer 32768 E + 16384 N + 32768 N
        #    (--fine-events: the layer launches alone, 32768 E + 16384 N + 32768 N (L-1)/L)
        from graph_neural_network_for_radar_perception_amd import engine as _eng
        ms = float(np.mean(durs['conv_fused']))
        ref_flops = 65536.0 * E + 16384.0 * N
        x3 = args.dtype == 'fp32' and _eng.F32_ARITH == 'x3'
        if x3 and not args.fine_events:
            flops = 32768.0 * E + 49152.0 * N
        elif x3:
            flops = 32768.0 * E + 16384.0 * N + 32768.0 * N * (args.layers - 1) / args.layers
        elif args.dtype == 'fp32':
            flops = 32768.0 * E + 49152.0 * N
        else:
            flops = 49152.0 * E + 32768.0 * N
        nbytes = E * (C * s + 8) + N * (2 * C * s + 4)     # e rows + (src,dst) once; x in/out once
        tf = flops / (ms * 1e-3) / 1e12
        ref_tf = ref_flops / (ms * 1e-3) / 1e12
        gbs = nbytes / (ms * 1e-3) / 1e9
        kern['conv_fused'].update(algorithmic_tflops=round(tf, 2), algorithmic_gbs=round(gbs, 1),
                                  flops_per_launch=flops, bytes_per_launch=nbytes,
                                  reference_form_tflops=round(ref_tf, 2))
        if x3:
            kname = ('conv_fused (conv_x3_sp_kernel = rg_conv_layer_x3: f32 products from exact '
                     '3-term bf16 splits on v_mfma_f32_32x32x16_bf16, gnn_blocks.py:96-113)')
            # roofline on the pipe it runs on: the bf16 matrix cores, which execute six bf16
            # products per f32 product
            conv_exec, conv_peak = 6.0, MFMA_PEAK_TFLOPS['bf16']
            kern['conv_fused']['bf16_mfma_tflops'] = round(6 * tf, 2)
        elif args.dtype == 'fp32':
            kname = ('conv_fused (rg_conv_layer_f32: per-node projection + fused layer launches, '
                     'gnn_blocks.py:96-113)')
        else:
            kname = 'conv_fused (rg_conv_layer_fused, gnn_blocks.py:96-113)'
        if x3 and not args.fine_events:  # one layer of the stack: edge + node launches + proj / L
            tparts = [('conv_x3_sp_kernel', 1.0), ('node_x3_kernel', 1.0),
                      ('proj_x3_kernel', 1.0 / args.layers)]
        elif x3:
            tparts = [('conv_x3_sp_kernel', 1.0), ('node_x3_kernel', 1.0)]
        else:
            tparts = 'conv_f32' if args.dtype == 'fp32' else 'fused_conv'
        traffic, tsrc = pmc_traffic(args, tparts)
    else:
        # message chain: gather x_i, x_j, e -> 192->128->64 MLP (norm + act) -> messages
        ms = float(np.mean(durs['message_chain']))
        flops = 65536.0 * E                              # 2*(192*128+128*64) per edge
        nbytes = E * (3 * C * s + C * s + 8)             # x_i, x_j, e read; msg write; 2 int32 idx
        tf = flops / (ms * 1e-3) / 1e12
        gbs = nbytes / (ms * 1e-3) / 1e9
        kern['message_chain'].update(algorithmic_tflops=round(tf, 2), algorithmic_gbs=round(gbs, 1),
                                     flops_per_launch=flops, bytes_per_launch=nbytes)
        kname = 'message_chain (rg_mlp_chain GATHER3, gnn_blocks.py:104-113)'
        traffic, tsrc = pmc_traffic(args, 'chain_kernel')
        agg_ms = float(np.mean(durs['segment_reduce']))
        agg_bytes = E * C * s + N * C * s + (N + 1) * 4     # SURVEY §8(d) B_agg
        agg_gbs = agg_bytes / (agg_ms * 1e-3) / 1e9
        kern['segment_reduce'].update(algorithmic_gbs=round(agg_gbs, 1), bytes_per_launch=agg_bytes,
                                      hbm_frac=round(agg_gbs / HBM_PEAK_GBS, 4))
    if 'edge_encoder' in durs:
        enc_ms = float(np.mean(durs['edge_encoder']))
        enc_flops = 118272.0 * E
        enc_tf = enc_flops / (enc_ms * 1e-3) / 1e12
        kern['edge_encoder'].update(algorithmic_tflops=round(enc_tf, 2), flops_per_launch=enc_flops)
        from graph_neural_network_for_radar_perception_amd import engine as _eng
        if args.dtype == 'fp32' and _eng.F32_ARITH == 'x3':
            # chain_x3_kernel: six bf16 products per f32 product on the bf16 matrix cores
            kern['edge_encoder'].update(bf16_mfma_tflops=round(6 * enc_tf, 2),
                                        mfma_frac=round(6 * enc_tf / MFMA_PEAK_TFLOPS['bf16'], 4))
        else:
            kern['edge_encoder']['mfma_frac'] = round(enc_tf / peak_tf, 4)
    frac_mfma = conv_exec * tf / conv_peak
    frac_hbm = gbs / HBM_PEAK_GBS
    if frac_mfma >= frac_hbm:
        roof = {'kernel': kname, 'bound': 'mfma', 'achieved': round(conv_exec * tf, 2),
                'peak': conv_peak, 'unit': 'TFLOP/s', 'frac': round(frac_mfma, 4),
                'traffic': traffic, 'hbm_frac': round(frac_hbm, 4)}
        if conv_exec != 1.0:
            roof.update(f32_tflops=round(tf, 2), executed_per_f32_flop=conv_exec,
                        f32_equivalent_peak=round(conv_peak / conv_exec, 1))
    else:
        roof = {'kernel': kname, 'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS,
                'unit': 'GB/s', 'frac': round(frac_hbm, 4), 'traffic': traffic,
                'mfma_frac': round(frac_mfma, 4)}
    roof.update(avg_ms=round(ms, 4),
                timing=('HIP events on the launch stream, timed region: ' +
                        ('one pair per launch' if args.fine_events else
                         'one pair around the conv stack per step, avg = span / layers') +
                        (f'; {args.streams} batches in flight (the next step\'s graph build '
                         'runs beside this conv stack)' if args.streams > 1 and not args.concurrent
                         else '') +
                        (f'; {args.streams} batches in flight on streams of their own (the next '
                         'step\'s build AND forward overlap this conv stack, so a span holds both '
                         'forwards\' kernels: avg_ms_isolated / frac_isolated are the kernel\'s own)'
                         if args.streams > 1 and args.concurrent else '')),
                flops_per_launch=flops)
    if iso_ms:
        # the same kernels timed in the forward-only loop (nothing runs beside them)
        roof.update(avg_ms_isolated=round(iso_ms, 4),
                    frac_isolated=round(roof['frac'] * ms / iso_ms, 4))
    if ref_tf is not None:
        roof['reference_form_tflops'] = round(ref_tf, 2)
    if traffic is not None:
        roof.update(traffic_unit='bytes/launch', traffic_source=tsrc,
                    algorithmic_bytes=nbytes, traffic_over_algorithmic=round(traffic / nbytes, 3))
    F = (84992.0 * N + 118272.0 * E + args.layers * (65536.0 * E + 16384.0 * N) + 99456.0 * N
         + 33024.0 * (E / 2) + 9088.0 * (N / 5))       # SURVEY §8(d) forward flops
    fwd_ms = fwd_elapsed / args.steps * 1e3
    add_cycles(kern, roof, clock)
    return {'value': frames_total / elapsed, 'elapsed': elapsed, 'ms_step': elapsed / args.steps * 1e3,
            'forward_fps': frames_total / fwd_elapsed, 'forward_ms': fwd_ms, 'E': E,
            'forward_tflops': F / (fwd_ms * 1e-3) / 1e12, 'roof': roof, 'kern': kern,
            'scatter': sc, 'rank_frames': rank_frames, 'clock': clock}


def main():
    args = parse()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        raise SystemExit(launch_ranks(args.gpus))
    world, rank, local = setup_dist(args.gpus)
    if not torch.cuda.is_available():
        raise SystemExit('bench.py needs a HIP device')
    if args.config == 'c4':
        return train_main(args, world, rank, local)
    if args.config == 'cls':
        return cls_main(args, world, rank, local)
    if args.config == 'frontend':
        return frontend_main(args, world, rank, local)
    if args.weights == 'trained' and args.layers != 7:
        raise SystemExit('--weights trained needs --layers 7 (the checkpoint has 7 conv blocks)')
    dev = torch.device('cuda', torch.cuda.current_device())  # set from LOCAL_RANK in setup_dist
    cfg = default_config(graph_convolution_stem_channels=[64] * args.layers,
                         k_number_nearest_points=args.k)
    sd = model_state(cfg, args.weights)
    log(f'config {args.config}, dtype {args.dtype}, weights {args.weights}')
    r = gnn_measure(args, world, dev, cfg, sd)
    log(f'{args.config}: {r["value"]:.1f} frames/s, {r["ms_step"]:.3f} ms/step')
    line = {
        'metric': METRIC, 'value': round(r['value'], 2), 'unit': 'frames/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(r['ms_step'], 3),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': args.dtype,
        'data': 'synthetic RadarScenes-shaped frames (SURVEY.md §8(d), seeded); '
                + ('weights of the trained checkpoint 1718175257362 (committed fixture)'
                   if args.weights == 'trained' else 'random-init weights of the yml architecture'),
        'config': {'workload': workload_name(args),
                   'frames_per_gpu': args.frames, 'nodes_per_frame': args.nodes,
                   'graph': args.graph, 'k': args.k if args.graph == 'knn' else None,
                   'eps2': args.eps2, 'layers': args.layers, 'edges_per_gpu': r['E'],
                   'edges_per_frame': round(r['E'] / args.frames, 1),
                   'parallelism': f'frame-parallel x{world} (no collective in the step)',
                   'frames_per_rank_timed': r['rank_frames'],
                   'streams': args.streams, 'concurrent_forwards': bool(args.concurrent and args.streams > 1),
                   'conv_waves': conv_waves_of(args),
                   'backend': dist.get_backend() if world > 1 else None},
        'forward_only_frames_per_s': round(r['forward_fps'], 2),
        'forward_algorithmic_tflops': round(r['forward_tflops'], 2),
        'roofline': r['roof'],
        'scatter_aggregate': dict(r['scatter'], kernel='rg_segment_reduce_ordered sum over the step\'s '
                                  'destination-major CSR, longest-first segment order (standalone; fused into the conv kernels in '
                                  'the step)', bound='hbm', peak_gbs=HBM_PEAK_GBS),
        'kernels': r['kern'],
        'clock': r['clock'],
    }
    if args.config == 'm' and not args.no_extra:
        # the same run also times BASELINE config 2 (bf16, random init) as an extra key
        a2 = argparse.Namespace(**vars(args))
        a2.config = 'c2'
        for key, v in PRESETS['c2'].items():
            setattr(a2, key, v)
        cfg2 = default_config(graph_convolution_stem_channels=[64] * a2.layers,
                              k_number_nearest_points=a2.k)
        r2 = gnn_measure(a2, world, dev, cfg2, model_state(cfg2, a2.weights), scatter=False)
        line['c2_bf16'] = {'value': round(r2['value'], 2), 'unit': 'frames/s',
                           'ms_per_step': round(r2['ms_step'], 3), 'dtype': 'bf16',
                           'workload': workload_name(a2), 'edges_per_gpu': r2['E'],
                           'forward_only_frames_per_s': round(r2['forward_fps'], 2),
                           'roofline': r2['roof'], 'kernels': r2['kern'], 'clock': r2['clock']}
    if rank == 0 and not args.no_cpu_baseline:  # after the timed region, every world size
        log('cpu baseline')
        cb = cpu_baseline(args, cfg, sd)
        line['cpu_baseline'] = cb
        line['gpu_over_cpu'] = round(line['value'] / cb['value'], 1)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()  # the other ranks wait for rank 0's CPU baseline
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
