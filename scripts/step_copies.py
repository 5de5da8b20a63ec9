"""Which host calls launch the runtime's copy / fill kernels (__amd_rocclr_copyBuffer,
__amd_rocclr_fillBuffer*) inside one bench step (GPU; diagnostic).

Usage: python scripts/step_copies.py [bench args, e.g. --config c5]
Builds the bench workload, warms it, then records two steps under torch.profiler with Python
stacks and prints, per copy / fill kernel, the torch op and the innermost repository frames
that issued it (with counts per step)."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from graph_neural_network_for_radar_perception_amd import _native as nat, synthetic  # noqa: E402
from graph_neural_network_for_radar_perception_amd.config import default_config  # noqa: E402
from graph_neural_network_for_radar_perception_amd.graph_features import FrameBatch  # noqa: E402
from graph_neural_network_for_radar_perception_amd.pipeline import (PipelinedSteps,  # noqa: E402
                                                                     RadarGNNPipeline)

STEPS = 2
# RG_STEPS_ONLY=N: no torch profiler -- warm up, then N plain steps (run under
# rocprofv3 --kernel-trace at two N to count the runtime's copy kernels per step)
ONLY = os.environ.get('RG_STEPS_ONLY')


def main():
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    args = bench.parse()
    dev = torch.device('cuda', 0)
    cfg = default_config(graph_convolution_stem_channels=[64] * args.layers,
                         k_number_nearest_points=args.k)
    model = bench.make_model(cfg, dev, bench.model_state(cfg, args.weights))
    mode = nat.GRAPH_RADIUS if args.graph == 'radius' else nat.GRAPH_KNN
    seeds = bench.rank_frame_seeds(0, args.frames, args.seed)
    frames = [synthetic.make_frame(args.nodes, s) for s in seeds]
    clusters = [synthetic.cluster_lists(args.nodes) for _ in seeds]
    batch = FrameBatch.from_frames(frames, clusters, device=dev)
    if args.streams > 1:
        stepper = PipelinedSteps(model, cfg, args.dtype, mode=mode, eps2=args.eps2,
                                 depth=args.streams)
    else:
        stepper = RadarGNNPipeline(model, cfg, args.dtype, mode=mode, eps2=args.eps2)
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.no_grad():
        for _ in range(max(args.warmup, args.streams)):
            stepper.step(batch)
        torch.cuda.synchronize()
        if ONLY is not None:
            for _ in range(int(ONLY)):
                stepper.step(batch)
            torch.cuda.synchronize()
            print(f'{ONLY} steps done')
            return
        with torch.profiler.profile(activities=acts, with_stack=True) as prof:
            for _ in range(STEPS):
                stepper.step(batch)
            torch.cuda.synchronize()
    kern = collections.Counter()
    sites = collections.Counter()
    for ev in prof.events():
        name = ev.name
        if ev.device_type == torch.autograd.DeviceType.CUDA:
            if 'rocclr' in name or 'Memcpy' in name or 'Memset' in name:
                kern[name] += 1
            continue
        # CPU side: ops whose subtree launched a copy / fill
        kids = [k for k in ev.kernels] if hasattr(ev, 'kernels') else []
        hit = [k for k in kids if 'rocclr' in k.name or 'Memcpy' in k.name or 'Memset' in k.name]
        if not hit or not name.startswith('aten::') and 'hip' not in name.lower():
            continue
        frames_ = [f for f in (ev.stack or []) if 'radar_perception_amd' in f or 'bench.py' in f]
        site = ' <- '.join(frames_[:3]) if frames_ else '(no repository frame)'
        for k in hit:
            sites[(name, k.name[:40], site)] += 1
    print(f'copy / fill kernels per step ({STEPS} steps profiled):')
    for k, n in kern.most_common():
        print(f'  {n / STEPS:6.1f}  {k[:100]}')
    print('issued by (op, kernel, repository frames), per step:')
    for (op, k, site), n in sites.most_common(40):
        print(f'  {n / STEPS:6.1f}  {op} [{k}]  {site}')


if __name__ == '__main__':
    main()
