"""kNN graph-build timing experiments (RG_KNN_EXP variants, wrong results by
construction): builds lib/variants/libradargnn_knn_<name>.so and, with --run, times
engine.build_graph on the BASELINE config-2 batch for each (HIP events, median of 20)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
EXPS = {'thread': ['RG_KNN_COOP=0'], 'cl16': ['RG_KNN_CL=16'], 'cl8': ['RG_KNN_CL=8'],
        'cl32': ['RG_KNN_CL=32'], 'cap64': ['RG_KNN_CAP=64'], 'cap128': ['RG_KNN_CAP=128'],
        'cap192': ['RG_KNN_CAP=192'], 'histonly': ['RG_KNN_COOP=0', 'RG_KNN_EXP=2']}


def time_one(frames=64, nodes=3000, k=int(os.environ.get('RG_EXP_K', 32))):
    import numpy as np
    import torch
    from graph_neural_network_for_radar_perception_amd import engine, synthetic
    dev = torch.device('cuda', 0)
    frs = [synthetic.make_frame(nodes, 1234 + i) for i in range(frames)]
    px = torch.from_numpy(np.concatenate([f['meas_px'] for f in frs])).to(dev)
    py = torch.from_numpy(np.concatenate([f['meas_py'] for f in frs])).to(dev)
    fptr = torch.tensor(np.arange(frames + 1) * nodes, dtype=torch.int32).to(dev)
    cache = {}
    ts = []
    for it in range(25):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        engine.build_graph(px, py, fptr, [nodes] * frames, k, float(os.environ.get('RG_EXP_EPS2', 25.0)),
                           ws_cache=cache)
        b.record()
        torch.cuda.synchronize()
        if it >= 5:
            ts.append(a.elapsed_time(b))
    print(f'{os.environ.get("RG_EXP_NAME", "?"):10s} build_graph {np.median(ts):.4f} ms', flush=True)


def main():
    if '--one' in sys.argv:
        time_one()
        return
    from graph_neural_network_for_radar_perception_amd import build
    sel = [a for a in sys.argv[1:] if not a.startswith('--')]
    exps = {k: v for k, v in EXPS.items() if not sel or k in sel[0].split(',')}
    if '--run' not in sys.argv:
        for name, v in exps.items():
            print(build.build_variant(f'knn_{name}', v, only=['graph_build.hip']))
        return
    for name in exps:
        lib = os.path.join(REPO, 'graph_neural_network_for_radar_perception_amd', 'lib', 'variants',
                           f'libradargnn_knn_{name}.so')
        env = dict(os.environ, RG_LIBRARY=lib, RG_EXP_NAME=name)
        r = subprocess.run([sys.executable, __file__, '--one'], env=env, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == '__main__':
    main()
