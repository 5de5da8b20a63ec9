"""Build the fused-conv timing experiments (RG_CONV_EXP variants) and, with --run, time
each with bench.py (RG_LIBRARY=<variant>).  Results are wrong by construction; only
kernels.conv_fused.avg_ms is read."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
EXPS_ALL = {'base': ['RG_CONV_EXP=0'], 'nogather': ['RG_CONV_EXP=1'], 'nonorm': ['RG_CONV_EXP=2'],
        'noagg': ['RG_CONV_EXP=3'], 'ct256': ['RG_CONV_CT=256'], 'prio': ['RG_CONV_PRIO=1'],
        'chain_noepi': ['RG_CHAIN_EXP=1'], 'chain_nomfma': ['RG_CHAIN_EXP=2'],
        'chain_nolds': ['RG_CHAIN_EXP=3'],
        'scalar': ['RG_NO_PK', '-fno-slp-vectorize'], 'nosplit': ['RG_PAIR_SPLIT=0'], 'pfx': ['RG_CONV_PFX=1'], 'noP': ['RG_CONV_EXP=4'], 'pfd4': ['RG_CONV_PFD4=2'],
        'pfd4b': ['RG_CONV_PFD4=2', 'RG_CONV_PFD=2']}
EXPS = {k: v for k, v in EXPS_ALL.items()
        if len(sys.argv) < 3 or k in sys.argv[2].split(',') or k == 'base'}


def main():
    from graph_neural_network_for_radar_perception_amd import build
    if '--run' not in sys.argv:
        for name, v in EXPS.items():
            print(build.build_variant(f'conv_{name}', v, only=['conv_fused.hip', 'chain_fast.hip']))
        return
    for name in EXPS:
        lib = os.path.join(REPO, 'graph_neural_network_for_radar_perception_amd', 'lib', 'variants',
                           f'libradargnn_conv_{name}.so')
        env = dict(os.environ, RG_LIBRARY=lib)
        r = subprocess.run([sys.executable, 'bench.py', '--steps', '5', '--warmup', '1',
                            '--no-cpu-baseline'], cwd=REPO, env=env, capture_output=True,
                           text=True, timeout=600)
        line = [x for x in r.stdout.splitlines() if x.startswith('{')]
        if r.returncode != 0 or not line:
            print(name, 'FAILED', r.returncode, r.stderr[-2000:])
            sys.exit(1)
        d = json.loads(line[-1])
        print(f"{name:12s} conv_fused {d['kernels']['conv_fused']['avg_ms']:.4f} ms  "
              f"edge_encoder {d['kernels']['edge_encoder']['avg_ms']:.4f} ms  "
              f"step {d['ms_per_step']:.3f} ms", flush=True)


if __name__ == '__main__':
    main()
