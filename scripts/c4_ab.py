"""A/B of training-step switches on the c4 bench:
python scripts/c4_ab.py NAME=0|1[,NAME=0|1...] [bench.py args...]
(NAME: a module-level flag of training.py, e.g. GATHERED_DMSG, FACTORED_MSG0)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from graph_neural_network_for_radar_perception_amd import training  # noqa: E402

for kv in sys.argv[1].split(','):
    k, v = kv.split('=')
    if not hasattr(training, k):
        raise SystemExit(f'training has no flag {k}')
    setattr(training, k, v == '1')
sys.argv = [os.path.join(REPO, 'bench.py')] + sys.argv[2:]
import bench  # noqa: E402

bench.main()
