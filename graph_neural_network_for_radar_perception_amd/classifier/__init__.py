"""Cluster-level classifier GNN (``modules/neural_net/classifier``):
the second consumer of the segmented-aggregate and row-MLP kernels."""
from .classifier import Model_Inference, Model_Training  # noqa: F401
from .engine import compute_edge_index  # noqa: F401
