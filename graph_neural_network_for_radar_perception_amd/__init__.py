"""MI355X-native radar point-cloud GNN (forward hot path of
UditBhaskar19/GRAPH_NEURAL_NETWORK_FOR_RADAR_PERCEPTION) on hand-written HIP kernels.

Drop-in entry points (same names / signatures as the reference):
  gnn_detector.Model_Inference, gnn_detector.Model_Training,
  gnn_detector.Model_Object_Classifier_Finetuning              (gnn_detector.py)
  loss.Loss_Graph, loss.Loss_Object_Class                      (loss.py)
  gnn_blocks.*, common.*                                       (gnn_blocks.py, common.py)
  graph_features.compute_adjacency_information / _v2,
  compute_node_features, compute_edge_features                 (graph_features.py)
  config.config                                                (set_config_gnn.py)
Batched device path: graph_features.FrameBatch / build_graph_batch,
pipeline.RadarGNNPipeline.
"""
from . import config, synthetic  # noqa: F401

__version__ = '0.1.0'


def native_available() -> bool:
    """True when libradargnn.so is built and loads."""
    from . import _native
    try:
        _native.lib()
        return True
    except _native.NativeLibraryError:
        return False
