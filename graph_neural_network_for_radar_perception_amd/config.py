"""Configuration object consumed by the model constructors.

Mirrors ``modules/set_configurations/set_config_gnn.py:10-113`` (class
``config``): attributes read by ``Model_Inference.__init__``
(``modules/neural_net/gnn/gnn_detector.py:37-59``), by the loss
(``modules/neural_net/gnn/loss.py:14-25``) and by the graph builder
(``datagen_gnn.py:67-77``).  ``config(path)`` reads the reference's own YAML
(``configuration_radarscenes_gnn.yml``); ``default_config()`` returns the same
values without a file.
"""
from __future__ import annotations

import math
from typing import Optional

# values of configuration_radarscenes_gnn.yml (line numbers cited per key)
_DEFAULTS = {
    'RANDOM': {'seed': 1234},                                            # yml:2
    'DATA_SELECTION_PARAM': {
        'temporal_window_size': 10,                                      # yml:12
        'ball_query_eps_square': 25,                                     # yml:13
        'k_number_nearest_points': 10,                                   # yml:14
        'reject_static_meas_by_ransac': False,
        'dataset_augmentation': True,
    },
    'DATASET_INFO': {'include_region_confidence': True},                 # yml:29
    'OBJECT_CATEGORIES': {                                               # yml:31-35
        'OBJECT_CLASS': ['CAR', 'PEDESTRIAN', 'PEDESTRIAN_GROUP', 'TWO_WHEELER',
                         'LARGE_VEHICLE', 'NONE', 'FALSE', 'STATIC'],
        'OBJECT_CLASS_WEIGHTS': [1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 0.5, 0.5],
        'OBJECT_CLASS_DYN': ['CAR', 'PEDESTRIAN', 'PEDESTRIAN_GROUP', 'TWO_WHEELER',
                             'LARGE_VEHICLE', 'NONE', 'FALSE'],
        'OBJECT_CLASS_WEIGHTS_DYN': [1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 0.5],
    },
    'GRID_LIMITS': {'max_x': 100, 'min_x': 0, 'max_y': 50, 'min_y': -50,  # yml:37-47
                    'min_sigma_x': 0.5, 'max_sigma_x': 2, 'min_sigma_y': 0.5,
                    'max_sigma_y': 2, 'dx': 0.5, 'dy': 0.5},
    'GNN_ARCHITECTURE': {                                                # yml:46-65
        'node_features': ['vr', 'rcs', 'timestamp', 'node_degree', 'range_conf', 'azi_conf'],
        'edge_features': ['dx', 'dy', 'dl', 'dvx', 'dvy', 'dv', 'dt'],
        'reg_offset': ['dx', 'dy'],
        'activation': 'leakyrelu',
        'normalization': 'channel_normalization',
        'num_groups': None,
        'reg_mu': [0, 0],
        'reg_sigma': [8, 4],
        'aggregation': 'add',
        'node_feat_enc_stem_channels': [256, 128, 64],
        'edge_feat_enc_stem_channels': [256, 128, 128, 64],
        'graph_convolution_stem_channels': [64, 64, 64, 64, 64, 64, 64],
        'msg_mlp_hidden_dim': 128,
        'num_blocks_to_compute_edge': 1,
        'hidden_node_channels_GAT': 512,
        'num_heads_GAT': 8,
        'link_pred_stem_channels': [64, 64, 64],
        'node_pred_stem_channels': [64, 64, 64],
        'num_edge_classes': 2,
    },
    'LOSS_WEIGHTS': {'obj_loss_cls': 1.0, 'node_loss_cls': 1.0,          # yml:67-71
                     'edge_loss_cls': 2.0, 'node_loss_reg': 5.0},
    'OPTIMIZATION': {'optim': 'sgd', 'max_training_iterations': 200000,  # yml:73-77
                     'learning_rate': 0.005, 'weight_decay': 0.0001},
    'FINETUNING': {'optim': 'sgd', 'max_training_iterations': 10000,
                   'learning_rate': 0.0005, 'weight_decay': 0.0001, 'clustering_eps': 1.5},
}


def _labels_to_id(labels):
    return {name: i for i, name in enumerate(labels)}


class config:
    """Flat attribute bag, same attribute names as ``set_config_gnn.config``."""

    def __init__(self, config_filepath: Optional[str] = None, overrides: Optional[dict] = None):
        if config_filepath is not None:
            import yaml
            with open(config_filepath, 'r') as fh:
                c = yaml.safe_load(fh)
        else:
            import copy
            c = copy.deepcopy(_DEFAULTS)
        arch = c['GNN_ARCHITECTURE']
        sel = c['DATA_SELECTION_PARAM']
        grid = c['GRID_LIMITS']
        cats = c['OBJECT_CATEGORIES']
        self.seed = c['RANDOM']['seed']
        self.window_size = sel['temporal_window_size']
        self.ball_query_eps_square = sel['ball_query_eps_square']
        self.k_number_nearest_points = sel['k_number_nearest_points']
        self.min_x, self.max_x = grid['min_x'], grid['max_x']
        self.min_y, self.max_y = grid['min_y'], grid['max_y']
        # set_config_gnn.py:41-44
        self.grid_min_th = 0
        self.grid_min_r = 0
        self.grid_max_th = math.pi * 0.5
        self.grid_max_r = math.sqrt(self.max_x ** 2 + self.max_y ** 2)
        self.node_features = arch['node_features']
        self.edge_features = arch['edge_features']
        self.reg_offset = arch['reg_offset']
        self.activation = arch['activation']
        self.norm_layer = arch['normalization']
        self.num_groups = arch['num_groups']
        self.reg_mu = arch['reg_mu']
        self.reg_sigma = arch['reg_sigma']
        self.aggregation = arch['aggregation']
        self.node_feat_enc_stem_channels = list(arch['node_feat_enc_stem_channels'])
        self.edge_feat_enc_stem_channels = list(arch['edge_feat_enc_stem_channels'])
        self.graph_convolution_stem_channels = list(arch['graph_convolution_stem_channels'])
        self.msg_mlp_hidden_dim = arch['msg_mlp_hidden_dim']
        self.num_blocks_to_compute_edge = arch['num_blocks_to_compute_edge']
        self.link_pred_stem_channels = list(arch['link_pred_stem_channels'])
        self.node_pred_stem_channels = list(arch['node_pred_stem_channels'])
        self.input_node_feat_dim = len(arch['node_features'])
        self.input_edge_feat_dim = len(arch['edge_features'])
        self.num_classes = len(cats['OBJECT_CLASS_DYN'])
        self.reg_offset_dim = len(arch['reg_offset'])
        self.offset_mu = arch['reg_mu']
        self.offset_sigma = arch['reg_sigma']
        self.num_edge_classes = arch['num_edge_classes']
        self.object_classes = cats['OBJECT_CLASS']
        self.class_weights = cats['OBJECT_CLASS_WEIGHTS']
        self.object_classes_dyn = cats['OBJECT_CLASS_DYN']
        self.class_weights_dyn = cats['OBJECT_CLASS_WEIGHTS_DYN']
        lw = c['LOSS_WEIGHTS']
        self.edge_cls_loss_weight = lw['edge_loss_cls']
        self.node_cls_loss_weight = lw['node_loss_cls']
        self.node_reg_loss_weight = lw['node_loss_reg']
        self.obj_cls_loss_weight = lw['obj_loss_cls']
        self.new_labels_to_id_dict_dyn = _labels_to_id(self.object_classes_dyn)
        opt = c['OPTIMIZATION']
        self.optim = opt['optim']
        self.max_train_iter = opt['max_training_iterations']
        self.learning_rate = opt['learning_rate']
        self.weight_decay = opt['weight_decay']
        self.include_region_confidence = c['DATASET_INFO']['include_region_confidence']
        self.clustering_eps = c['FINETUNING']['clustering_eps']
        for k, v in (overrides or {}).items():
            setattr(self, k, v)


def default_config(**overrides) -> config:
    """The yml configuration, with optional attribute overrides
    (e.g. ``graph_convolution_stem_channels=[64]*3`` for BASELINE config 1)."""
    return config(None, overrides)


# values of configuration_radarscenes_classifier.yml (line numbers cited per key)
_CLASSIFIER_DEFAULTS = {
    'CLUSTERING': {'clustering_eps': 1.4, 'valid_cluster_num_meas_thr': 2,   # yml:5-8
                   'meas_noise_var': 1},
    'GNN_ARCHITECTURE': {                                                    # yml:10-18
        'node_features': ['px', 'py', 'r', 'th', 'rcs'],
        'activation': 'leakyrelu',
        'aggregation': 'sum',
        'node_feat_enc_stem_channels': [256, 128, 128],
        'graph_convolution_stem_channels': [128, 128, 128, 128, 128],
        'msg_mlp_hidden_dim': 128,
        'node_pred_stem_channels': [128, 128, 128],
    },
    'OPTIMIZATION': {'optim': 'sgd', 'max_training_iterations': 100000,      # yml:20-24
                     'learning_rate': 0.001, 'weight_decay': 0.0001},
}


class classifier_config(config):
    """``set_config_classifier.config`` (set_config_classifier.py:9-52): the detector
    attributes plus the ``classifier_*`` ones read by classifier/classifier.py:11-20.
    Note the reference's own quirk kept as written: the classifier's OPTIMIZATION values
    overwrite the detector's ``optim`` / ``learning_rate`` / ``weight_decay``."""

    def __init__(self, config_gnn_filepath: Optional[str] = None,
                 config_classifier_filepath: Optional[str] = None,
                 overrides: Optional[dict] = None):
        super().__init__(config_gnn_filepath)
        if config_classifier_filepath is not None:
            import yaml
            with open(config_classifier_filepath, 'r') as fh:
                c = yaml.safe_load(fh)
        else:
            import copy
            c = copy.deepcopy(_CLASSIFIER_DEFAULTS)
        cl = c['CLUSTERING']
        self.clustering_eps = cl['clustering_eps']
        self.valid_cluster_num_meas_thr = cl['valid_cluster_num_meas_thr']
        import numpy as np
        self.meas_noise_cov = cl['meas_noise_var'] * np.eye(2, dtype=np.float32)
        a = c['GNN_ARCHITECTURE']
        self.classifier_node_features = list(a['node_features'])
        self.classifier_input_node_feat_dim = len(a['node_features'])
        self.classifier_activation = a['activation']
        self.classifier_aggregation = a['aggregation']
        self.classifier_node_feat_enc_stem_channels = list(a['node_feat_enc_stem_channels'])
        self.classifier_graph_convolution_stem_channels = list(a['graph_convolution_stem_channels'])
        self.classifier_msg_mlp_hidden_dim = a['msg_mlp_hidden_dim']
        self.classifier_node_pred_stem_channels = list(a['node_pred_stem_channels'])
        o = c['OPTIMIZATION']
        self.optim = o['optim']
        self.max_train_iter = o['max_training_iterations']
        self.learning_rate = o['learning_rate']
        self.weight_decay = o['weight_decay']
        for k, v in (overrides or {}).items():
            setattr(self, k, v)


def default_classifier_config(**overrides) -> classifier_config:
    """The classifier yml configuration (on top of the detector yml), with overrides."""
    return classifier_config(None, None, overrides)
