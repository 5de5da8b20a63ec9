"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Runs only in the build container, where /root/reference exists (it never runs on
the GPU box; nothing in tests/ imports this file).  It imports the reference's
own modules and records their outputs on seeded synthetic frames:

  * graph build: ``modules/compute_features/graph_features.py`` imports with
    numpy only -- these fixtures are produced by the unmodified reference code.
  * model forward: ``modules/neural_net/gnn/gnn_detector.py`` imports two
    third-party packages that are NOT installed here (no network):
      - ``torch_geometric`` (>= 2.5.0, README.md:156; no lockfile) for
        ``MessagePassing`` (call sites gnn_blocks.py:8,57,106,112);
      - ``torchvision`` for ``ops.sigmoid_focal_loss`` (lossfunc.py:5,55),
        training-only.
    For these two, ``_install_third_party_restatements`` registers in-memory
    modules that restate their PUBLISHED algorithms (PyG 2.5
    ``MessagePassing.propagate`` with ``flow='source_to_target'``:
    x_i = x[edge_index[1]], x_j = x[edge_index[0]], aggregate at
    edge_index[1] with ``scatter_add_`` / mean / ``scatter_reduce_(amax,
    include_self=False)``; torchvision ``sigmoid_focal_loss``).  Everything
    else executed is the reference's own code.  Parity for the PyG part is
    therefore anchored on its published semantics, not on a pinned run of PyG
    ("parity unpinned" for that part).

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from graph_neural_network_for_radar_perception_amd import synthetic  # noqa: E402

CKPT = os.path.join(REF, 'model_weights/gnn/1718175257362/graph_based_detector.pt')


def _install_third_party_restatements():
    """In-memory restatement of the two absent third-party APIs (see module doc)."""
    class MessagePassing(torch.nn.Module):
        def __init__(self, aggr='add', flow='source_to_target', **kwargs):
            super().__init__()
            self.aggr = aggr
            self.flow = flow

        def propagate(self, edge_index, size=None, **kwargs):
            x = kwargs['x']
            i, j = (1, 0) if self.flow == 'source_to_target' else (0, 1)
            x_i = x.index_select(0, edge_index[i])
            x_j = x.index_select(0, edge_index[j])
            # PyG passes message() only the arguments its signature names
            import inspect
            names = inspect.signature(self.message).parameters
            args = {'x_i': x_i, 'x_j': x_j, 'edge_attr': kwargs.get('edge_attr')}
            msg = self.message(**{k: v for k, v in args.items() if k in names})
            n = x.shape[0]
            idx = edge_index[i].view(-1, 1).expand_as(msg)
            if self.aggr in ('add', 'sum'):
                out = msg.new_zeros((n, msg.shape[1])).scatter_add_(0, idx, msg)
            elif self.aggr == 'mean':
                out = msg.new_zeros((n, msg.shape[1])).scatter_add_(0, idx, msg)
                cnt = msg.new_zeros((n,)).scatter_add_(0, edge_index[i], msg.new_ones((msg.shape[0],)))
                out = out / cnt.clamp(min=1).view(-1, 1)
            elif self.aggr == 'max':
                out = msg.new_zeros((n, msg.shape[1])).scatter_reduce_(
                    0, idx, msg, reduce='amax', include_self=False)
            else:
                raise ValueError(self.aggr)
            return out

    class GATv2Conv(torch.nn.Module):  # gnn_attention.py:9 -- unused variant
        def __init__(self, *a, **k):
            raise NotImplementedError('GATv2Conv is not restated (unused by the reference)')

    def sigmoid_focal_loss(inputs, targets, alpha=0.25, gamma=2.0, reduction='none'):
        p = torch.sigmoid(inputs)
        ce = F.binary_cross_entropy_with_logits(inputs, targets, reduction='none')
        p_t = p * targets + (1 - p) * (1 - targets)
        loss = ce * ((1 - p_t) ** gamma)
        if alpha >= 0:
            loss = (alpha * targets + (1 - alpha) * (1 - targets)) * loss
        if reduction == 'mean':
            return loss.mean()
        if reduction == 'sum':
            return loss.sum()
        return loss

    pyg = types.ModuleType('torch_geometric')
    pyg_nn = types.ModuleType('torch_geometric.nn')
    pyg_conv = types.ModuleType('torch_geometric.nn.conv')
    pyg_conv.MessagePassing = MessagePassing
    pyg_conv.GATv2Conv = GATv2Conv
    pyg_nn.conv = pyg_conv
    pyg_nn.GATv2Conv = GATv2Conv
    pyg.nn = pyg_nn
    tv = types.ModuleType('torchvision')
    tv_ops = types.ModuleType('torchvision.ops')
    tv_ops.sigmoid_focal_loss = sigmoid_focal_loss
    tv.ops = tv_ops
    sys.modules.update({'torch_geometric': pyg, 'torch_geometric.nn': pyg_nn,
                        'torch_geometric.nn.conv': pyg_conv,
                        'torchvision': tv, 'torchvision.ops': tv_ops})


def _ref_graph(frame, eps, knn):
    from modules.compute_features.graph_features import (
        compute_adjacency_information, compute_node_features, compute_edge_features)
    from modules.set_configurations.set_config_gnn import config
    cfg = config(os.path.join(REF, 'configuration_radarscenes_gnn.yml'))
    adj = compute_adjacency_information(frame, eps, knn)
    ef = compute_edge_features(frame, adj['adj_list'])
    nf = compute_node_features(frame, adj['degree'], include_region_confidence=True,
                               min_range=cfg.grid_min_r, max_range=cfg.grid_max_r,
                               min_azimuth=cfg.grid_min_th, max_azimuth=cfg.grid_max_th)
    return adj, nf, ef


def _frame_arrays(frame):
    return {k: frame[k] for k in ('meas_px', 'meas_py', 'meas_vx', 'meas_vy',
                                  'meas_vr', 'meas_rcs', 'meas_timestamp')}


def make_graph_fixtures():
    cases = [(2, 10, 25.0), (8, 10, 25.0), (11, 10, 25.0), (12, 10, 25.0), (50, 10, 25.0),
             (500, 16, 25.0), (1000, 32, 25.0), (3000, 10, 25.0), (300, 8, 4.0)]
    for n, k, eps in cases:
        seed = synthetic.SEED0 + 7 * n + k
        fr = synthetic.make_frame(n, seed)
        adj, nf, ef = _ref_graph(fr, eps, k)
        out = dict(_frame_arrays(fr))
        out.update(n=n, k=k, eps=eps, seed=seed,
                   adj_list=adj['adj_list'].astype(np.int32),
                   degree=adj['degree'].astype(np.int32),
                   node_features=nf.astype(np.float32),
                   node_features_f64=nf,
                   edge_features=ef.astype(np.float32))
        np.savez_compressed(os.path.join(HERE, f'graph_N{n}_k{k}.npz'), **out)
        print('graph', n, k, adj['adj_list'].shape)
    # tie lattice: distances tie massively; numpy's default argsort is unstable,
    # so the reference's neighbour choice at ties is implementation-defined.
    from modules.compute_features.graph_features import compute_adjacency_information, compute_ball_query
    fr = synthetic.make_frame(400, 99, lattice=True)
    adj = compute_adjacency_information(fr, 25.0, 10)
    np.savez_compressed(os.path.join(HERE, 'graph_lattice_N400_k10.npz'),
                        **_frame_arrays(fr), n=400, k=10, eps=25.0,
                        adj_list=adj['adj_list'].astype(np.int32),
                        degree=adj['degree'].astype(np.int32))
    # pure radius graph (compute_ball_query semantics; BASELINE config 5 shape, small)
    fr = synthetic.make_frame(2000, 4242)
    pxy = np.stack((fr['meas_px'], fr['meas_py']), axis=-1)
    d = np.expand_dims(pxy[:, None, :] - pxy[None, :, :], -1)
    dist = (d.transpose(0, 1, 3, 2) @ d).squeeze(-1).squeeze(-1)
    gated = compute_ball_query(dist, 2.5)
    np.savez_compressed(os.path.join(HERE, 'graph_radius_N2000.npz'),
                        **_frame_arrays(fr), n=2000, eps=2.5,
                        adj_list=np.stack(np.where(gated), 0).astype(np.int32))
    print('lattice/radius done')


def _model(cfg, seed=None, ckpt=None):
    from modules.neural_net.gnn.gnn_detector import Model_Training
    if seed is not None:
        torch.manual_seed(seed)
    m = Model_Training(cfg, 'cpu')
    if ckpt is not None:
        sd = torch.load(ckpt, map_location='cpu', weights_only=True)
        m.load_state_dict(sd)
    return m.eval()


def _forward_case(name, cfg, n, k, seed_frame, model_seed=None, ckpt=None,
                  save_weights=False, intermediates=False):
    fr = synthetic.make_frame(n, seed_frame)
    adj, nf, ef = _ref_graph(fr, cfg.ball_query_eps_square, k)
    model = _model(cfg, seed=model_seed, ckpt=ckpt)
    clusters = synthetic.cluster_lists(n)
    node_t = torch.from_numpy(nf).to(torch.float32)
    edge_t = torch.from_numpy(ef).to(torch.float32)
    ei_t = torch.from_numpy(adj['adj_list']).to(torch.int64)
    adj_t = torch.from_numpy(adj['adj_matrix']).to(torch.bool)
    cl_t = [torch.from_numpy(c) for c in clusters]
    inter = {}
    hooks = []
    if intermediates:
        p = model.pred
        hooks.append(p.encode_node_feat.register_forward_hook(
            lambda m, i, o: inter.__setitem__('x_enc', o.detach().numpy().copy())))
        hooks.append(p.encode_edge_feat.register_forward_hook(
            lambda m, i, o: inter.__setitem__('e_enc', o.detach().numpy().copy())))
        for li, blk in enumerate(p.pass_messages.conv_blk):
            hooks.append(blk.register_forward_hook(
                (lambda li_: lambda m, i, o: inter.__setitem__(f'x_l{li_}', o.detach().numpy().copy()))(li)))
    with torch.no_grad():
        outs = model.pred(node_t, edge_t, ei_t, adj_t, cl_t)
    for h in hooks:
        h.remove()
    sd = model.state_dict()
    fp = {('fp/' + k): np.array([v.double().sum().item(), v.double().abs().sum().item()])
          for k, v in sd.items()}
    data = dict(_frame_arrays(fr))
    data.update(n=n, k=k, eps=float(cfg.ball_query_eps_square), frame_seed=seed_frame,
                L=len(cfg.graph_convolution_stem_channels), aggregation=cfg.aggregation,
                model_seed=-1 if model_seed is None else model_seed,
                node_features=nf.astype(np.float32), edge_features=ef.astype(np.float32),
                edge_index=adj['adj_list'].astype(np.int32),
                cluster_ptr=np.cumsum([0] + [len(c) for c in clusters]).astype(np.int64),
                cluster_idx=np.concatenate(clusters).astype(np.int64),
                node_cls=outs[0].numpy(), node_reg=outs[1].numpy(),
                link_cls=outs[2].numpy(), obj_cls=outs[3].numpy(), **fp)
    for k_, v in inter.items():
        data['inter/' + k_] = v
    if save_weights:
        for k_, v in sd.items():
            data['w/' + k_] = v.numpy()
    np.savez_compressed(os.path.join(HERE, name + '.npz'), **data)
    print('model', name, 'E', adj['adj_list'].shape[1], 'U', outs[2].shape[0])


def make_model_fixtures():
    from modules.set_configurations.set_config_gnn import config
    ycfg = os.path.join(REF, 'configuration_radarscenes_gnn.yml')
    # trained checkpoint (metric shape M uses it), yml architecture, k=10
    cfg = config(ycfg)
    _forward_case('model_trained_N50', cfg, 50, 10, 5001, ckpt=CKPT,
                  save_weights=True, intermediates=True)
    _forward_case('model_trained_N500', cfg, 500, 10, 5002, ckpt=CKPT)
    # BASELINE config 1: N=500, k=16, L=3, random init torch.manual_seed(1234)
    cfg = config(ycfg)
    cfg.graph_convolution_stem_channels = [64, 64, 64]
    cfg.k_number_nearest_points = 16
    _forward_case('model_random_L3_N500_k16', cfg, 500, 16, 5003, model_seed=1234)
    # config 2 per-frame structure (k=32, L=6) at a small N
    cfg = config(ycfg)
    cfg.graph_convolution_stem_channels = [64] * 6
    _forward_case('model_random_L6_N300_k32', cfg, 300, 32, 5004, model_seed=4321)
    # other PyG aggregations (restated semantics; parity unpinned)
    for aggr in ('mean', 'max'):
        cfg = config(ycfg)
        cfg.graph_convolution_stem_channels = [64, 64]
        cfg.aggregation = aggr
        _forward_case(f'model_random_{aggr}_N200', cfg, 200, 10, 5005, model_seed=77,
                      intermediates=True)
    # mixed widths: residual_connection path (gnn_blocks.py:84-94) + non-default widths
    cfg = config(ycfg)
    cfg.node_feat_enc_stem_channels = [128, 96]
    cfg.edge_feat_enc_stem_channels = [64, 32]
    cfg.graph_convolution_stem_channels = [64, 32]
    cfg.msg_mlp_hidden_dim = 96
    cfg.link_pred_stem_channels = [32, 32]
    cfg.node_pred_stem_channels = [32, 64]
    cfg.num_blocks_to_compute_edge = 2
    _forward_case('model_random_widths_N120', cfg, 120, 10, 5006, model_seed=99,
                  save_weights=True, intermediates=True)


def make_proposal_fixtures():
    """Simple_DBSCAN (clustering.py:43-93) on predicted centres, both adjacency modes,
    and the full proposal branch of Model_Inference (gnn_detector.py:164-195)."""
    from modules.inference.clustering import Simple_DBSCAN
    from modules.compute_groundtruth.compute_offsets import unnormalize_gt_offsets
    from modules.compute_features.graph_features import compute_adjacency_information
    from modules.set_configurations.set_config_gnn import config
    cfg = config(os.path.join(REF, 'configuration_radarscenes_gnn.yml'))
    mu, sigma, eps = cfg.reg_mu, cfg.reg_sigma, float(cfg.clustering_eps)
    for n, seed in ((400, 6001), (1500, 6002)):
        fr = synthetic.make_frame(n, seed)
        rng = np.random.default_rng(seed)
        offsets = rng.normal(0.0, 0.15, (n, 2)).astype(np.float32)
        other_xy = np.stack([fr['meas_px'], fr['meas_py']], -1).astype(np.float32)
        deltas = unnormalize_gt_offsets(torch.from_numpy(offsets).clone(), mu, sigma)
        centres = (torch.from_numpy(other_xy) + deltas).numpy()
        db = Simple_DBSCAN(eps)
        db.cluster_nodes(centres)
        ids_off = db.meas_to_cluster_id.astype(np.int64)
        adj = compute_adjacency_information(fr, 25.0, 10)
        r, c = np.nonzero(np.triu(adj['adj_matrix'], k=1))
        pred_edges = (rng.random(r.shape[0]) < 0.6).astype(np.int64)
        db2 = Simple_DBSCAN(eps, compute_adj_mat_from_links=True)
        db2.cluster_nodes(centres, pred_edges.copy(), adj['adj_matrix'])
        ids_links = db2.meas_to_cluster_id.astype(np.int64)
        np.savez_compressed(os.path.join(HERE, f'proposals_dbscan_N{n}.npz'),
                            other_xy=other_xy, offsets=offsets, mu=np.array(mu, np.float64),
                            sigma=np.array(sigma, np.float64), eps=eps, centres=centres,
                            ids_offsets=ids_off, ids_links=ids_links, pred_edges=pred_edges,
                            adj_list=adj['adj_list'].astype(np.int32))
        print('proposals', n, 'clusters', ids_off.max() + 1, ids_links.max() + 1)
    # full branch with the trained checkpoint
    n, k = 300, 10
    fr = synthetic.make_frame(n, 5007)
    adj, nf, ef = _ref_graph(fr, cfg.ball_query_eps_square, k)
    model = _model(cfg, ckpt=CKPT)
    other = np.stack([fr['meas_px'], fr['meas_py'], fr['meas_vx'], fr['meas_vy']], -1).astype(np.float32)
    data = dict(_frame_arrays(fr))
    data.update(n=n, k=k, eps_graph=float(cfg.ball_query_eps_square), eps=eps,
                node_features=nf.astype(np.float32), edge_features=ef.astype(np.float32),
                edge_index=adj['adj_list'].astype(np.int32), other_features=other)
    for tag, links in (('off', False), ('links', True)):
        model.pred.set_param_for_proposal_extraction(eps, links)
        with torch.no_grad():
            outs = model.pred(torch.from_numpy(nf).float(), torch.from_numpy(ef).float(),
                              torch.from_numpy(adj['adj_list']).long(),
                              torch.from_numpy(adj['adj_matrix']), None,
                              other_features=torch.from_numpy(other))
        cl = outs[4]
        data.update({f'{tag}/node_cls': outs[0].numpy(), f'{tag}/node_reg': outs[1].numpy(),
                     f'{tag}/link_cls': outs[2].numpy(), f'{tag}/obj_cls': outs[3].numpy(),
                     f'{tag}/cluster_ptr': np.cumsum([0] + [len(c) for c in cl]).astype(np.int64),
                     f'{tag}/cluster_idx': np.concatenate([c.numpy() for c in cl]).astype(np.int64)})
        print('model proposals', tag, 'clusters', len(cl))
    for k_, v in model.state_dict().items():
        data['w/' + k_] = v.numpy()
    np.savez_compressed(os.path.join(HERE, 'proposals_model_trained_N300.npz'), **data)


def make_training_fixtures():
    """Model_Training.forward + Loss_Graph (loss.py:37-76) + backward + two
    torch.optim.SGD steps (set_param_for_training_gnn.py:44-46: momentum 0.9, lr and
    weight decay from the yml) on a 2-frame batch with synthetic labels
    (synthetic.make_labels) -- the reference's own training step (training.py:66-85)."""
    from modules.set_configurations.set_config_gnn import config
    from modules.neural_net.gnn.gnn_detector import Model_Training
    cfg = config(os.path.join(REF, 'configuration_radarscenes_gnn.yml'))
    sizes, seeds = (160, 100), (7001, 7002)
    frames, graphs, labels = [], [], []
    for n, sd_ in zip(sizes, seeds):
        fr = synthetic.make_frame(n, sd_)
        adj, nf, ef = _ref_graph(fr, cfg.ball_query_eps_square, cfg.k_number_nearest_points)
        frames.append(fr)
        graphs.append((adj, nf, ef))
        labels.append(synthetic.make_labels(fr, adj['adj_list'], cfg.num_classes, sd_))
    torch.manual_seed(2024)
    model = Model_Training(cfg, 'cpu')
    init = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    params = [p for p in model.parameters() if p.requires_grad]
    opt = torch.optim.SGD(params, momentum=0.9, lr=cfg.learning_rate, weight_decay=cfg.weight_decay)
    lab = {'node_class': [torch.from_numpy(l['node_class']) for l in labels],
           'node_offsets': [torch.from_numpy(l['node_offsets']) for l in labels],
           'edge_class': [torch.from_numpy(l['edge_class']) for l in labels],
           'cluster_node_idx': [[torch.from_numpy(c) for c in l['cluster_node_idx']] for l in labels],
           'cluster_labels': [torch.from_numpy(l['cluster_labels']) for l in labels]}
    args = dict(node_features=[torch.from_numpy(g[1]).float() for g in graphs],
                edge_features=[torch.from_numpy(g[2]).float() for g in graphs],
                edge_index=[torch.from_numpy(g[0]['adj_list']).long() for g in graphs],
                adj_matrix=[torch.from_numpy(g[0]['adj_matrix']) for g in graphs])
    data = {}
    model.train()
    for step in (1, 2):
        loss, acc = model(labels=lab, **args)
        total = loss['loss_node_cls'] + loss['loss_node_reg'] + loss['loss_edge_cls'] + loss['loss_obj_cls']
        total.backward()
        for k_, v in loss.items():
            data[f's{step}/{k_}'] = np.float64(v.item())
        for k_, v in acc.items():
            data[f's{step}/{k_}'] = np.float64(float(v))
        if step == 1:
            for name, p in model.named_parameters():
                data['g1/' + name] = p.grad.detach().numpy().copy()
        opt.step()
        opt.zero_grad()
    for k_, v in model.state_dict().items():
        data['w2/' + k_] = v.numpy()
    for k_, v in init.items():
        data['w/' + k_] = v
    for f, (fr, g, l) in enumerate(zip(frames, graphs, labels)):
        for k_, v in _frame_arrays(fr).items():
            data[f'f{f}/{k_}'] = v
        data[f'f{f}/node_features'] = g[1].astype(np.float32)
        data[f'f{f}/edge_features'] = g[2].astype(np.float32)
        data[f'f{f}/edge_index'] = g[0]['adj_list'].astype(np.int32)
        data[f'f{f}/node_class'] = l['node_class']
        data[f'f{f}/node_offsets'] = l['node_offsets']
        data[f'f{f}/edge_class'] = l['edge_class']
        data[f'f{f}/cluster_ptr'] = np.cumsum([0] + [len(c) for c in l['cluster_node_idx']]).astype(np.int64)
        data[f'f{f}/cluster_idx'] = np.concatenate(l['cluster_node_idx']).astype(np.int64)
        data[f'f{f}/cluster_labels'] = l['cluster_labels']
    data.update(n_frames=len(sizes), lr=cfg.learning_rate, weight_decay=cfg.weight_decay,
                momentum=0.9)
    np.savez_compressed(os.path.join(HERE, 'train_yml_2frames.npz'), **data)
    print('training', {k: v for k, v in data.items() if k.startswith('s')})


def make_norm_fixtures():
    """layer_normalization / group_normalization (common.py:223-253; normalization is a
    yml choice, configuration_radarscenes_gnn.yml:51-52): the reference's Model_Inference
    forward frame by frame (its statistics run over a whole frame's rows: nodes, edges,
    pairs or clusters) and one Model_Training step (loss.backward()) on a 2-frame batch."""
    from modules.set_configurations.set_config_gnn import config
    from modules.neural_net.gnn.gnn_detector import Model_Training
    for norm, groups in (('layer_normalization', None), ('group_normalization', 4)):
        cfg = config(os.path.join(REF, 'configuration_radarscenes_gnn.yml'))
        cfg.norm_layer = norm
        cfg.num_groups = groups
        cfg.graph_convolution_stem_channels = [64, 64]
        sizes, seeds = (120, 90), (9101, 9102)
        torch.manual_seed(31)
        model = Model_Training(cfg, 'cpu')
        frames, graphs, labels = [], [], []
        data = {}
        for f, (n, sd_) in enumerate(zip(sizes, seeds)):
            fr = synthetic.make_frame(n, sd_)
            adj, nf, ef = _ref_graph(fr, cfg.ball_query_eps_square, cfg.k_number_nearest_points)
            lb = synthetic.make_labels(fr, adj['adj_list'], cfg.num_classes, sd_)
            frames.append(fr)
            graphs.append((adj, nf, ef))
            labels.append(lb)
            model.eval()
            with torch.no_grad():
                outs = model.pred(torch.from_numpy(nf).float(), torch.from_numpy(ef).float(),
                                  torch.from_numpy(adj['adj_list']).long(),
                                  torch.from_numpy(adj['adj_matrix']),
                                  [torch.from_numpy(c) for c in lb['cluster_node_idx']])
            for key, v in zip(('node_cls', 'node_reg', 'link_cls', 'obj_cls'), outs):
                data[f'f{f}/{key}'] = v.numpy()
            data[f'f{f}/node_features'] = nf.astype(np.float32)
            data[f'f{f}/edge_features'] = ef.astype(np.float32)
            data[f'f{f}/edge_index'] = adj['adj_list'].astype(np.int32)
            data[f'f{f}/node_class'] = lb['node_class']
            data[f'f{f}/node_offsets'] = lb['node_offsets']
            data[f'f{f}/edge_class'] = lb['edge_class']
            data[f'f{f}/cluster_ptr'] = np.cumsum([0] + [len(c) for c in lb['cluster_node_idx']]).astype(np.int64)
            data[f'f{f}/cluster_idx'] = np.concatenate(lb['cluster_node_idx']).astype(np.int64)
            data[f'f{f}/cluster_labels'] = lb['cluster_labels']
        for k_, v in model.state_dict().items():
            data['w/' + k_] = v.numpy()
        lab = {'node_class': [torch.from_numpy(l['node_class']) for l in labels],
               'node_offsets': [torch.from_numpy(l['node_offsets']) for l in labels],
               'edge_class': [torch.from_numpy(l['edge_class']) for l in labels],
               'cluster_node_idx': [[torch.from_numpy(c) for c in l['cluster_node_idx']] for l in labels],
               'cluster_labels': [torch.from_numpy(l['cluster_labels']) for l in labels]}
        model.train()
        loss, acc = model(node_features=[torch.from_numpy(g[1]).float() for g in graphs],
                          edge_features=[torch.from_numpy(g[2]).float() for g in graphs],
                          edge_index=[torch.from_numpy(g[0]['adj_list']).long() for g in graphs],
                          adj_matrix=[torch.from_numpy(g[0]['adj_matrix']) for g in graphs],
                          labels=lab)
        total = loss['loss_node_cls'] + loss['loss_node_reg'] + loss['loss_edge_cls'] + loss['loss_obj_cls']
        total.backward()
        for k_, v in loss.items():
            data[f's1/{k_}'] = np.float64(v.item())
        for name, p_ in model.named_parameters():
            data['g1/' + name] = p_.grad.detach().numpy().copy()
        data.update(n_frames=len(sizes), norm_layer=norm, num_groups=-1 if groups is None else groups,
                    L=2)
        tag = 'layer' if norm == 'layer_normalization' else 'group'
        np.savez_compressed(os.path.join(HERE, f'norm_{tag}_2frames.npz'), **data)
        print('norm', norm, {k: v for k, v in data.items() if k.startswith('s1')})


def make_max_training_fixture():
    """Training with aggregation 'max' (gnn_blocks.py:57: MessagePassing(aggr=cfg.aggregation)
    trains any aggregation through autograd): the reference's Model_Training, 2 conv blocks,
    one loss.backward() on a 2-frame batch -> losses and every parameter gradient."""
    from modules.set_configurations.set_config_gnn import config
    from modules.neural_net.gnn.gnn_detector import Model_Training
    cfg = config(os.path.join(REF, 'configuration_radarscenes_gnn.yml'))
    cfg.aggregation = 'max'
    cfg.graph_convolution_stem_channels = [64, 64]
    sizes, seeds = (150, 110), (9201, 9202)
    torch.manual_seed(41)
    model = Model_Training(cfg, 'cpu')
    data, graphs, labels = {}, [], []
    for f, (n, sd_) in enumerate(zip(sizes, seeds)):
        fr = synthetic.make_frame(n, sd_)
        adj, nf, ef = _ref_graph(fr, cfg.ball_query_eps_square, cfg.k_number_nearest_points)
        lb = synthetic.make_labels(fr, adj['adj_list'], cfg.num_classes, sd_)
        graphs.append((adj, nf, ef))
        labels.append(lb)
        data[f'f{f}/node_features'] = nf.astype(np.float32)
        data[f'f{f}/edge_features'] = ef.astype(np.float32)
        data[f'f{f}/edge_index'] = adj['adj_list'].astype(np.int32)
        data[f'f{f}/node_class'] = lb['node_class']
        data[f'f{f}/node_offsets'] = lb['node_offsets']
        data[f'f{f}/edge_class'] = lb['edge_class']
        data[f'f{f}/cluster_ptr'] = np.cumsum([0] + [len(c) for c in lb['cluster_node_idx']]).astype(np.int64)
        data[f'f{f}/cluster_idx'] = np.concatenate(lb['cluster_node_idx']).astype(np.int64)
        data[f'f{f}/cluster_labels'] = lb['cluster_labels']
    for k_, v in model.state_dict().items():
        data['w/' + k_] = v.numpy()
    lab = {'node_class': [torch.from_numpy(l['node_class']) for l in labels],
           'node_offsets': [torch.from_numpy(l['node_offsets']) for l in labels],
           'edge_class': [torch.from_numpy(l['edge_class']) for l in labels],
           'cluster_node_idx': [[torch.from_numpy(c) for c in l['cluster_node_idx']] for l in labels],
           'cluster_labels': [torch.from_numpy(l['cluster_labels']) for l in labels]}
    model.train()
    loss, acc = model(node_features=[torch.from_numpy(g[1]).float() for g in graphs],
                      edge_features=[torch.from_numpy(g[2]).float() for g in graphs],
                      edge_index=[torch.from_numpy(g[0]['adj_list']).long() for g in graphs],
                      adj_matrix=[torch.from_numpy(g[0]['adj_matrix']) for g in graphs],
                      labels=lab)
    total = loss['loss_node_cls'] + loss['loss_node_reg'] + loss['loss_edge_cls'] + loss['loss_obj_cls']
    total.backward()
    for k_, v in loss.items():
        data[f's1/{k_}'] = np.float64(v.item())
    for k_, v in acc.items():
        data[f's1/{k_}'] = np.float64(float(v))
    for name, p_ in model.named_parameters():
        data['g1/' + name] = p_.grad.detach().numpy().copy()
    data.update(n_frames=len(sizes), aggregation='max', L=2)
    np.savez_compressed(os.path.join(HERE, 'train_max_2frames.npz'), **data)
    print('max training', {k: v for k, v in data.items() if k.startswith('s1')})


def make_finetune_fixtures():
    """Model_Object_Classifier_Finetuning (gnn_detector.py:481-519) with the trained
    checkpoint, frozen except predict_class (set_param_for_finetuning_obj_classifier.py:31-34):
    loss, accuracy and the predict_class gradients of one step on 2 frames (proposals from
    the predicted offsets, majority-vote object labels), then the same in eval mode under
    no_grad (the validation call of finetuning.py:85-96)."""
    from modules.set_configurations.set_config_gnn import config
    from modules.neural_net.gnn.gnn_detector import Model_Object_Classifier_Finetuning
    cfg = config(os.path.join(REF, 'configuration_radarscenes_gnn.yml'))
    torch.manual_seed(5)
    model = Model_Object_Classifier_Finetuning(cfg)
    sd = torch.load(CKPT, map_location='cpu', weights_only=True)
    model.load_state_dict(sd)
    model.pred.freeze_layers_except_object_class_predictor()
    sizes, seeds = (300, 260), (9301, 9302)
    data = {}
    args = {k: [] for k in ('node_features', 'edge_features', 'other_features', 'edge_index',
                            'adj_matrix', 'node_class_labels')}
    for f, (n, sd_) in enumerate(zip(sizes, seeds)):
        fr = synthetic.make_frame(n, sd_)
        adj, nf, ef = _ref_graph(fr, cfg.ball_query_eps_square, cfg.k_number_nearest_points)
        lb = synthetic.make_labels(fr, adj['adj_list'], cfg.num_classes, sd_)
        other = np.stack([fr['meas_px'], fr['meas_py'], fr['meas_vx'], fr['meas_vy']], -1).astype(np.float32)
        args['node_features'].append(torch.from_numpy(nf).float())
        args['edge_features'].append(torch.from_numpy(ef).float())
        args['other_features'].append(torch.from_numpy(other))
        args['edge_index'].append(torch.from_numpy(adj['adj_list']).long())
        args['adj_matrix'].append(torch.from_numpy(adj['adj_matrix']))
        args['node_class_labels'].append(torch.from_numpy(lb['node_class']))
        data[f'f{f}/node_features'] = nf.astype(np.float32)
        data[f'f{f}/edge_features'] = ef.astype(np.float32)
        data[f'f{f}/edge_index'] = adj['adj_list'].astype(np.int32)
        data[f'f{f}/other_features'] = other
        data[f'f{f}/node_class'] = lb['node_class']
    model.train()
    loss, acc = model(**args)
    loss.backward()
    data['loss'] = np.float64(loss.item())
    data['accuracy'] = np.float64(float(acc))
    for name, p_ in model.named_parameters():
        if p_.requires_grad:
            data['g/' + name] = p_.grad.detach().numpy().copy()
    model.eval()
    with torch.no_grad():
        loss_e, acc_e = model(**args)
    data['eval_loss'] = np.float64(loss_e.item())
    data['eval_accuracy'] = np.float64(float(acc_e))
    data.update(n_frames=len(sizes))
    np.savez_compressed(os.path.join(HERE, 'finetune_trained_2frames.npz'), **data)
    print('finetune', data['loss'], data['accuracy'], data['eval_loss'],
          sorted(k for k in data if k.startswith('g/')))


def make_classifier_fixtures():
    """Cluster-level classifier GNN (modules/neural_net/classifier):
    the reference's own Model_Training(cfg) -- pred forward per sample and the loss over
    a batch of samples -- on synthetic object samples (synthetic.make_objects).  The
    edges come from the oracle's restatement of compute_edge_index: the reference's
    datagen_classifier imports h5py (absent) through read_data."""
    sys.path.insert(0, REPO)
    from oracle.classifier_ref import compute_edge_index
    from modules.set_configurations.set_config_classifier import config
    from modules.neural_net.classifier.classifier import Model_Training
    ycfg = os.path.join(REF, 'configuration_radarscenes_gnn.yml')
    ccfg = os.path.join(REF, 'configuration_radarscenes_classifier.yml')

    def case(name, cfg, n_objs, seed0, model_seed, save_weights=True):
        torch.manual_seed(model_seed)
        m = Model_Training(cfg).eval()
        # the N(0, 0.01) head init makes every logit ~ the -ln 99 bias; scale the last
        # Linear so that the logits depend visibly on the pooled features
        with torch.no_grad():
            m.pred.predict_node.pred_cls.head[1].weight.mul_(100.0)
        samples = [synthetic.make_objects(n, seed0 + i) for i, n in enumerate(n_objs)]
        nf = [torch.from_numpy(s['node_features']) for s in samples]
        ei = [torch.from_numpy(compute_edge_index(s['object_size'].tolist())) for s in samples]
        osz = [torch.from_numpy(s['object_size']) for s in samples]
        gt = [torch.from_numpy(s['object_class']) for s in samples]
        data = {}
        with torch.no_grad():
            for i in range(len(samples)):
                data[f's{i}/logits'] = m.pred(nf[i], ei[i], osz[i]).numpy()
                data[f's{i}/node_features'] = samples[i]['node_features']
                data[f's{i}/object_size'] = samples[i]['object_size']
                data[f's{i}/object_class'] = samples[i]['object_class']
                data[f's{i}/edge_index'] = ei[i].numpy().astype(np.int32)
            data['loss'] = np.float64(m(nf, ei, osz, gt).item())
        sd = m.state_dict()
        for k_, v in sd.items():
            data['fp/' + k_] = np.array([v.double().sum().item(), v.double().abs().sum().item()])
            if save_weights:
                data['w/' + k_] = v.numpy()
        data.update(n_samples=len(samples), model_seed=model_seed,
                    aggregation=cfg.classifier_aggregation)
        np.savez_compressed(os.path.join(HERE, name + '.npz'), **data)
        print('classifier', name, 'loss', data['loss'],
              'nodes', [int(s['object_size'].sum()) for s in samples])

    case('classifier_yml', config(ycfg, ccfg), (40, 25, 9), 8001, 1234)
    for aggr in ('mean', 'max'):
        cfg = config(ycfg, ccfg)
        cfg.classifier_aggregation = aggr
        cfg.classifier_graph_convolution_stem_channels = [128, 128]
        case(f'classifier_{aggr}', cfg, (30,), 8100, 77, save_weights=True)
    cfg = config(ycfg, ccfg)
    cfg.classifier_node_feat_enc_stem_channels = [96, 64]
    cfg.classifier_graph_convolution_stem_channels = [128, 64]
    cfg.classifier_msg_mlp_hidden_dim = 96
    cfg.classifier_node_pred_stem_channels = [64, 32]
    case('classifier_widths', cfg, (20, 7), 8200, 99)


def make_extra_features_fixture():
    """graph_convolution with augmented node features (gnn_blocks.py:116-164 with
    append_extra_features = [True, False, True], in_extra_feature_dim = 16; the blocks with
    the flag concatenate (x, extra, agg) before their update MLP, gnn_blocks.py:69-72, 107):
    the reference's own module, seeded init, on a reference-built kNN graph with random node,
    edge and extra features.  A second case adds a residual projection (48 -> 64 channels)
    and mean aggregation, a third an extra width of 3."""
    from modules.neural_net.gnn.gnn_blocks import graph_convolution
    from modules.compute_features.graph_features import compute_adjacency_information

    def case(name, n, in_c, stems, aggr, flags, seed, d_extra=16):
        frame = synthetic.make_frame(n, 9100 + seed)
        adj = compute_adjacency_information(frame, 25.0, 10)
        ei = torch.from_numpy(np.asarray(adj['adj_list']).astype(np.int64))
        torch.manual_seed(seed)
        m = graph_convolution(in_node_channels=in_c, in_edge_channels=64, stem_channels=stems,
                              msg_mlp_hidden_dim=128, activation='leakyrelu', aggregation=aggr,
                              norm_layer='channel_normalization', num_groups=None,
                              append_extra_features=flags, in_extra_feature_dim=d_extra)
        g = torch.Generator().manual_seed(seed + 1)
        x = torch.randn(n, in_c, generator=g)
        e = torch.randn(ei.shape[1], 64, generator=g)
        extra = torch.randn(n, d_extra, generator=g)
        with torch.no_grad():
            out = m(x, e, ei, extra)
        data = {'w/' + k: v.detach().numpy() for k, v in m.state_dict().items()}
        data.update(x=x.numpy(), e=e.numpy(), edge_index=ei.numpy(), extra=extra.numpy(),
                    out=out.numpy(), in_c=np.int64(in_c), stems=np.asarray(stems, np.int64),
                    flags=np.asarray(flags, np.int64), aggregation=np.asarray(aggr),
                    d_extra=np.int64(d_extra))
        np.savez_compressed(os.path.join(HERE, name + '.npz'), **data)
        print('wrote', name, out.shape)

    case('conv_extra_N300', 300, 64, [64, 64, 64], 'add', [True, False, True], 31)
    case('conv_extra_proj_N200', 200, 48, [64, 64], 'mean', [False, True], 32)
    # an extra width that is not a multiple of 4 (unaligned aggregate columns)
    case('conv_extra_odd_N150', 150, 64, [64, 64], 'add', [True, True], 33, d_extra=3)


def main():
    sys.path.insert(0, REF)
    _install_third_party_restatements()
    torch.set_num_threads(8)
    if '--classifier-only' in sys.argv:
        make_classifier_fixtures()
        return
    if '--training-only' in sys.argv:
        make_training_fixtures()
        return
    if '--norm-only' in sys.argv:
        make_norm_fixtures()
        return
    if '--finetune-only' in sys.argv:
        make_finetune_fixtures()
        return
    if '--max-training-only' in sys.argv:
        make_max_training_fixture()
        return
    if '--extra-only' in sys.argv:
        make_extra_features_fixture()
        return
    if '--proposals-only' not in sys.argv:
        make_graph_fixtures()
        make_model_fixtures()
    make_proposal_fixtures()
    make_training_fixtures()
    make_norm_fixtures()
    make_max_training_fixture()
    make_finetune_fixtures()
    make_classifier_fixtures()
    make_extra_features_fixture()


if __name__ == '__main__':
    main()
