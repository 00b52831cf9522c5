"""Drop-in nn.Modules of the reference hot path, computed by the HIP library.

Same class names, constructor arguments, parameter names/shapes, state_dict keys
and RNG consumption order as the reference, so a model built after
``torch.manual_seed(s)`` holds bit-identical initial parameters:

  GraphAttentionLayer   GAT.py:6-35        (also Ablation.py:86-115, LLP.py:117-146)
  GAT                   GAT.py:38-58
  LLPGAT                LLP.py:148-168     (GAT whose forward takes external features)
  OursLayer3            Ablation.py:235-277
  ablation3             Ablation.py:279-301  (its heads run as ONE multi-head launch)
  LinkPredictor         LLP.py:86-115
  OursLayer, Ours       Ours.py:29-167 (full MSHA: inter + city/province attention)
  GraphConvolution, GCN model.py:11-64     (SpMM over the same CSR/CSC machinery)

Adjacency arguments may be dense (N, M) tensors (as in train.py; the CSR/CSC view
is built once on the GPU and cached) or prebuilt ``Graph`` objects.  Every
attention op runs on the GPU through include/msha_gnn.h; CPU tensors raise.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import functional as MF
from . import replay
import math

from .graph import Graph, graph_for, graph_of, groups_for

ALPHA = 0.2  # LeakyReLU slope of the reference layers (Ablation.py:241, :267)


def _graph(adj) -> Graph:
    return adj if isinstance(adj, Graph) else graph_for(adj)


def _xavier_param(*shape):
    p = nn.Parameter(torch.zeros(size=shape))
    nn.init.xavier_uniform_(p.data, gain=1.414)
    return p


def _features_with_gdp(n_rows, n_features, gdp):
    """``cat(rand([N, d])[:, :-1], gdp)`` -- learnable table whose last column is
    the county GDP (GAT.py:41-42, Ablation.py:283-284)."""
    gdp_values = torch.tensor(list(gdp.values())).view(-1, 1)
    return nn.Parameter(torch.cat((torch.rand([n_rows, n_features])[:, :-1], gdp_values), dim=1))


class GraphAttentionLayer(nn.Module):
    """GAT.py:6-35.  Its score concatenates h_i with itself, so the attention is
    mask/deg and the layer is ``elu(dropout(mask/deg) * (input @ W))``; the
    ``a`` parameter is kept (state_dict parity) and receives a zero gradient,
    which is what the reference's ~1e-7 gradient is up to rounding."""

    def __init__(self, in_features, out_features, dropout):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.dropout = dropout
        self.W = _xavier_param(in_features, out_features)
        self.a = _xavier_param(2 * out_features, 1)

    def forward(self, input, adj):
        g = _graph(adj)
        h = MF.project_scores(input, self.W)  # GAT.py:21 on the MFMA GEMM
        return MF.gal(g, h, self.dropout, self.training, zero_grad_of=self.a)


class GAT(nn.Module):
    """GAT.py:38-58: heads of GraphAttentionLayer over a learnable feature table."""

    def __init__(self, n_features, n_classes, n_heads, dropout, gdp, N):
        super().__init__()
        self.features = _features_with_gdp(N, n_features, gdp)
        self.n_classes = n_classes
        self.n_heads = n_heads
        self.dropout = dropout
        self.attentions = [GraphAttentionLayer(n_features, n_classes, dropout=dropout)
                           for _ in range(n_heads)]
        for i, attention in enumerate(self.attentions):
            self.add_module(f"attention_{i}", attention)
        self.out_att = GraphAttentionLayer(n_features * n_heads, n_classes, dropout=dropout)

    def _body(self, x, adj):
        g = _graph(adj)
        x = F.dropout(x, self.dropout, training=self.training)
        x = torch.cat([att(x, g) for att in self.attentions], dim=1)
        x = F.dropout(x, self.dropout, training=self.training)
        x = F.elu(self.out_att(x, g))
        return F.log_softmax(x, dim=1)

    def forward(self, adj):
        return self._body(self.features, adj)


class LLPGAT(GAT):
    """LLP.py:148-168: the teacher GAT of the link-prediction script -- same layers,
    no feature table, ``forward(input, adj)``."""

    def __init__(self, n_features, n_classes, n_heads, dropout, gdp=None, N=None):
        nn.Module.__init__(self)
        self.n_classes = n_classes
        self.n_heads = n_heads
        self.dropout = dropout
        self.attentions = [GraphAttentionLayer(n_features, n_classes, dropout=dropout)
                           for _ in range(n_heads)]
        for i, attention in enumerate(self.attentions):
            self.add_module(f"attention_{i}", attention)
        self.out_att = GraphAttentionLayer(n_features * n_heads, n_classes, dropout=dropout)

    def forward(self, input, adj):
        return self._body(input, adj)


class OursLayer3(nn.Module):
    """Ablation.py:235-277: bipartite source->recipient attention with BN'd u/v
    aggregates and ``elu(u @ v.T)``.  a3/a4/bn3 exist (state_dict parity) but, as
    in the reference, take no part in the forward."""

    def __init__(self, in_features, out_features, dropout):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.alpha = ALPHA
        self.dropout = dropout
        self.W1 = nn.Parameter(torch.zeros(size=(in_features, out_features)))
        self.W2 = nn.Parameter(torch.zeros(size=(in_features, out_features)))
        nn.init.xavier_uniform_(self.W1.data, gain=1.414)
        nn.init.xavier_uniform_(self.W2.data, gain=1.414)
        self.a = _xavier_param(2 * out_features, 1)
        self.a3 = _xavier_param(2 * out_features, 1)
        self.a4 = _xavier_param(2 * out_features, 1)
        self.leakyrelu = nn.LeakyReLU(self.alpha)
        self.bn1 = nn.BatchNorm1d(out_features)
        self.bn2 = nn.BatchNorm1d(out_features)
        self.bn3 = nn.BatchNorm1d(out_features)

    def epilogue(self, u, v, count=True):
        """Ablation.py:273-277 on the aggregates: BN + LeakyReLU + u @ v.T + elu.
        (u, v arrive as head slices of the fused (rows, H, F) outputs; BatchNorm1d's
        backward is ~30x slower on the strided view, so they are made contiguous.)"""
        v_out = MF.bn_lrelu(v.contiguous(), self.bn1, self.alpha, count)
        u_out = MF.bn_lrelu(u.contiguous(), self.bn2, self.alpha, count)
        # u_out @ v_out.T on the library GEMM: its backward's v-side product reduces over
        # all N rows (deterministic split-K instead of a 2-workgroup BLAS tile)
        return F.elu(MF.matmul(u_out, v_out.t()))

    def forward(self, Sinput, Rinput, inter_adj, city_adj, province_adj, source_index):
        return fused_ours_layer3([self], Sinput, Rinput, _graph(inter_adj), self.training)[0]


def _epilogues(heads, us, vs):
    """Per-head BN epilogues; the heads' BatchNorm step counters advance in one foreach
    add instead of one launch per BatchNorm."""
    outs = [head.epilogue(us[k], vs[k], count=False) for k, head in enumerate(heads)]
    ctr = [bn.num_batches_tracked for h in heads for bn in (h.bn1, h.bn2)
           if bn.training and bn.track_running_stats and bn.momentum is not None]
    if ctr:
        torch._foreach_add_(ctr, 1)
    return outs


def _score_halves(heads, name):
    """(H, 2, F) stack of the heads' (2F, 1) score vectors ``name``: [:, 0] = a[:F],
    [:, 1] = a[F:]."""
    Fd = heads[0].out_features
    return torch.stack([getattr(h, name).view(2, Fd) for h in heads])


def _head_fusable(heads, graph: Graph, training) -> bool:
    """The model head (msha_head_fwd/bwd) covers the model's tail when the shape fits its
    LDS budget, the BatchNorms share eps / momentum (exponential average), and either
    training (batch statistics) or no autograd (eval)."""
    if not (training or not torch.is_grad_enabled()):
        return False
    bns = [bn for h in heads for bn in (h.bn1, h.bn2)]
    if any(bn.momentum is None or bn.eps != bns[0].eps or bn.momentum != bns[0].momentum
           or bn.training != training or not bn.affine for bn in bns):
        return False
    # eval without running statistics (track_running_stats=False): torch normalises with
    # the batch statistics there, which the head's eval path does not do
    if not training and any(bn.running_mean is None or bn.running_var is None for bn in bns):
        return False
    return MF.head_supported(graph, len(heads), heads[0].out_features)


def _model_tail(model, graph: Graph, u, v):
    """Ablation.py:273-277 per head + :298-301 (Ours.py:100-109 + :163-167) on the fused
    model head: one row pass from the (N, H, F) / (M, H, F) aggregates to log-probs."""
    heads = model.attentions
    return MF.model_head(graph, u, v, [(h.bn2, h.bn1) for h in heads], model.out_att.W,
                         model.out_att.a, model.dropout, model.training, heads[0].alpha)


def _tail_unfused(model, graph: Graph, u, v):
    """The same tail as per-head epilogue launches + out_att + ATen (shapes the model
    head does not cover, eval with autograd)."""
    outs = _epilogues(model.attentions, u.unbind(1), v.unbind(1))
    x = torch.cat(outs, dim=1)
    x = F.dropout(x, model.dropout, training=model.training)
    x = F.elu(model.out_att(x, graph))
    return F.log_softmax(x, dim=1)


def _attention_uv3(heads, s_input, r_input, graph: Graph, training, packed=False):
    """OursLayer3 inter attention of all heads: (u (N, H, F), v (M, H, F)).  ``packed``:
    the heads' packed parameters when the caller already has them (model_prologue)."""
    H = len(heads)
    Fd = heads[0].out_features
    n, m = s_input.shape[0], r_input.shape[0]
    if graph.n_cols != m or graph.n_rows != n:
        raise ValueError(f"inter_adj is {graph.n_rows}x{graph.n_cols}, features are {n} "
                         f"sources x {m} recipients")
    if packed is False:
        packed = MF.pack_heads(heads, intra=False)
    if packed is not None:  # one launch (and one in the backward)
        W1, W2, a_r, a_l = packed
    else:
        W1 = heads[0].W1 if H == 1 else torch.cat([h.W1 for h in heads], dim=1)
        W2 = heads[0].W2 if H == 1 else torch.cat([h.W2 for h in heads], dim=1)
        # Ablation.py:262-267: a[:F] scores the recipient (column) side h1, a[F:] the source
        a_r, a_l = _score_halves(heads, "a").unbind(1)  # (H, F) each
    h1, er = MF.project_scores(r_input, W1, ar=a_r, heads=H)  # (M, H*F), (M, H)
    h2, el = MF.project_scores(s_input, W2, al=a_l, heads=H)  # (N, H*F), (N, H)
    return MF.edge_attention(graph, el, er, h1.view(m, H, Fd), hs=h2.view(n, H, Fd),
                             p=heads[0].dropout, training=training)


def fused_ours_layer3(heads, s_input, r_input, graph: Graph, training):
    """All heads of an ablation3 in one launch: projections stacked along features,
    one (H-head) edge-attention forward/backward, per-head BN epilogues."""
    u, v = _attention_uv3(heads, s_input, r_input, graph, training)
    # unbind: the backward stacks the head gradients in one copy (u[:, k] selects would
    # zero-fill and copy a full (rows, H, F) gradient per head and add them)
    return _epilogues(heads, u.unbind(1), v.unbind(1))


class ablation3(nn.Module):  # noqa: N801  (reference class name)
    """Ablation.py:279-301: n_heads OursLayer3 -> cat -> dropout -> GAL -> elu ->
    log_softmax over recipients."""

    def __init__(self, in_features, out_features, n_classes, n_heads, dropout, gdp, Scount,
                 Rcount):
        super().__init__()
        self.Sfeatures = _features_with_gdp(Scount, in_features, gdp)
        self.Rfeatures = nn.Parameter(torch.rand([Rcount, in_features]))
        self.n_classes = n_classes
        self.n_heads = n_heads
        self.dropout = dropout
        self.attentions = [OursLayer3(in_features, out_features, dropout=dropout)
                           for _ in range(n_heads)]
        for i, attention in enumerate(self.attentions):
            self.add_module(f"attention_{i}", attention)
        self.out_att = GraphAttentionLayer(n_classes * n_heads, n_classes, dropout=dropout)

    def forward(self, inter_adj, city_adj, province_adj, source_index):
        if replay.eligible(self, source_index):  # one graph replay each way (replay.py)
            return replay.run(self, lambda s: self._forward(inter_adj, city_adj, province_adj,
                                                             s),
                              (inter_adj, city_adj, province_adj), source_index)
        return self._forward(inter_adj, city_adj, province_adj, source_index)

    def _forward(self, inter_adj, city_adj, province_adj, source_index):
        g = _graph(inter_adj)
        # feature dropout + head packing: one launch (and one autograd node) each way
        s_input, r_input, packed = MF.model_prologue(self.Sfeatures, self.Rfeatures,
                                                     self.dropout, self.training,
                                                     self.attentions, intra=False)
        u, v = _attention_uv3(self.attentions, s_input, r_input, g, self.training, packed)
        if _head_fusable(self.attentions, g, self.training):
            return _model_tail(self, g, u, v)
        return _tail_unfused(self, g, u, v)


class LinkPredictor(torch.nn.Module):
    """LLP.py:86-115.  'mlp': the used layers lins[:-1] each run as ONE fused
    (hadamard) Linear + ReLU + dropout [+ sigmoid] MFMA launch; as in the reference
    the last Linear is built but never applied, so the output is (B, hidden).
    'inner': sigmoid(sum(x_i * x_j, -1)), one fused gather-free reduction launch."""

    def __init__(self, predictor, in_channels, hidden_channels, out_channels, num_layers,
                 dropout):
        super().__init__()
        self.predictor = predictor
        self.lins = torch.nn.ModuleList()
        self.lins.append(torch.nn.Linear(in_channels, hidden_channels))
        for _ in range(num_layers - 2):
            self.lins.append(torch.nn.Linear(hidden_channels, hidden_channels))
        self.lins.append(torch.nn.Linear(hidden_channels, out_channels))
        self.dropout = dropout

    def reset_parameters(self):
        for lin in self.lins:
            lin.reset_parameters()

    def forward(self, x_i, x_j):
        if self.predictor == "inner":
            return MF.pair_inner(x_i, x_j)
        used = self.lins[:-1]
        if self.predictor != "mlp" or len(used) == 0:
            # LLP.py:104-115: any other predictor string takes neither branch and the
            # reference returns sigmoid(x_i * x_j), shape (B, F).  (num_layers <= 2 still
            # builds two Linears, LLP.py:93-96, so 'mlp' always applies one.)
            return MF.pair_hadamard_sigmoid(x_i, x_j)
        x = None
        for k, lin in enumerate(used):
            last = k == len(used) - 1
            if k == 0:
                x = MF.pair_layer(x_i, x_j, lin.weight, lin.bias, self.dropout, self.training,
                                  sigmoid=last)
            else:
                x = MF.pair_layer(x, None, lin.weight, lin.bias, self.dropout, self.training,
                                  sigmoid=last)
        return x

    def score_pairs(self, h, src, dst):
        """Inference with the caller's gather fused (LLP.py:233): predictor(h[src], h[dst])."""
        if self.predictor == "inner":
            return MF.score_pairs(h, src, dst, "inner")
        if len(self.lins) != 2:
            return self.forward(h[src], h[dst])
        return MF.score_pairs(h, src, dst, "mlp", self.lins[0].weight, self.lins[0].bias)


class OursLayer(OursLayer3):
    """Ours.py:29-109: OursLayer3's inter attention plus the intra-source attention
    of the batch ``source_index`` over its city / province groups (joint normaliser
    SUM_county).  city_adj / province_adj: dense same-group masks (as the reference)
    or ``data.GroupAdjacency``."""

    def forward(self, Sinput, Rinput, inter_adj, city_adj, province_adj, source_index,
                record=False, Coeff12=None, Coeff3=None, Coeff4=None):
        return fused_ours_layer([self], Sinput, Rinput, _graph(inter_adj), city_adj,
                                province_adj, source_index, self.training, record, Coeff12,
                                Coeff3, Coeff4)[0]


def fused_ours_layer(heads, s_input, r_input, graph: Graph, city_adj, province_adj,
                     source_index, training, record=False, Coeff12=None, Coeff3=None,
                     Coeff4=None):
    u, v = _attention_uv(heads, s_input, r_input, graph, city_adj, province_adj, source_index,
                         training, record, Coeff12, Coeff3, Coeff4)
    return _epilogues(heads, u.unbind(1), v.unbind(1))  # one stacked gradient copy


def _attention_uv(heads, s_input, r_input, graph: Graph, city_adj, province_adj,
                  source_index, training, record=False, Coeff12=None, Coeff3=None,
                  Coeff4=None, packed=False):
    """OursLayer inter + intra attention of all heads: (u (N, H, F), v (M, H, F))."""
    H = len(heads)
    Fd = heads[0].out_features
    n, m = s_input.shape[0], r_input.shape[0]
    if graph.n_cols != m or graph.n_rows != n:
        raise ValueError(f"inter_adj is {graph.n_rows}x{graph.n_cols}, features are {n} "
                         f"sources x {m} recipients")
    groups = groups_for(city_adj, province_adj, s_input.device)
    # e3 = lrelu(cat(h2_b, h2_b) @ a3) = lrelu(h2_b . (a3[:F] + a3[F:]))  (Ours.py:74-75)
    if packed is False:
        packed = MF.pack_heads(heads, intra=True)
    if packed is not None:  # one launch (and one in the backward)
        W1, W2, a_r, a_l, a3s, a4s = packed
    else:
        W1 = heads[0].W1 if H == 1 else torch.cat([h.W1 for h in heads], dim=1)
        W2 = heads[0].W2 if H == 1 else torch.cat([h.W2 for h in heads], dim=1)
        # (H, 2, F) views of the score vectors: their halves by unbind / sum, whose
        # backward is one stack / expand kernel
        a_r, a_l = _score_halves(heads, "a").unbind(1)
        a3s = _score_halves(heads, "a3").sum(1)
        a4s = _score_halves(heads, "a4").sum(1)
    h1, er = MF.project_scores(r_input, W1, ar=a_r, heads=H)
    h2, el = MF.project_scores(s_input, W2, al=a_l, heads=H)
    src = torch.as_tensor(source_index, device=s_input.device)
    u, v, attd, bstat = MF.ours_attention(graph, groups, src, el, er, h1.view(m, H, Fd),
                                          h2.view(n, H, Fd), a3s, a4s, p=heads[0].dropout,
                                          training=training, return_aux=True)
    if record:
        _record(attd, bstat, graph, groups, src, heads, Coeff12, Coeff3, Coeff4)
    return u, v


class _RecordState:
    """Where record mode leaves the whole inter attention when no ``train`` module is
    loaded (the reference assigns it to ``train.Coeff12new``, Ours.py:93)."""

    Coeff12new = None


record_state = _RecordState()


def _record(attd, bstat, graph, groups, src, heads, Coeff12, Coeff3, Coeff4):
    """Ours.py:92-96 attention dump for Explainer (record=True).  As the reference:
    the (N, M) post-dropout inter attention is assigned to ``train.Coeff12new`` (the
    ``train`` module when one is loaded, else ``layers.record_state``); the batch rows of
    the (B, N) city / province attention go to Coeff3[source_index] /
    Coeff4[source_index]; the Coeff12 argument is not written.  Every head overwrites,
    so the last head's values remain.  Off the hot path (torch scatter); Record() runs
    in eval mode (train.py:284-291), so the values are dropout-free."""
    import sys

    H = len(heads)
    dev = attd.device
    rows = torch.repeat_interleave(torch.arange(graph.n_rows, device=dev), graph.deg().long())
    dense = torch.zeros(graph.n_rows, graph.n_cols, device=dev)
    dense[rows, graph.col.long()] = attd[: graph.n_edges, H - 1]
    record_state.Coeff12new = dense
    train_mod = sys.modules.get("train")
    if train_mod is not None:
        train_mod.Coeff12new = dense
    (g3, _, _), (g4, _, _) = groups._keep
    for Cf, gid, col in ((Coeff3, g3, 5), (Coeff4, g4, 6)):
        if Cf is None:
            continue
        same = (gid[src.long()][:, None] == gid[None, :]).to(Cf.dtype)
        Cf[src.long()] = same * bstat[: src.numel(), H - 1, col][:, None].to(Cf.dtype)


class Ours(nn.Module):
    """Ours.py:144-167: n_heads OursLayer (one fused launch set) -> cat -> dropout ->
    GAL -> elu -> log_softmax."""

    def __init__(self, in_features, out_features, n_classes, n_heads, dropout, gdp, Scount,
                 Rcount):
        super().__init__()
        self.Sfeatures = _features_with_gdp(Scount, in_features, gdp)
        self.Rfeatures = nn.Parameter(torch.rand([Rcount, in_features]))
        self.n_classes = n_classes
        self.n_heads = n_heads
        self.dropout = dropout
        self.attentions = [OursLayer(in_features, out_features, dropout=dropout)
                           for _ in range(n_heads)]
        for i, attention in enumerate(self.attentions):
            self.add_module(f"attention_{i}", attention)
        self.out_att = GraphAttentionLayer(n_classes * n_heads, n_classes, dropout=dropout)

    def forward(self, inter_adj, city_adj, province_adj, source_index, record=False,
                Coeff12=None, Coeff3=None, Coeff4=None):
        if not record and replay.eligible(self, source_index):  # replay.py
            return replay.run(self, lambda s: self._forward(inter_adj, city_adj, province_adj,
                                                             s),
                              (inter_adj, city_adj, province_adj), source_index)
        return self._forward(inter_adj, city_adj, province_adj, source_index, record, Coeff12,
                             Coeff3, Coeff4)

    def _forward(self, inter_adj, city_adj, province_adj, source_index, record=False,
                 Coeff12=None, Coeff3=None, Coeff4=None):
        g = _graph(inter_adj)
        s_input, r_input, packed = MF.model_prologue(self.Sfeatures, self.Rfeatures,
                                                     self.dropout, self.training,
                                                     self.attentions, intra=True)
        u, v = _attention_uv(self.attentions, s_input, r_input, g, city_adj, province_adj,
                             source_index, self.training, record, Coeff12, Coeff3, Coeff4,
                             packed)
        if _head_fusable(self.attentions, g, self.training):
            return _model_tail(self, g, u, v)
        return _tail_unfused(self, g, u, v)


class GraphConvolution(nn.Module):
    """model.py:11-45: ``adj^T @ (input @ W) + b`` with the reference's SCALAR bias
    (``Parameter(torch.tensor(out_features))``, model.py:23) and its init order
    (rand weight, then uniform(-1/sqrt(out), 1/sqrt(out)) for weight and bias).
    ``adj`` may be the dense adjacency (A^T @ support) or its ``.t()`` view
    (A @ support); both run the HIP SpMM on A's cached CSR/CSC."""

    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.rand([in_features, out_features]))
        if bias:
            self.bias = nn.Parameter(torch.tensor(out_features, dtype=torch.float32))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        stdv = 1.0 / math.sqrt(self.weight.size(1))
        self.weight.data.uniform_(-stdv, stdv)
        if self.bias is not None:
            self.bias.data.uniform_(-stdv, stdv)

    def forward(self, input, adj):
        if isinstance(adj, Graph):
            raise TypeError("GraphConvolution needs the dense adjacency (its values weight "
                            "the propagation)")
        g, transposed = graph_of(adj)
        base = adj._base if transposed else adj
        support = MF.project_scores(input, self.weight)  # model.py:36 on the MFMA GEMM
        # model.py:37: adj.transpose(0, 1) @ support
        output = MF.spmm(g, g.values(base), support, transpose=not transposed)
        return output + self.bias if self.bias is not None else output

    def __repr__(self):
        return f"{self.__class__.__name__} ({self.in_features} -> {self.out_features})"


class GCN(nn.Module):
    """model.py:48-64: features (N, nfeat + 1) with the GDP column, gc1 on adj, gc2 on
    adj.t(), log_softmax over nhid (gc3 is built and never used, as in the reference)."""

    def __init__(self, nfeat, nhid, nclass, dropout, gdp, N):
        super().__init__()
        gdp_values = torch.tensor(list(gdp.values())).view(-1, 1)
        self.features = nn.Parameter(torch.cat((torch.rand([N, nfeat])[:, :], gdp_values), dim=1))
        self.gc1 = GraphConvolution(nfeat + 1, nhid)
        self.gc2 = GraphConvolution(nhid, nhid)
        self.gc3 = GraphConvolution(nhid, nclass)
        self.dropout = dropout

    def forward(self, adj):
        x = F.relu(self.gc1(self.features, adj))
        x = F.dropout(x, self.dropout, training=self.training)
        x = F.relu(self.gc2(x, adj.t()))
        return F.log_softmax(x, dim=1)
