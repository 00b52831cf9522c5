"""Dense CPU restatement of the reference's train.py iteration (TEST INFRASTRUCTURE /
CPU BASELINE: imported only by bench.py's cpu_baseline leg and by tests; never by the
product package).

It follows the reference's own dense formulation op for op, so its CPU time is the cost
of the reference's path on this host:

  layer3_fwd   Ablation.py:260-277  OursLayer3.forward: h1 = R W1, h2 = S W2, the
               (N, M, 2F) expand+cat score tensor, masked softmax (-9e15), dropout,
               BatchNorm1d + LeakyReLU of att.T @ h2 and att @ h1, elu(u @ v.T)
  gal_fwd      GAT.py:20-35 / Ablation.py:100-115  GraphAttentionLayer.forward
  ablation3    Ablation.py:295-301  dropout(S, R) -> heads -> cat -> dropout -> GAL ->
               elu -> log_softmax
  train_step   train.py:221-232  zero_grad, forward, nll_loss(out[source_index]),
               backward, Adam(lr 1e-3, weight_decay 5e-4)
  score_pairs  LLP.py:104-115 with the caller's gather (LLP.py:233): mlp / inner

Parameters are plain tensors (no nn.Module), in the reference's shapes; BatchNorm runs
with batch statistics and updates running buffers like nn.BatchNorm1d in train mode.
Pinned by tests/test_oracle_golden.py against the sub512 fixture (the reference's own
outputs, loss and gradients).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

NEG = -9e15


def layer3_fwd(S, R, p, adj, dropout, training):
    """Ablation.py:260-277."""
    h1 = torch.mm(R, p["W1"])
    h2 = torch.mm(S, p["W2"])
    N, M = adj.shape
    Fd = h1.shape[1]
    inter = torch.cat([h1.unsqueeze(0).expand(N, -1, -1), h2.unsqueeze(1).expand(-1, M, -1)],
                      dim=2).view(N, -1, 2 * Fd)
    e12 = F.leaky_relu(torch.matmul(inter, p["a"]).squeeze(2), negative_slope=0.2)
    att = torch.where(adj > 0, e12, NEG * torch.ones_like(e12))
    att = F.softmax(att, dim=1)
    att = F.dropout(att, dropout, training=training)
    v = F.leaky_relu(F.batch_norm(att.t() @ h2, p["bn1_running_mean"], p["bn1_running_var"],
                                  p["bn1_weight"], p["bn1_bias"], training, 0.1, 1e-5), 0.2)
    u = F.leaky_relu(F.batch_norm(att @ h1, p["bn2_running_mean"], p["bn2_running_var"],
                                  p["bn2_weight"], p["bn2_bias"], training, 0.1, 1e-5), 0.2)
    return F.elu(u @ v.t())


def gal_fwd(x, W, a, adj, dropout, training):
    """GAT.py:20-35."""
    h = torch.mm(x, W)
    N, M = h.size()
    rep = h.unsqueeze(1).expand(-1, M, -1)
    e = F.leaky_relu(torch.matmul(torch.cat([rep, rep], dim=2), a).squeeze(2), 0.2)
    att = torch.where(adj > 0, e, NEG * torch.ones_like(e))
    att = F.dropout(F.softmax(att, dim=1), dropout, training=training)
    return F.elu(torch.mul(att, h))


def ablation3(params, adj, dropout, training):
    """Ablation.py:295-301."""
    s = F.dropout(params["Sfeatures"], dropout, training=training)
    r = F.dropout(params["Rfeatures"], dropout, training=training)
    x = torch.cat([layer3_fwd(s, r, hp, adj, dropout, training) for hp in params["heads"]],
                  dim=1)
    x = F.dropout(x, dropout, training=training)
    x = F.elu(gal_fwd(x, params["out_W"], params["out_a"], adj, dropout, training))
    return F.log_softmax(x, dim=1)


def init_params(n, m, fin=128, fd=64, heads=2, gen=None):
    """Reference-shaped parameters (Ablation.py:236-258, :280-293), xavier-like scale."""
    g = gen or torch.Generator().manual_seed(0)

    def xav(*shape):
        bound = 1.414 * (6.0 / (shape[0] + shape[1])) ** 0.5
        return ((torch.rand(*shape, generator=g) * 2 - 1) * bound).requires_grad_(True)

    hp = []
    for _ in range(heads):
        d = {"W1": xav(fin, fd), "W2": xav(fin, fd), "a": xav(2 * fd, 1)}
        for bn in ("bn1", "bn2"):
            d[f"{bn}_weight"] = torch.ones(fd, requires_grad=True)
            d[f"{bn}_bias"] = torch.zeros(fd, requires_grad=True)
            d[f"{bn}_running_mean"] = torch.zeros(fd)
            d[f"{bn}_running_var"] = torch.ones(fd)
        hp.append(d)
    return {"Sfeatures": torch.rand(n, fin, generator=g).requires_grad_(True),
            "Rfeatures": torch.rand(m, fin, generator=g).requires_grad_(True),
            "heads": hp, "out_W": xav(m * heads, m), "out_a": xav(2 * m, 1)}


def leaves(params):
    out = [params["Sfeatures"], params["Rfeatures"], params["out_W"], params["out_a"]]
    for d in params["heads"]:
        out += [v for k, v in d.items() if v.requires_grad]
    return out


def train_step(params, opt, adj, src, dst, dropout=0.5):
    """train.py:225-232: one iteration of the reference's loop."""
    opt.zero_grad()
    out = ablation3(params, adj, dropout, True)
    loss = F.nll_loss(out[src], dst)
    loss.backward()
    opt.step()
    return loss


def score_pairs(h, src, dst, mode, W=None, b=None):
    """LLP.py:233 gather + LLP.py:104-115 ('mlp': one used Linear, eval mode)."""
    x = h[src] * h[dst]
    if mode == "mlp":
        x = F.relu(F.linear(x, W, b))
    elif mode == "inner":
        x = torch.sum(x, dim=-1)
    return torch.sigmoid(x)
