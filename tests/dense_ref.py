"""Dense PyTorch restatement of the reference modules, run in fp64 on the CPU.

TEST INFRASTRUCTURE ONLY: the torch reference of the floating-point path, used by the
full-size parity tests (tests/test_gpu_parity_full.py) where the per-row numpy oracle
has no backward.  It follows the reference's own dense formulation step by step
(masked scores with -9e15, ``softmax(dim=1)``, BatchNorm1d batch statistics, the joint
``SUM_county`` normaliser without max subtraction), so autograd gives the reference's
gradients in fp64:

  ours_layer     Ours.py:54-109   (OursLayer.forward, record off, dropout 0)
  ours_layer3    Ablation.py:260-277 (OursLayer3.forward, dropout 0)
  gal            Ablation.py:100-115 / GAT.py:20-35 (GraphAttentionLayer.forward)
  model          Ours.py:160-167 / Ablation.py:295-301 (Ours / ablation3 .forward)

Inputs are fp64 tensors; ``mask`` is the (N, M) boolean ``inter_adj > 0``; city / prov
are (N,) group ids (the reference's N x N same-group masks, restricted to the batch
rows ``src`` that Ours.py:81-82 reads).

``br`` (optional, per layer): LeakyReLU branch masks to evaluate the reference on --
"edge" (N, M) for the edge scores, "u" (N, F) / "v" (M, F) for the BatchNorm outputs,
"p3" / "p4" (B,) for the intra scores; True = the x > 0 branch.  LeakyReLU's derivative
jumps from 1 to 0.2 at 0, so where an input sits within rounding of 0 the fp64 and the
fp32 runs may take different branches and their gradients differ by a factor 5 there
(a discontinuity of the reference itself).  The full-size tests pass the branches the
GPU took (read off its stored intermediates), so the fp64 reference differentiates the
same piecewise-linear function; elsewhere the masks equal ``x > 0``.
"""
import torch
import torch.nn.functional as F

NEG = -9e15  # the reference's masked-score fill (Ablation.py:268, Ours.py:64)


def _lrelu(x, br, key):
    if br is None or br.get(key) is None:
        return F.leaky_relu(x, 0.2)
    return torch.where(br[key], x, 0.2 * x)


def _bn(x, w, b, training, rm=None, rv=None):
    if training:
        return F.batch_norm(x, None, None, w, b, training=True, eps=1e-5)
    return F.batch_norm(x, rm, rv, w, b, training=False, eps=1e-5)


def _inter(S, R, p, mask, br=None):
    """h1, h2 and the masked-softmax inter attention (Ours.py:58-67 = Ablation.py:262-270)."""
    h1 = R @ p["W1"]
    h2 = S @ p["W2"]
    Fd = h1.shape[1]
    a = p["a"].reshape(-1)
    # cat([h1_j, h2_i]) @ a, without materialising (N, M, 2F)
    e12 = _lrelu((h2 @ a[Fd:])[:, None] + (h1 @ a[:Fd])[None, :], br, "edge")
    att = torch.softmax(torch.where(mask, e12, torch.full_like(e12, NEG)), dim=1)
    return h1, h2, att


def _epilogue(u, v, p, training, br=None):
    """Ablation.py:273-277 / Ours.py:100-109."""
    v_out = _lrelu(_bn(v, p["bn1_weight"], p["bn1_bias"], training,
                       p.get("bn1_running_mean"), p.get("bn1_running_var")), br, "v")
    u_out = _lrelu(_bn(u, p["bn2_weight"], p["bn2_bias"], training,
                       p.get("bn2_running_mean"), p.get("bn2_running_var")), br, "u")
    return F.elu(u_out @ v_out.t())


def ours_layer3(S, R, p, mask, training, br=None):
    h1, h2, att = _inter(S, R, p, mask, br)
    return _epilogue(att @ h1, att.t() @ h2, p, training, br)


def ours_layer(S, R, p, mask, city, prov, src, training, br=None):
    """Ours.py:54-109 with record off and dropout 0."""
    h1, h2, att = _inter(S, R, p, mask, br)
    hb = h2[src]
    Fd = h1.shape[1]
    a3, a4 = p["a3"].reshape(-1), p["a4"].reshape(-1)
    # cat([h2_b, h2_b]) @ a3 is constant along n (Ours.py:71-75)
    e3 = _lrelu(hb @ a3[:Fd] + hb @ a3[Fd:], br, "p3")[:, None].expand(-1, S.shape[0])
    e4 = _lrelu(hb @ a4[:Fd] + hb @ a4[Fd:], br, "p4")[:, None].expand(-1, S.shape[0])
    m3 = city[src][:, None] == city[None, :]
    m4 = prov[src][:, None] == prov[None, :]
    x3 = torch.where(m3, e3, torch.full_like(e3, NEG))
    x4 = torch.where(m4, e4, torch.full_like(e4, NEG))
    SUM = torch.exp(x3).sum(1, keepdim=True) + torch.exp(x4).sum(1, keepdim=True) \
        + torch.exp(att[src]).sum(1, keepdim=True)
    att3 = torch.exp(x3) / SUM
    att4 = torch.exp(x4) / SUM
    u = att @ h1 + att3.t() @ hb + att4.t() @ hb
    return _epilogue(u, att.t() @ h2, p, training, br)


def gal(x, W, mask):
    """GraphAttentionLayer (GAT.py:20-35): its score is constant along a row."""
    h = x @ W
    e = torch.zeros_like(h)  # lrelu(cat(h_i, h_i) @ a) is a per-row constant
    att = torch.softmax(torch.where(mask, e, torch.full_like(e, NEG)), dim=1)
    return F.elu(att * h)


def model(Sf, Rf, heads, out_W, mask, training, city=None, prov=None, src=None, brs=None):
    """ablation3.forward (Ablation.py:295-301) or, with city/prov/src, Ours.forward
    (Ours.py:160-167): heads -> cat -> GAL -> elu -> log_softmax.  ``brs``: one branch
    dict per head."""
    brs = brs or [None] * len(heads)
    if city is None:
        xs = [ours_layer3(Sf, Rf, p, mask, training, b) for p, b in zip(heads, brs)]
    else:
        xs = [ours_layer(Sf, Rf, p, mask, city, prov, src, training, b)
              for p, b in zip(heads, brs)]
    x = torch.cat(xs, dim=1)
    return F.log_softmax(F.elu(gal(x, out_W, mask)), dim=1)


def layer_params(layer, dtype=torch.float64, requires_grad=True):
    """fp64 CPU leaves of an OursLayer / OursLayer3's parameters and BN buffers, keyed
    like gnn_oracle's parameter dicts (W1, W2, a, a3, a4, bn{1,2}_{weight,bias,...})."""
    p = {}
    for k in ("W1", "W2", "a", "a3", "a4"):
        p[k] = getattr(layer, k).detach().to("cpu", dtype).clone().requires_grad_(requires_grad)
    for bn in ("bn1", "bn2"):
        m = getattr(layer, bn)
        p[f"{bn}_weight"] = m.weight.detach().to("cpu", dtype).clone().requires_grad_(
            requires_grad)
        p[f"{bn}_bias"] = m.bias.detach().to("cpu", dtype).clone().requires_grad_(requires_grad)
        p[f"{bn}_running_mean"] = m.running_mean.detach().to("cpu", dtype).clone()
        p[f"{bn}_running_var"] = m.running_var.detach().to("cpu", dtype).clone()
    return p


GRAD_KEYS = {"W1": "W1", "W2": "W2", "a": "a", "a3": "a3", "a4": "a4",
             "bn1_weight": "bn1.weight", "bn1_bias": "bn1.bias", "bn2_weight": "bn2.weight",
             "bn2_bias": "bn2.bias"}
