"""Where the C4 bf16 weight gradient's error comes from.

Prints the smallest tol_close bar (|d| <= t |ref| + t max|ref|) each candidate meets
against the fp64 dW = X^T (d_hc + d_el (x) al + d_er (x) ar) of the fp64 oracle:
  library    W.grad from the library's bf16 backward;
  dh_fp32    X^T of the GPU's leaf gradients combined in fp32 (no bf16 rounding of dh);
  dh_bf16    the same dh rounded to bf16 (the MFMA operand today);
  dhc_ref    X^T of the fp64 d_hc with the GPU's d_el / d_er (the edge kernels' d_hc error
             removed).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import msha_loader  # noqa: E402

msha_loader.load()


def bar(got, ref):
    m = np.abs(ref).max()
    return float(np.max(np.abs(got - ref) / (np.abs(ref) + m)))


def main():
    import bench
    from msha_gnn_amd import functional as MF
    from msha_gnn_amd.graph import Graph
    from oracle import cpu_oracle
    from oracle import gnn_oracle as O

    cuda = torch.device("cuda:0")
    n, fin, H, Fd = 100_000, 128, 8, 16
    rowptr, col = bench.synth_graph(n, 2_000_000, seed=0)
    graph = Graph.from_csr(rowptr, col, n, cuda)
    colptr, perm = O.csr_to_csc(rowptr, col, n)
    csc_row = O.edge_rows(rowptr)[perm]
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(7)
    X = torch.rand(n, fin, generator=g).to(cuda, dt)
    W = (torch.randn(fin, H * Fd, generator=g) * fin ** -0.5).to(cuda, dt).requires_grad_(True)
    al = torch.randn(H, Fd, generator=g).to(cuda).requires_grad_(True)
    ar = torch.randn(H, Fd, generator=g).to(cuda).requires_grad_(True)
    dU = torch.randn(n, H, Fd, generator=g).to(cuda, dt)
    h, el, er = MF.project_scores(X, W, al, ar, heads=H)
    f64 = lambda t: t.detach().double().cpu().numpy()  # noqa: E731
    X64, al64, ar64 = f64(X), f64(al), f64(ar)
    el64, er64, hc64 = f64(el), f64(er), f64(h).reshape(n, H, Fd)
    u_ref, lse_ref = cpu_oracle.edge_attention_fwd(rowptr, col, el64, er64, hc64, fp64=True)
    d_el_ref, d_er_ref, d_hc_ref = cpu_oracle.edge_attention_bwd(
        rowptr, col, colptr, csc_row, perm, el64, er64, hc64, lse_ref, u_ref, f64(dU), fp64=True)
    dh_ref = d_hc_ref + d_el_ref[:, :, None] * al64[None] + d_er_ref[:, :, None] * ar64[None]
    dW_ref = X64.T @ dh_ref.reshape(n, H * Fd)

    u = MF.edge_attention(graph, el, er, h.view(n, H, Fd))
    u.backward(dU)
    el_l, er_l = (x.detach().clone().requires_grad_(True) for x in (el, er))
    hc_l = h.detach().view(n, H, Fd).clone().requires_grad_(True)
    MF.edge_attention(graph, el_l, er_l, hc_l).backward(dU)
    d_el, d_er, d_hc = f64(el_l.grad), f64(er_l.grad), f64(hc_l.grad)
    dh = d_hc + d_el[:, :, None] * al64[None] + d_er[:, :, None] * ar64[None]
    dh_b = f64(torch.as_tensor(dh, dtype=torch.float32).to(torch.bfloat16))
    dhc_ref = d_hc_ref + d_el[:, :, None] * al64[None] + d_er[:, :, None] * ar64[None]
    res = {"library": bar(f64(W.grad), dW_ref),
           "dh_fp32": bar(X64.T @ dh.reshape(n, -1), dW_ref),
           "dh_bf16": bar(X64.T @ dh_b.reshape(n, -1), dW_ref),
           "dhc_ref": bar(X64.T @ dhc_ref.reshape(n, -1), dW_ref),
           "d_hc_vs_ref": bar(d_hc, d_hc_ref), "d_el_vs_ref": bar(d_el, d_el_ref),
           "max_dW_ref": float(np.abs(dW_ref).max())}
    print(res, flush=True)


if __name__ == "__main__":
    main()
