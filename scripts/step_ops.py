"""Which ATen ops (and which lines of msha_gnn_amd) launch the small kernels of the
configs[1] train step: torch.profiler over a few eager Ours steps, op table grouped by
the top of the Python stack."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import msha_loader  # noqa: E402

msha = msha_loader.load()
from msha_gnn_amd import layers  # noqa: E402
from msha_gnn_amd.data import GroupAdjacency  # noqa: E402

dev = torch.device("cuda:0")
n, m, flows, city, prov, gdp_arr = bench._year_graph("2015")
src_t = torch.as_tensor(flows[:, 0], device=dev)
dst_t = torch.as_tensor(flows[:, 1], device=dev)
adj = msha.normalize_adjacency_matrix(msha.inter_adjacency(src_t, dst_t, n, m))
cadj = GroupAdjacency(torch.as_tensor(city, device=dev))
padj = GroupAdjacency(torch.as_tensor(prov, device=dev))
gdp = {i: float(x) for i, x in enumerate(gdp_arr)}
torch.manual_seed(0)
model = layers.Ours(128, 64, m, 2, 0.5, gdp, n, m).to(dev)
from msha_gnn_amd import functional as MF  # noqa: E402
from msha_gnn_amd.optim import Adam  # noqa: E402

opt = Adam(model.parameters(), lr=1e-3, weight_decay=5e-4)  # bench.train_step_leg's step
opt.fuse_dropout_grad(model.Sfeatures)
si = torch.randint(0, len(flows), (64,), device=dev)
s_i, r_i = src_t[si], dst_t[si]


def body():
    opt.zero_grad(set_to_none=True)
    out = model(adj, cadj, padj, s_i)
    loss = MF.nll_loss_rows(out, s_i, r_i)
    loss.backward()
    opt.step()


for _ in range(3):
    body()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    body()
    torch.cuda.synchronize()
table = prof.key_averages(group_by_stack_n=4).table(sort_by="device_time_total", row_limit=60,
                                                    max_name_column_width=40,
                                                    max_src_column_width=90)
print(table)
