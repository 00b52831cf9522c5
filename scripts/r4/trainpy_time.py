"""train.py-as-written step time (bench.train_py_literal_leg) for ablation3 and Ours on the
2015 graph, then a host-time breakdown of the literal iteration by phase (to, zero_grad,
forward, nll, item, backward, step; wall clock per phase, no extra syncs -- the item
phase is where the host waits for the forward) and, with --prof, a torch.profiler table
of one window (self CPU time per op)."""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
for kind in ("ablation3", "Ours"):
    print(json.dumps(bench.train_py_literal_leg(dev, kind)), flush=True)


def phases(kind, iters=300):
    import msha_loader

    msha_loader.load()
    from msha_gnn_amd import trainpy

    with tempfile.TemporaryDirectory() as d:
        bench.write_train_py_year(d)
        with trainpy.namespace(d, dev) as ns:
            tp = trainpy.TrainPy(ns, dev, model_kind=kind)
            batches = [b for _, b in zip(range(64), tp.train_loader)]
            acc = dict.fromkeys(("to", "zero_grad", "forward", "nll", "item", "backward", "step"), 0.0)
            for i in range(iters + 20):
                s_idx, r_idx = batches[i % len(batches)]
                t0 = time.perf_counter()
                s_idx = s_idx.to(dev)
                r_idx = r_idx.to(dev)
                t1 = time.perf_counter()
                tp.optimizer.zero_grad()
                t2 = time.perf_counter()
                out = tp.model(tp.inter_adj, tp.city_adj, tp.province_adj, s_idx)
                t3 = time.perf_counter()
                loss = tp.F.nll_loss(out[s_idx], r_idx)
                t4 = time.perf_counter()
                loss.item()
                t5 = time.perf_counter()
                loss.backward()
                t6 = time.perf_counter()
                tp.optimizer.step()
                t7 = time.perf_counter()
                if i >= 20:
                    for k, a, b in (("to", t0, t1), ("zero_grad", t1, t2), ("forward", t2, t3),
                                    ("nll", t3, t4), ("item", t4, t5), ("backward", t5, t6),
                                    ("step", t6, t7)):
                        acc[k] += (b - a) * 1e3 / iters
            torch.cuda.synchronize()
            print(json.dumps({"model": kind, "phase_ms": {k: round(v, 4) for k, v in acc.items()},
                              "total_ms": round(sum(acc.values()), 4)}), flush=True)
            if "--prof" in sys.argv:
                from torch.profiler import ProfilerActivity, profile

                with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as p:
                    for i in range(20):
                        tp.iteration(batches[i % len(batches)])
                    torch.cuda.synchronize()
                print(p.key_averages().table(sort_by="self_cpu_time_total", row_limit=40))


if "--phases" in sys.argv or "--prof" in sys.argv:
    for kind in ("ablation3", "Ours"):
        phases(kind)
