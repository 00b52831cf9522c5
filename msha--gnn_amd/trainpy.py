"""train.py as written, on the drop-in modules (``msha--gnn_amd/dropin/``).

``namespace(data_dir, device)`` runs train.py:1-15's imports exactly as the script
writes them, with the drop-in directory first on ``sys.path``, into a fresh namespace;
``setup`` then runs train.py:180-213 (dataset, split, loader, the three
``normalize_adjacency_matrix`` calls, the model, ``optim.Adam``, ``.to(device)``) and
``iteration`` one pass of the ``train()`` loop body, train.py:222-232, statement for
statement: ``.to(device)`` of the batch, ``optimizer.zero_grad()``, the model forward,
``F.nll_loss(output[source_index], recipient_index)``, ``loss.item()``, ``backward()``,
``optimizer.step()`` -- torch's Adam, no HIP graph, no fused loss.  Used by
tests/test_dropin.py and by bench.py's ``train_py_literal`` leg.

``write_year`` writes a year's data in the reference's ``anonymous_data`` formats
(Adjacent / GDP json, Flow csv with one row per flow, dataset.py:208-237).
"""
from __future__ import annotations

import contextlib
import json
import os
import sys

import torch

DROPIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dropin")
REF_MODULES = ("Ablation", "model", "HGANE", "dataset", "_boot", "GAT", "Ours", "LLP")

TRAIN_PY_IMPORTS = ("from __future__ import division\n"
                    "from __future__ import print_function\n"
                    "import time\n"
                    "import argparse\n"
                    "from Ablation import *\n"
                    "import torch.optim as optim\n"
                    "import gc\n"
                    "from model import *\n"
                    "from HGANE import *\n"
                    "from torch.utils.data import Dataset, DataLoader, random_split\n"
                    "import dataset\n"
                    "from dataset import *\n")


def write_year(path, year, city, prov, gdp, flows, m):
    """Adjacent{year}.json, GDP{year}.json, Flow{year}.csv under ``path``."""
    n = len(city)
    adj = {"source_index": {str(i): [int(city[i]), int(prov[i])] for i in range(n)},
           "recipient_index": {f"r{j}": j for j in range(m)}}
    with open(os.path.join(path, f"Adjacent{year}.json"), "w") as f:
        f.write(json.dumps(adj))
    with open(os.path.join(path, f"GDP{year}.json"), "w") as f:
        f.write(json.dumps({"GDP_embedding": {str(i): float(g) for i, g in enumerate(gdp)}}))
    lines = ["source,recipient,city,province"] + [f"{s},{r},{city[s]},{prov[s]}" for s, r in flows]
    with open(os.path.join(path, f"Flow{year}.csv"), "w", encoding="gb18030") as f:
        f.write("\n".join(lines) + "\n")


@contextlib.contextmanager
def namespace(data_dir, device, year="2015"):
    """train.py:1-15's imports through the drop-in directory, into a fresh namespace."""
    saved = {k: sys.modules.pop(k) for k in REF_MODULES if k in sys.modules}
    env = {k: os.environ.get(k) for k in ("MSHA_DATA_DIR", "MSHA_YEAR", "MSHA_DEVICE")}
    os.environ.update(MSHA_DATA_DIR=str(data_dir), MSHA_YEAR=str(year), MSHA_DEVICE=str(device))
    sys.path.insert(0, DROPIN)
    ns = {}
    try:
        exec(compile(TRAIN_PY_IMPORTS, "train.py:1-15", "exec"), ns)
        yield ns
    finally:
        sys.path.remove(DROPIN)
        for k in REF_MODULES:
            sys.modules.pop(k, None)
        sys.modules.update(saved)
        for k, v in env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


class TrainPy:
    """train.py:180-213 on a namespace from ``namespace``; ``model_kind`` 'ablation3'
    (the model train.py:206 builds) or 'Ours' (the full MSHA model train.py:44-176
    defines)."""

    def __init__(self, ns, device, dropout=0.5, model_kind="ablation3", seed=0,
                 batch_size=64, dtype=None):
        torch.manual_seed(seed)
        Dataset = ns["dataset"].HigherDataset()
        train_size = int(0.9 * len(Dataset))
        test_size = len(Dataset) - train_size
        train_dataset, _ = ns["random_split"](Dataset, [train_size, test_size])
        self.train_loader = ns["DataLoader"](train_dataset, batch_size=batch_size, shuffle=True)
        Scount, Rcount = Dataset.get_count()
        inter_adj, city_adj, province_adj = Dataset.get_adjacent()
        nrm = ns["normalize_adjacency_matrix"]
        inter_adj = nrm(inter_adj)
        city_adj = nrm(city_adj)
        province_adj = nrm(province_adj)
        GDP = Dataset.get_gdp()
        torch.manual_seed(seed)
        if model_kind == "ablation3":
            model = ns["ablation3"](in_features=128, out_features=64, n_classes=Rcount, n_heads=2,
                                    dropout=dropout, gdp=GDP, Scount=Scount, Rcount=Rcount)
        else:  # train.py's Ours(in, out, classes, heads, dropout, gdp, Scount, Rcount)
            import Ours as _ours  # noqa: N813  (the drop-in module, first on sys.path)

            model = _ours.Ours(128, 64, Rcount, 2, dropout, GDP, Scount, Rcount)
        self.optimizer = ns["optim"].Adam(model.parameters(), lr=0.001, weight_decay=5e-4)
        self.model = model.to(device) if dtype is None else model.to(device, dtype)
        self.inter_adj = inter_adj.to(device)
        self.city_adj = city_adj.to(device)
        self.province_adj = province_adj.to(device)
        self.device = device
        self.F = ns["F"]
        self.model.train()

    def iteration(self, data):
        """train.py:222-232 for one ``data`` = (source_index, recipient_index) from the
        loader; returns ``loss_train.item()``."""
        source_index, recipient_index = data
        source_index = source_index.to(self.device)
        recipient_index = recipient_index.to(self.device)

        self.optimizer.zero_grad()
        output = self.model(self.inter_adj, self.city_adj, self.province_adj, source_index)
        loss_train = self.F.nll_loss(output[source_index], recipient_index)
        loss = loss_train.item()
        loss_train.backward()
        self.optimizer.step()
        return loss
