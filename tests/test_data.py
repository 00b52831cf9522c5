"""Graph ingestion (data.HigherDataset) on a file tree written from the fixtures."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import golden


@pytest.fixture()
def data_dir(tmp_path):
    """anonymous_data-style files for the 512-source subgraph (2015) + a 2016 year
    without flows."""
    z = golden("sub512.npz")
    n, m = 512, 32
    rng = np.random.default_rng(0)
    city, prov = rng.integers(0, 40, n), rng.integers(0, 9, n)
    for year, with_flows in (("2015", True), ("2016", False)):
        adj = {"source_index": {str(i): [int(city[i]), int(prov[i])] for i in range(n)},
               "recipient_index": {f"p{j}": j for j in range(m)}}
        (tmp_path / f"Adjacent{year}.json").write_text(json.dumps(adj))
        (tmp_path / f"GDP{year}.json").write_text(
            json.dumps({"GDP_embedding": {str(i): float(g) for i, g in enumerate(z["gdp"])}}))
        if with_flows:
            lines = ["source,recipient"] + [f"{s},{r},{city[s]},{prov[s]}" for s, r in z["flows"]]
            (tmp_path / f"Flow{year}.csv").write_text("\n".join(lines) + "\n", encoding="gb18030")
    return str(tmp_path)


def test_dataset_interface(msha, data_dir):
    from msha_gnn_amd.data import HigherDataset

    z = golden("sub512.npz")
    ds = HigherDataset(data_dir, "2015", device="cpu")
    assert len(ds) == len(z["flows"]) and ds.get_count() == (512, 32)
    assert ds[3] == tuple(int(x) for x in z["flows"][3])
    assert list(ds.get_gdp().values())[:3] == [float(x) for x in z["gdp"][:3]]
    syn = HigherDataset(data_dir, "2016", device="cpu")
    syn2 = HigherDataset(data_dir, "2016", device="cpu")
    assert syn.synthetic and np.array_equal(syn.source, syn2.source)  # seeded by the year
    pairs = set(zip(syn.source.tolist(), syn.recipient.tolist()))
    assert len(pairs) == len(syn)  # distinct (source, recipient) edges
    assert syn.source.max() < 512 and syn.recipient.max() < 32


@pytest.mark.gpu
def test_dataset_adjacency_on_gpu(cuda, msha, data_dir):
    from msha_gnn_amd.data import HigherDataset

    z = golden("sub512.npz")
    ds = HigherDataset(data_dir, "2015", device=cuda)
    inter, city, prov = ds.get_adjacent()
    np.testing.assert_array_equal(inter.cpu().numpy(), z["counts"])
    norm = msha.normalize_adjacency_matrix(inter)
    np.testing.assert_array_equal(norm.cpu().numpy(), z["adj_norm"])
    assert msha.normalize_adjacency_matrix(city) is city  # group masks pass through
    d = city.dense().cpu().numpy()
    assert d.shape == (512, 512) and np.all(np.diag(d) == 1)
