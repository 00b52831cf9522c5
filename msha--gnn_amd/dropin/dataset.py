"""Drop-in for the reference's dataset.py as train.py uses it (train.py:14-15
``import dataset`` / ``from dataset import *``, train.py:181 ``dataset.HigherDataset()``).

``HigherDataset()`` keeps the reference's zero-argument constructor (dataset.py:208-237)
and interface (``__getitem__`` -> (source, recipient), ``__len__``, ``get_count``,
``get_gdp``, ``get_adjacent``, dataset.py:239-255).  What the reference hard-codes is
taken from the environment instead:

  MSHA_DATA_DIR  the ``anonymous_data`` directory (reference: an absolute
                 /data/home/... path); default ``./anonymous_data``
  MSHA_YEAR      the year (reference: the module global ``year = '2018'``,
                 dataset.py:11); the module global ``year`` is kept and read at
                 construction time, so ``dataset.year = '2015'`` works as well
  MSHA_DEVICE    where the adjacencies are built (default: cuda when available)

The adjacencies come from ``msha_gnn_amd.data.HigherDataset``: the (N, M) flow-count
matrix accumulated on the GPU, city / province as group-id ``GroupAdjacency`` (the
reference's dense N x N masks, dataset.py:260-277, which ``normalize_adjacency_matrix``
passes through).  The reference's pre-anonymisation ETL (``HigherDataset_temp``,
``majorClassify``, the scipy helpers, dataset.py:13-205, :332-390) is not on the path.
"""
import csv  # noqa: F401  (names the reference module exports to ``from dataset import *``)
import json  # noqa: F401
import os
import time  # noqa: F401

import numpy as np  # noqa: F401
import scipy.sparse as sp  # noqa: F401
import torch
from torch.utils.data import Dataset  # noqa: F401

import _boot  # noqa: F401
from msha_gnn_amd import data as _data

year = os.environ.get("MSHA_YEAR", "2018")  # dataset.py:11


class HigherDataset(_data.HigherDataset):
    """dataset.py:208-255 with the zero-argument constructor."""

    def __init__(self):
        data_dir = os.environ.get("MSHA_DATA_DIR", os.path.join(os.getcwd(), "anonymous_data"))
        if not os.path.isdir(data_dir):
            raise FileNotFoundError(f"HigherDataset: data directory {data_dir!r} not found "
                                    "(set MSHA_DATA_DIR to the anonymous_data directory)")
        dev = os.environ.get("MSHA_DEVICE")
        super().__init__(data_dir, str(year), device=dev)
