"""Drop-in for the hot-path parts of the reference's model.py (train.py:10
``from model import *``): normalize_adjacency_matrix on the GPU, and the names
train.py picks up through this star import (torch, nn, F, np and the host-side
metric helpers), and GCN / GraphConvolution (model.py:11-64) on the HIP SpMM."""
import numpy as np  # noqa: F401
import torch  # noqa: F401
import torch.nn as nn  # noqa: F401
import torch.nn.functional as F  # noqa: F401

import _boot  # noqa: F401
from msha_gnn_amd.graph import normalize_adjacency_matrix  # noqa: F401
from msha_gnn_amd.layers import GCN, GraphConvolution  # noqa: F401
from msha_gnn_amd.metrics import (calculate_accuracy, calculate_auc,  # noqa: F401
                                  calculate_precision_recall)
