"""Drop-in for the reference's GAT.py (GraphAttentionLayer, GAT)."""
import torch  # noqa: F401
import torch.nn as nn  # noqa: F401
import torch.nn.functional as F  # noqa: F401

import _boot  # noqa: F401
from msha_gnn_amd.layers import GAT, GraphAttentionLayer  # noqa: F401
