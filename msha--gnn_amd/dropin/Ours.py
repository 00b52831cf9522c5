"""Drop-in for the classes of the reference's Ours.py (the reference module imports
train.py at load time, Ours.py:5): OursLayer, Ours and GraphAttentionLayer."""
import torch  # noqa: F401
import torch.nn as nn  # noqa: F401
import torch.nn.functional as F  # noqa: F401

import _boot  # noqa: F401
from msha_gnn_amd.layers import GraphAttentionLayer, Ours, OursLayer  # noqa: F401

K = 100  # Ours.py:7
