"""Drop-in classes of the reference's LLP.py (the script itself is a training
driver): LinkPredictor and the teacher GAT with forward(input, adj)."""
import torch  # noqa: F401
import torch.nn as nn  # noqa: F401
import torch.nn.functional as F  # noqa: F401

import _boot  # noqa: F401
from msha_gnn_amd.layers import GraphAttentionLayer, LinkPredictor  # noqa: F401
from msha_gnn_amd.layers import LLPGAT as GAT  # noqa: F401

Teacher_LinkPredictor = LinkPredictor  # LLP.py:170-198 is the same module
