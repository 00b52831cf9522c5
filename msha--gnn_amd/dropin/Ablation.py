"""Drop-in for the reference's Ablation.py (train.py:6 ``from Ablation import *``).

Put this directory first on sys.path; ablation3 / OursLayer3 / GraphAttentionLayer
then run on the MI355X HIP kernels with the reference's signatures and state_dict.
"""
import torch  # noqa: F401  (the reference module exports these names)
import torch.nn as nn  # noqa: F401
import torch.nn.functional as F  # noqa: F401

import _boot  # noqa: F401
from msha_gnn_amd.layers import GraphAttentionLayer, OursLayer3, ablation3  # noqa: F401

K = 100  # Ablation.py:5 module constant
