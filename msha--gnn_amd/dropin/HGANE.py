"""Drop-in for the reference's HGANE.py as train.py:12 star-imports it.

HGANE.py defines one model, a different ``GraphAttentionLayer`` (in, out, Scount,
Rcount, gdp, dropout; HGANE.py:11-76) that train.py never builds (its model is
``ablation3``, train.py:206).  That model is outside the accelerated path (SURVEY.md
§2), so this module exports the reference module's names with the class standing in
as a marker that says so when constructed.  (In the reference the star import rebinds
``GraphAttentionLayer`` in train.py's namespace to HGANE's class too.)
"""
import random  # noqa: F401
import sys  # noqa: F401

import numpy as np  # noqa: F401
import torch  # noqa: F401
import torch.nn as nn
import torch.nn.functional as F  # noqa: F401
from sklearn.metrics import roc_auc_score  # noqa: F401
from sklearn.preprocessing import label_binarize  # noqa: F401

import _boot  # noqa: F401


class GraphAttentionLayer(nn.Module):
    """HGANE.py:11-76 (not accelerated: outside the GAT / link-scoring hot path)."""

    def __init__(self, in_features, out_features, Scount, Rcount, gdp, dropout=0.5):
        raise NotImplementedError("HGANE.GraphAttentionLayer (HGANE.py:11-76) is outside the "
                                  "MI355X hot path; use Ablation / Ours / GAT models")
