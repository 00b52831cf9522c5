"""Puts the repository root on sys.path and mounts msha--gnn_amd as msha_gnn_amd."""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
import msha_loader  # noqa: E402

msha = msha_loader.load()
