"""msha_gnn_amd -- MI355X-native GAT message passing / link scoring for MSHA--GNN.

Import via ``msha_loader.load()`` (the directory name is not an identifier).
The compute path is the gfx950 HIP library ``lib/libmsha_gnn.so`` (C ABI in
``include/msha_gnn.h``); there is no CPU fallback.
"""
from . import _lib
from ._lib import MshaLibraryError, available
from .graph import Graph, clear_cache, graph_for, inter_adjacency, normalize_adjacency_matrix

__all__ = ["Graph", "graph_for", "clear_cache", "inter_adjacency", "normalize_adjacency_matrix",
           "MshaLibraryError", "available", "functional", "layers"]


def __getattr__(name):
    # heavier submodules on first use
    if name in ("functional", "layers"):
        import importlib

        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
