"""Import the product package from ``msha--gnn_amd/`` under the module name ``msha_gnn_amd``.

The directory name carries the project's double dash, which is not a Python
identifier, so it is mounted explicitly:

    import msha_loader
    msha = msha_loader.load()          # == sys.modules["msha_gnn_amd"]
    from msha_gnn_amd import layers    # works afterwards
"""
import importlib.util
import os
import sys

PKG_NAME = "msha_gnn_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "msha--gnn_amd")


def load():
    mod = sys.modules.get(PKG_NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        PKG_NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        sys.modules.pop(PKG_NAME, None)
        raise
    return mod
