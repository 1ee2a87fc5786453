"""Registers the package directory `ece1782-smith-waterman-cuda_amd/` (whose
name is not a Python identifier) as the importable module `sw_amd`."""
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(REPO, "ece1782-smith-waterman-cuda_amd")


def load():
    mod = sys.modules.get("sw_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "sw_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["sw_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
