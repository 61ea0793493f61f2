"""Import helper: the package directory `clustered-low-rank-sdp-solver_amd/` is not a valid
Python identifier, so it is loaded under the module name ``clrsdp_amd``."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "clustered-low-rank-sdp-solver_amd")


def load():
    if "clrsdp_amd" in sys.modules:
        return sys.modules["clrsdp_amd"]
    spec = importlib.util.spec_from_file_location(
        "clrsdp_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["clrsdp_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_build():
    spec = importlib.util.spec_from_file_location("clrsdp_amd_build", os.path.join(PKG_DIR, "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod
