"""Load real-time-anomaly-prediction-in-distributed-systems_amd/ as `rtap_amd`.

The package directory name (fixed by the build layout) contains hyphens, so
it cannot be imported by name; this registers it under an importable alias.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "real-time-anomaly-prediction-in-distributed-systems_amd")
NAME = "rtap_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
