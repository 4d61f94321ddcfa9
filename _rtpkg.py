"""Registers the package directory `ppo-radiotherapy_amd/` (hyphenated, so not
importable by name) as the module `ppo_radiotherapy_amd`.

Every entry point at the repo root (environment.py, train.py, networks.py,
bench.py, __graft_entry__.py, tests) does `import _rtpkg` first."""
import importlib.util
import os
import sys

NAME = "ppo_radiotherapy_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ppo-radiotherapy_amd")


def load():
    mod = sys.modules.get(NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod


load()
