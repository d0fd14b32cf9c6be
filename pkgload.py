"""Loads the package directory ``redis-bloomfilter_amd/`` as module ``redis_bloomfilter_amd``.

The directory name is fixed by the project layout and carries a hyphen, so it
cannot be imported with a plain ``import``.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "redis-bloomfilter_amd")
NAME = "redis_bloomfilter_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        sys.modules.pop(NAME, None)
        raise
    return mod
