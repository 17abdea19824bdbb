"""Import alias: maps the package directory ``imagerestoration-development-unrolling_amd/``
(whose name is not a Python identifier) to the importable package ``irdu_amd``."""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "imagerestoration-development-unrolling_amd")
_spec = importlib.util.spec_from_file_location(__name__, os.path.join(_PKG_DIR, "__init__.py"),
                                               submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
