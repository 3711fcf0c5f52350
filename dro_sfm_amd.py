"""Import shim for the ``dro-sfm_amd/`` package directory.

The package directory carries the project's hyphenated name, which Python
cannot import by name; this module re-binds ``dro_sfm_amd`` to that directory
so ``import dro_sfm_amd.networks.depth_pose`` etc. resolve normally.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "dro-sfm_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_DIR, "__init__.py"),
                                     submodule_search_locations=[_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
