"""Import shim: makes the package directory ``point-cloud-cnn-segmentation_amd/``
importable as ``pcs_amd`` (a hyphenated directory name is not a Python identifier).

``import pcs_amd`` replaces this module in ``sys.modules`` with the real package, so
``from pcs_amd.model import PointNetSegmentation`` works as usual.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_dir = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "point-cloud-cnn-segmentation_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_dir, "__init__.py"),
                                     submodule_search_locations=[_dir])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
