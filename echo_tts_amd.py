"""Import shim: exposes the package directory ``echo-tts_amd/`` as ``echo_tts_amd``.

The directory name carries a hyphen (project layout convention), which Python
cannot import directly. This module builds a proper package spec for that
directory and replaces itself in ``sys.modules`` with it.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_dir = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "echo-tts_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_dir, "__init__.py"),
                                     submodule_search_locations=[_dir])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
