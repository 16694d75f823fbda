"""Import alias for the ``penr-oz-neural-network-v3-torch-ddp_amd`` package directory.

The framework's source lives in ``penr-oz-neural-network-v3-torch-ddp_amd/`` (a name Python
cannot import directly because of the hyphens).  This shim points the ``penroz`` package's
search path at that directory, so ``import penroz.models.model`` loads
``penr-oz-neural-network-v3-torch-ddp_amd/models/model.py``.
"""
import os as _os

_ROOT = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                      "penr-oz-neural-network-v3-torch-ddp_amd")
__path__ = [_ROOT]

with open(_os.path.join(_ROOT, "__init__.py")) as _f:
    exec(compile(_f.read(), _os.path.join(_ROOT, "__init__.py"), "exec"))
