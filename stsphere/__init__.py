"""Importable name for the framework package.

The source tree lives in ``sharding-the-sphere-fall-2025-jax-devlab-examples_amd/``
(a directory name that is not a Python identifier).  This shim points the
package search path there, so ``import stsphere.models.swe`` etc. resolve to
the files in that directory, and then runs its ``__init__``.
"""
import os as _os

_SRC = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "sharding-the-sphere-fall-2025-jax-devlab-examples_amd",
)
__path__ = [_SRC]
with open(_os.path.join(_SRC, "__init__.py")) as _f:
    exec(compile(_f.read(), _os.path.join(_SRC, "__init__.py"), "exec"))
