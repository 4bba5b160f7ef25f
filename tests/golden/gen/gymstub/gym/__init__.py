"""Offline stand-in for the few gym 0.26 names the reference envs touch.

Test infrastructure only (fixture generation in the build container): gym is
not installed here and there is no network.  Only what
`Environments/Env_hybrid_multi_*.py:1-9` and `Environments/__init__.py:1`
import is provided.  `spaces.Dict` sorts plain-dict keys like gym 0.26 does,
which fixes the flat observation order to car|env|ped.
"""
from . import spaces, utils, envs  # noqa: F401
from .envs.registration import make, register  # noqa: F401


class Env:
    metadata = {}

    def __init__(self, *a, **k):
        pass
