"""graph-marl_amd — MI355X-native vectorised rollout + training path for
graph-marl's routing environment and NetMon GNN.

Import with ``importlib.import_module("graph-marl_amd")`` (the package directory
name is not a Python identifier) after putting the repository root on sys.path.
"""
from . import _lib  # noqa: F401
from .routing import EVAL_SEEDS, Network, Routing, build_seed_list  # noqa: F401

__all__ = ["Network", "Routing", "build_seed_list", "EVAL_SEEDS"]
