"""The reference's ``utils.py`` API (utils.py:1-32): ``get_vars``, ``cluster_spec``,
``FastSaver`` -- re-exported from where they live in this package."""
from ..cluster import cluster_spec  # noqa: F401
from ..train.saver import FastSaver  # noqa: F401
from ..variables import get_vars  # noqa: F401
