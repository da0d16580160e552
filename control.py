"""Reference-compatible import path: ``from control import ...`` as in the reference's
train.py (train.py:19-21).  Re-exports differential_transformer_replication_amd.control."""
from differential_transformer_replication_amd.control import *  # noqa: F401,F403
from differential_transformer_replication_amd.control import __all__  # noqa: F401
