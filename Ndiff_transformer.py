"""Reference-compatible import path: ``from Ndiff_transformer import ...`` as in the reference's
train.py (train.py:19-21).  Re-exports differential_transformer_replication_amd.Ndiff_transformer."""
from differential_transformer_replication_amd.Ndiff_transformer import *  # noqa: F401,F403
from differential_transformer_replication_amd.Ndiff_transformer import __all__  # noqa: F401
