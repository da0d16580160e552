"""Reading the reference's checkpoint files without executing anything from them.

Two formats exist:

* ``save_pretrained`` files (Ndiff_transformer.py:251-265): ``{model_args,
  model_state}`` -- tensors and plain numbers, so ``torch.load(weights_only=True)``
  reads them as they are (``AlternatingDiffTransformer.from_pretrained``).
* ``best_model.pt`` (train.py:310-317): ``{model_state_dict, optimizer_state_dict,
  scheduler_state_dict, iter_num, best_val_loss, config}`` where ``config`` is a
  pickled instance of the reference's ``TrainingConfig`` class
  (``__main__.TrainingConfig`` when written by ``python train.py``).  PyTorch's
  weights-only loader refuses that class.  ``load_reference_checkpoint`` admits
  exactly that one name, mapped to an inert record class defined here: the loader
  creates the record with ``object.__new__`` and copies the pickled attribute dict
  into it, which runs no code from the file.  Every other global is still refused.

This repository's own ``train()`` writes the same keys with ``config`` as a plain
dict (``dataclasses.asdict``), so its files load with ``weights_only=True`` and
``load_reference_checkpoint`` reads both.
"""
from __future__ import annotations

import dataclasses
from typing import Any, Dict

import torch


def _record(module: str) -> type:
    cls = type("TrainingConfig", (), {"__doc__": "inert stand-in for the reference TrainingConfig "
                                                 "(attributes only; no methods run on load)"})
    cls.__module__ = module
    cls.__qualname__ = "TrainingConfig"
    return cls


# the names the reference's TrainingConfig is pickled under: run as a script, or imported as train
_RECORDS = [_record("__main__"), _record("train")]


def load_reference_checkpoint(path: str, map_location="cpu") -> Dict[str, Any]:
    """Load a reference ``best_model.pt`` (or one of ours) with the weights-only
    unpickler; ``config`` comes back as a plain dict of the pickled attributes."""
    with torch.serialization.safe_globals(_RECORDS):
        ckpt = torch.load(path, weights_only=True, map_location=map_location)
    cfg = ckpt.get("config")
    if cfg is not None and not isinstance(cfg, dict):
        cfg = dict(vars(cfg))
    return dict(ckpt, config=cfg)


def training_config_from(cfg: Dict[str, Any]):
    """This repository's TrainingConfig from a checkpoint's config dict (fields the
    reference has; extra or missing ones keep our defaults)."""
    from .train import TrainingConfig
    names = {f.name for f in dataclasses.fields(TrainingConfig)}
    return TrainingConfig(**{k: v for k, v in cfg.items() if k in names})
