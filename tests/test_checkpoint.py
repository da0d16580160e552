"""Checkpoint / state-format compatibility against files the
REFERENCE wrote (tests/golden/make_ckpt_golden.py):

* ``save_pretrained`` -> ``from_pretrained`` (Ndiff_transformer.py:243-265), both
  directions, read with the weights-only loader;
* a reference-layout ``best_model.pt`` (train.py:310-317), whose ``config`` is a
  pickled ``TrainingConfig`` object: read by ``checkpoint.load_reference_checkpoint``
  without unpickling anything but tensors, numbers and one inert record class;
  its model, optimizer and scheduler states load into this repository's objects.
"""
import dataclasses
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_err

from differential_transformer_replication_amd import Ndiff_transformer as ND
from differential_transformer_replication_amd import control as C
from differential_transformer_replication_amd.checkpoint import load_reference_checkpoint, training_config_from
from differential_transformer_replication_amd.train import CosineWarmupScheduler, TrainingConfig

SAVE_PRETRAINED = os.path.join(GOLDEN, "ref_save_pretrained.pt")
BEST_MODEL = os.path.join(GOLDEN, "ref_best_model.pt")


@pytest.fixture(scope="module")
def ckpt_golden():
    return np.load(os.path.join(GOLDEN, "ckpt_golden.npz"))


def test_reference_save_pretrained_loads_weights_only():
    ref = torch.load(SAVE_PRETRAINED, weights_only=True)
    m = ND.AlternatingDiffTransformer.from_pretrained(SAVE_PRETRAINED)
    assert m.block_size == 24 and len(m.blocks) == 2 and m.blocks[0].diff_attn.heads[0].n_terms == 3
    sd = m.state_dict()
    for k, v in ref["model_state"].items():
        assert k in sd, k
        assert torch.equal(sd[k], v), k
    assert set(sd) == set(ref["model_state"])          # tril is virtual here but still a state_dict key


def test_save_pretrained_round_trip(tmp_path):
    m = ND.AlternatingDiffTransformer.from_pretrained(SAVE_PRETRAINED)
    path = tmp_path / "ours.pt"
    m.save_pretrained(str(path))
    ours = torch.load(str(path), weights_only=True)
    ref = torch.load(SAVE_PRETRAINED, weights_only=True)
    assert ours["model_args"] == ref["model_args"]
    assert set(ours["model_state"]) == set(ref["model_state"])
    for k, v in ref["model_state"].items():
        assert torch.equal(ours["model_state"][k], v), k
    m2 = ND.AlternatingDiffTransformer.from_pretrained(str(path))
    for (k, a), (k2, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k == k2 and torch.equal(a, b), k


def test_reference_best_model_refused_by_plain_weights_only_loader():
    # the reason load_reference_checkpoint exists: `config` is a pickled class instance
    with pytest.raises(Exception):
        torch.load(BEST_MODEL, weights_only=True)


def test_reference_best_model_state_loads(ckpt_golden):
    ck = load_reference_checkpoint(BEST_MODEL)
    assert ck["iter_num"] == 500 and torch.is_tensor(ck["best_val_loss"])
    cfg = ck["config"]
    assert isinstance(cfg, dict) and cfg["n_embd"] == 64 and cfg["learning_rate"] == pytest.approx(3.2e-4)
    tc = training_config_from(cfg)
    assert isinstance(tc, TrainingConfig) and tc.n_layer == 2 and tc.warmup_iters == cfg["warmup_iters"]
    V, E, H, L, T = (int(v) for v in ckpt_golden["ctrl_cfg"])
    model = C.StandardTransformer(V, E, H, L, T, 0.0)
    model.load_state_dict(ck["model_state_dict"], strict=True)
    model.eval()
    with torch.no_grad():
        logits, _ = model(torch.from_numpy(ckpt_golden["idx"]))
    assert rel_err(logits, ckpt_golden["logits_ctrl"]) < 1e-5
    opt = torch.optim.AdamW(model.parameters(), lr=tc.learning_rate, betas=(tc.beta1, tc.beta2),
                            weight_decay=tc.weight_decay)
    opt.load_state_dict(ck["optimizer_state_dict"])
    assert all(int(s["step"]) == 1 for s in opt.state.values())
    sched = CosineWarmupScheduler(opt, tc.warmup_iters, tc.max_iters, tc.min_lr)
    sched.load_state_dict(ck["scheduler_state_dict"])
    assert sched.last_epoch == 1


def test_own_checkpoint_format_is_weights_only(tmp_path):
    """train() writes config as a plain dict: both loaders read it."""
    cfg = TrainingConfig(model="control", n_embd=64, n_head=2, n_layer=2, block_size=24, vocab_size=97)
    m = C.StandardTransformer(97, 64, 4, 2, 24, 0.0)
    path = tmp_path / "best_model.pt"
    torch.save({"model_state_dict": m.state_dict(), "iter_num": 3, "best_val_loss": 1.0,
                "config": dataclasses.asdict(cfg)}, str(path))
    a = torch.load(str(path), weights_only=True)
    b = load_reference_checkpoint(str(path))
    assert a["config"] == b["config"] == dataclasses.asdict(cfg)


@pytest.mark.gpu
def test_from_pretrained_logits_on_gpu(ckpt_golden):
    """The reference-written save_pretrained file, loaded weights-only, run on the
    HIP path: logits match the reference's own (fp32, 1e-4)."""
    m = ND.AlternatingDiffTransformer.from_pretrained(SAVE_PRETRAINED).to("cuda").eval()
    with torch.no_grad():
        logits, _ = m(torch.from_numpy(ckpt_golden["idx"]).to("cuda"))
    assert rel_err(logits.float().cpu(), ckpt_golden["logits_ndiff"]) < 1e-4
