"""Checkpoint fixtures written BY THE REFERENCE, in the build
container only (the reference never travels to the GPU box).  Outputs are data:

  ref_save_pretrained.pt   AlternatingDiffTransformer.save_pretrained of a tiny
                           seeded reference model (Ndiff_transformer.py:251-265):
                           {model_args, model_state}, tensors and numbers only
  ref_best_model.pt        the dict train.py:310-317 saves, built from reference
                           objects: a tiny StandardTransformer (the model train.py
                           trains), AdamW after one step, the reference
                           CosineWarmupScheduler, and ``config`` = an instance of
                           the reference TrainingConfig pickled as
                           ``__main__.TrainingConfig`` (what ``python train.py``
                           writes) -- the part a weights-only loader must not execute
  ckpt_golden.npz          the reference models' logits on a fixed batch

train.py imports tiktoken and wandb at module level (absent here, and unused by
what this script touches): empty stand-in modules satisfy those two imports.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_ckpt_golden.py
"""
import os
import sys
import types

import numpy as np
import torch

REF = os.environ.get("DTA_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
for name in ("tiktoken", "wandb"):
    sys.modules.setdefault(name, types.ModuleType(name))

import Ndiff_transformer as ref_ndiff        # noqa: E402
import train as ref_train                    # noqa: E402


def main():
    # --- save_pretrained of a tiny N-diff model (lambdas randomised: SURVEY semantic 4)
    torch.manual_seed(21)
    m = ref_ndiff.AlternatingDiffTransformer(97, 64, 2, 2, 24, 0.0, n_terms=3)
    g = torch.Generator().manual_seed(22)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "lambda_" in n:
                p.copy_(torch.randn(p.shape, generator=g) * 0.1)
    m.save_pretrained(os.path.join(OUT, "ref_save_pretrained.pt"))
    idx = torch.randint(0, 97, (2, 24), generator=g)
    m.eval()
    with torch.no_grad():
        logits_nd, _ = m(idx)

    # --- train.py's best_model.pt layout with the reference's own objects
    import __main__
    cfg_cls = ref_train.TrainingConfig
    cfg_cls.__module__ = "__main__"            # as pickled by `python train.py`
    __main__.TrainingConfig = cfg_cls
    cfg = cfg_cls()
    cfg.n_embd, cfg.n_head, cfg.n_layer, cfg.block_size, cfg.vocab_size = 64, 2, 2, 24, 97
    torch.manual_seed(23)
    ctrl = ref_train.StandardTransformer(cfg.vocab_size, cfg.n_embd, cfg.n_head * 2, cfg.n_layer,
                                         cfg.block_size, cfg.dropout)
    opt = torch.optim.AdamW(ctrl.parameters(), lr=cfg.learning_rate, betas=(cfg.beta1, cfg.beta2),
                            weight_decay=cfg.weight_decay)
    sched = ref_train.CosineWarmupScheduler(opt, warmup_steps=cfg.warmup_iters, max_steps=cfg.max_iters,
                                            min_lr=cfg.min_lr)
    x = torch.randint(0, 97, (2, 24), generator=g)
    y = torch.randint(0, 97, (2, 24), generator=g)
    _, loss = ctrl(x, y)
    loss.backward()
    opt.step()
    sched.step()
    ctrl.eval()
    with torch.no_grad():
        logits_ctrl, _ = ctrl(idx)
    torch.save({"model_state_dict": ctrl.state_dict(), "optimizer_state_dict": opt.state_dict(),
                "scheduler_state_dict": sched.state_dict(), "iter_num": 500,
                "best_val_loss": loss.detach(), "config": cfg}, os.path.join(OUT, "ref_best_model.pt"))
    np.savez_compressed(os.path.join(OUT, "ckpt_golden.npz"), idx=idx.numpy(),
                        logits_ndiff=logits_nd.numpy(), logits_ctrl=logits_ctrl.numpy(),
                        ctrl_cfg=np.array([cfg.vocab_size, cfg.n_embd, cfg.n_head * 2, cfg.n_layer,
                                           cfg.block_size]))
    print("wrote", sorted(f for f in os.listdir(OUT) if f.startswith(("ref_", "ckpt_"))))


if __name__ == "__main__":
    main()
