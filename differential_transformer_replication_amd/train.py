"""Training driver (reference train.py surface) with data-parallel training.

Mirrors the reference's ``TrainingConfig``, ``TextDataset``,
``CosineWarmupScheduler``, ``estimate_loss`` and ``train`` (train.py:57-337):
AdamW (betas 0.9/0.95, wd 0.1), cosine warmup schedule, grad clip 1.0, mixed
precision, periodic eval and best-checkpoint saving.  Differences, all
deliberate:

* Data parallel over one process per GPU (torchrun env vars; RCCL), with the
  bucketed, backward-overlapped gradient all-reduce of ``dp.py``.  Each rank
  samples disjoint windows (``DistributedSampler`` semantics, seeded).
* The TinyStories download + BPE tokenizer (train.py:27-55, 153-180) needs a
  network; ``data='synthetic'`` (default) uses seeded uniform tokens over the
  same vocabulary.  A local token file (``.npy``/``.pt``) can be given instead.
* ``dtype='bf16'`` (default) runs autocast bf16 with no GradScaler; ``'fp16'``
  reproduces the reference (autocast fp16 + GradScaler); ``'fp32'`` disables
  autocast.
* wandb (absent, online) is replaced by stdout / JSONL.

Run:  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m \
          differential_transformer_replication_amd.train --model diff
"""
from __future__ import annotations

import argparse
import contextlib
import dataclasses
import json
import math
import os
import time
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist
from torch.optim import AdamW
from torch.optim.lr_scheduler import LRScheduler

from .dp import BucketedAllReduce


@dataclass
class TrainingConfig:
    """Defaults follow train.py:57-93; the DP/data/dtype fields are new."""
    model: str = "control"           # train.py constructs StandardTransformer (:223-230)
    n_embd: int = 768
    n_head: int = 4
    n_layer: int = 8
    block_size: int = 512
    dropout: float = 0.0
    n_terms: int = 4
    vocab_size: int = 12000
    batch_size: int = 1024
    grad_acc_steps: int = 1
    micro_batch_size: int = 32
    max_iters: int = 40_000
    eval_interval: int = 500
    eval_iters: int = 200
    learning_rate: float = 3.2e-4
    min_lr: float = 6e-5
    weight_decay: float = 0.1
    beta1: float = 0.9
    beta2: float = 0.95
    warmup_iters: int = 1000
    device: str = "cuda"
    backend: str = "nccl"
    log_interval: int = 10
    dtype: str = "bf16"               # bf16 | fp16 | fp32
    data: str = "synthetic"           # synthetic | path to a 1-d token tensor (.npy / .pt)
    num_tokens: int = 4_000_000
    seed: int = 1337
    bucket_cap_mb: float = 64.0
    ckpt_path: Optional[str] = "best_model.pt"
    log_jsonl: Optional[str] = None


class TextDataset(torch.utils.data.Dataset):
    """Windows of block_size tokens and their 1-shifted targets (train.py:95-107)."""

    def __init__(self, tokens, block_size, device):
        self.tokens = tokens.to(device)
        self.block_size = block_size
        self.device = device

    def __len__(self):
        return len(self.tokens) - self.block_size

    def __getitem__(self, idx):
        return self.tokens[idx:idx + self.block_size], self.tokens[idx + 1:idx + self.block_size + 1]


class CosineWarmupScheduler(LRScheduler):
    """Linear warmup then cosine decay to min_lr (train.py:109-123)."""

    def __init__(self, optimizer, warmup_steps, max_steps, min_lr=0.0):
        self.warmup_steps = warmup_steps
        self.max_steps = max_steps
        self.min_lr = min_lr
        super().__init__(optimizer)

    def get_lr(self):
        step = self.last_epoch
        if step < self.warmup_steps:
            return [base * step / self.warmup_steps for base in self.base_lrs]
        progress = (step - self.warmup_steps) / (self.max_steps - self.warmup_steps)
        factor = 0.5 * (1.0 + math.cos(math.pi * progress))
        return [self.min_lr + (base - self.min_lr) * factor for base in self.base_lrs]


def build_model(cfg: TrainingConfig) -> torch.nn.Module:
    if cfg.model == "diff":
        from .diff_transformer import DiffTransformer
        return DiffTransformer(cfg.vocab_size, cfg.n_embd, cfg.n_head, cfg.n_layer, cfg.block_size, cfg.dropout)
    if cfg.model == "ndiff":
        from .Ndiff_transformer import AlternatingDiffTransformer
        return AlternatingDiffTransformer(cfg.vocab_size, cfg.n_embd, cfg.n_head, cfg.n_layer, cfg.block_size,
                                          cfg.dropout, n_terms=cfg.n_terms)
    if cfg.model == "control":
        from .control import StandardTransformer
        # train.py:226 doubles the heads since each control head is twice as wide
        return StandardTransformer(cfg.vocab_size, cfg.n_embd, cfg.n_head * 2, cfg.n_layer, cfg.block_size,
                                   cfg.dropout)
    raise ValueError(f"unknown model {cfg.model!r}")


class ShardedWindows:
    """Seeded random windows, disjoint across ranks per step (DistributedSampler
    semantics over TextDataset's index space)."""

    def __init__(self, tokens: torch.Tensor, block_size: int, micro_batch: int, rank: int, world: int, seed: int):
        self.tokens = tokens
        self.T = block_size
        self.mb = micro_batch
        self.rank, self.world = rank, world
        self.gen = torch.Generator(device="cpu").manual_seed(seed)
        self.n = tokens.numel() - block_size - 1

    def next(self):
        idx = torch.randint(0, self.n, (self.world, self.mb), generator=self.gen)[self.rank].to(self.tokens.device)
        ar = torch.arange(self.T + 1, device=self.tokens.device)
        win = self.tokens[idx[:, None] + ar[None, :]]
        return win[:, :-1].contiguous(), win[:, 1:].contiguous()   # TextDataset yields contiguous windows


def load_tokens(cfg: TrainingConfig, device) -> torch.Tensor:
    if cfg.data == "synthetic":
        g = torch.Generator(device="cpu").manual_seed(cfg.seed)
        return torch.randint(0, cfg.vocab_size, (cfg.num_tokens,), generator=g).to(device)
    if cfg.data.endswith(".npy"):
        import numpy as np
        return torch.from_numpy(np.load(cfg.data, allow_pickle=False).astype("int64")).to(device)
    return torch.load(cfg.data, weights_only=True).long().to(device)


@torch.no_grad()
def estimate_loss(model, batches, cfg: TrainingConfig, ctx):
    """Mean loss over eval_iters batches per split (train.py:125-139)."""
    model.eval()
    out = {}
    for split, it in batches.items():
        losses = torch.zeros(cfg.eval_iters, device=cfg.device)
        for k in range(cfg.eval_iters):
            X, Y = it.next()
            with ctx():
                _, loss = model(X, Y)
            losses[k] = loss.float()
        out[split] = losses.mean()
    model.train()
    return out


def _autocast(cfg: TrainingConfig):
    if cfg.dtype == "fp32":
        return lambda: torch.autocast("cuda", enabled=False)
    dt = torch.bfloat16 if cfg.dtype == "bf16" else torch.float16
    return lambda: torch.autocast("cuda", dtype=dt)


def setup_distributed(cfg: TrainingConfig):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if cfg.device == "cuda":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device(cfg.device)
    if world > 1 and not dist.is_initialized():
        backend = cfg.backend if dev.type == "cuda" else "gloo"
        if backend == "nccl":
            dist.init_process_group(backend, device_id=dev)
        else:
            dist.init_process_group(backend)
    return world, rank, dev


_BUCKET_CLIP = os.environ.get("DTA_BUCKET_CLIP", "1") != "0"    # A/B switch: 0 = per-parameter clip


class Trainer:
    """One optimizer step = grad_acc_steps micro-steps + DP sync + clip + AdamW."""

    def __init__(self, cfg: TrainingConfig, model: torch.nn.Module, world: int, rank: int, device,
                 reduce_single: bool = False):
        self.cfg, self.model, self.world, self.rank = cfg, model, world, rank
        # reduce_single: launch every bucket's all-reduce from the backward hooks even in a
        # 1-rank group (bench.py times the hook / launch overhead an N-rank run carries)
        self.sync = BucketedAllReduce(model, cfg.bucket_cap_mb, reduce_single=reduce_single)
        self.opt = AdamW(model.parameters(), lr=cfg.learning_rate, betas=(cfg.beta1, cfg.beta2),
                         weight_decay=cfg.weight_decay, fused=device.type == "cuda")
        self.sched = CosineWarmupScheduler(self.opt, cfg.warmup_iters, cfg.max_iters, cfg.min_lr)
        self.scaler = torch.amp.GradScaler("cuda") if cfg.dtype == "fp16" else None
        self.ctx = _autocast(cfg)

    def step(self, get_batch) -> torch.Tensor:
        cfg = self.cfg
        total = None
        for micro in range(cfg.grad_acc_steps):
            X, Y = get_batch()
            last = micro == cfg.grad_acc_steps - 1
            with (contextlib.nullcontext() if last else self.sync.no_sync()):
                with self.ctx():
                    _, loss = self.model(X, Y)
                    loss = loss / cfg.grad_acc_steps
                if self.scaler is not None:
                    self.scaler.scale(loss).backward()
                else:
                    loss.backward()
            total = loss.detach() if total is None else total + loss.detach()
        self.sync.synchronize()
        if self.scaler is not None:
            self.scaler.unscale_(self.opt)
        if _BUCKET_CLIP:                 # clip_grad_norm_(model.parameters(), 1.0) over the buckets
            self.sync.clip_grad_norm_(1.0)
        else:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), 1.0)
        if self.scaler is not None:
            self.scaler.step(self.opt)
            self.scaler.update()
        else:
            self.opt.step()
        self.sync.zero_grad()            # keeps the bucket views (never set_to_none)
        self.sched.step()
        return total


def train(cfg: TrainingConfig):
    world, rank, dev = setup_distributed(cfg)
    torch.manual_seed(cfg.seed)
    model = build_model(cfg).to(dev)
    tokens = load_tokens(cfg, dev)
    n = int(0.9 * tokens.numel())
    train_it = ShardedWindows(tokens[:n], cfg.block_size, cfg.micro_batch_size, rank, world, cfg.seed + 1)
    val_it = ShardedWindows(tokens[n:], cfg.block_size, cfg.micro_batch_size, rank, world, cfg.seed + 2)
    tr = Trainer(cfg, model, world, rank, dev)
    best = float("inf")
    log = open(cfg.log_jsonl, "a") if (cfg.log_jsonl and rank == 0) else None
    t0 = time.time()
    for it in range(1, cfg.max_iters + 1):
        loss = tr.step(train_it.next)
        if it % cfg.log_interval == 0 and rank == 0:
            rec = {"iter": it, "loss": float(loss) * 1.0, "lr": tr.sched.get_last_lr()[0],
                   "tokens_per_s": cfg.log_interval * cfg.grad_acc_steps * cfg.micro_batch_size
                   * cfg.block_size * world / (time.time() - t0)}
            t0 = time.time()
            print(json.dumps(rec), flush=True)
            if log:
                log.write(json.dumps(rec) + "\n")
        if it % cfg.eval_interval == 0:
            losses = estimate_loss(model, {"train": train_it, "val": val_it}, cfg, tr.ctx)
            if world > 1:
                for v in losses.values():
                    dist.all_reduce(v)
                    v /= world
            if rank == 0:
                print(json.dumps({"iter": it, "train_loss": float(losses["train"]),
                                  "val_loss": float(losses["val"])}), flush=True)
                if losses["val"] < best and cfg.ckpt_path:
                    best = float(losses["val"])
                    torch.save({"model_state_dict": model.state_dict(),
                                "optimizer_state_dict": tr.opt.state_dict(),
                                "scheduler_state_dict": tr.sched.state_dict(),
                                "iter_num": it, "best_val_loss": best,
                                "config": dataclasses.asdict(cfg)}, cfg.ckpt_path)
    if log:
        log.close()
    return model


# ----------------------------------------------------------------- bench ---
CFG4 = dict(model="diff", vocab_size=12000, n_embd=1024, n_head=8, n_layer=20, block_size=2048, dropout=0.0,
            micro_batch_size=16)
# BASELINE configs[2]: N-term model, ~125M at n_terms=4 (hs = 768 / (2*6) = 64)
CFG3 = dict(model="ndiff", vocab_size=12000, n_embd=768, n_head=6, n_layer=10, block_size=2048, dropout=0.0,
            micro_batch_size=16)


# CPU / gloo dry run of the multi-rank path (bench.py --device cpu): a small control model
CPU_DRY = dict(model="control", vocab_size=256, n_embd=64, n_head=2, n_layer=2, block_size=32, dropout=0.0,
               micro_batch_size=4, device="cpu", dtype="fp32")

PEAK_BF16_TFLOPS = 2516.6          # MI355X dense bf16 MFMA peak (MI355X_MICROARCH.md)


def model_flops_per_token(model: torch.nn.Module, cfg: TrainingConfig) -> float:
    """Training FLOPs per token: 6 x (parameters in matmuls: everything but the
    token / position embedding tables) + the attention core's causal-halved
    fwd+bwd matmuls per token, 3 * H * T * (N*hs + dv) per layer."""
    skip = 0
    for name, p in model.named_parameters():
        if name.endswith("tok_emb.weight") or name.endswith("pos_emb.weight") or \
                name.endswith("token_embedding_table.weight") or name.endswith("position_embedding_table.weight"):
            skip += p.numel()
    dense = sum(p.numel() for p in model.parameters()) - skip
    if cfg.model == "control":
        H, hs, N, dv = cfg.n_head * 2, cfg.n_embd // (cfg.n_head * 2), 1, cfg.n_embd // (cfg.n_head * 2)
    else:
        H, hs = cfg.n_head, cfg.n_embd // (2 * cfg.n_head)
        N, dv = (cfg.n_terms if cfg.model == "ndiff" else 2), 2 * hs
    attn = 3.0 * H * cfg.block_size * (N * hs + dv) * cfg.n_layer
    return 6.0 * dense + attn


def train_bench(args, world, rank):
    """bench.py --mode train: BASELINE configs[3] -- ~350M DiffTransformer
    (12000, 1024, 8, 20, 2048), micro-batch 16 x 2048 per GPU, bf16 autocast,
    AdamW, DP all-reduce.  value = tokens/s over all ranks.  With --model ndiff:
    BASELINE configs[2] -- AlternatingDiffTransformer(12000, 768, 6, 10, 2048,
    n_terms=--n-terms), micro-batch 16 x 2048.  model "cpu-dry": a small control
    model on CPU over gloo (bench.py --device cpu), fp32."""
    arch = getattr(args, "model", "diff")
    if arch == "cpu-dry":
        cfg = TrainingConfig(**CPU_DRY, warmup_iters=10, max_iters=1000)
        dev = torch.device("cpu")
    else:
        base = CFG3 if arch == "ndiff" else CFG4
        extra = {"n_terms": args.n_terms} if arch == "ndiff" else {}
        cfg = TrainingConfig(**base, **extra, warmup_iters=100, max_iters=10_000, dtype="bf16")
        dev = torch.device("cuda", torch.cuda.current_device())
    cuda = dev.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    torch.manual_seed(cfg.seed)
    model = build_model(cfg).to(dev)
    nparams = sum(p.numel() for p in model.parameters())
    g = torch.Generator(device="cpu").manual_seed(cfg.seed + rank)
    tokens = torch.randint(0, cfg.vocab_size, (4_000_000 if cuda else 100_000,), generator=g).to(dev)
    it = ShardedWindows(tokens, cfg.block_size, cfg.micro_batch_size, rank, world, cfg.seed)
    single = bool(getattr(args, "reduce_single", False)) and cuda and world == 1
    if single and not dist.is_initialized():
        raise RuntimeError("reduce_single needs an initialised (1-rank) process group")
    tr = Trainer(cfg, model, world, rank, dev, reduce_single=single)
    for _ in range(args.warmup):
        tr.step(it.next)
    sync()
    t0 = time.perf_counter()
    loss = torch.zeros(())
    for _ in range(args.steps):
        loss = tr.step(it.next)
    sync()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    tok = world * cfg.micro_batch_size * cfg.block_size * max(args.steps, 1)
    tps = tok / el if el > 0 else 0.0
    fpt = model_flops_per_token(model, cfg)
    workload = {"cpu-dry": "CPU/gloo dry run: StandardTransformer(256,64,4,2,32) training step",
                "ndiff": f"cfg3: AlternatingDiffTransformer(12000,768,6,10,2048,n_terms={cfg.n_terms}) training step",
                }.get(arch, "cfg4: DiffTransformer(12000,1024,8,20,2048) DP training step")
    res = {"metric": "train tokens/sec", "value": round(tps, 1), "unit": "tokens/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / max(args.steps, 1) * 1e3, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "bf16" if cfg.dtype == "bf16" else cfg.dtype, "data": "synthetic", "final_loss": float(loss),
           "config": {"workload": workload, "params": nparams, "micro_batch_per_gpu": cfg.micro_batch_size,
                      "global_batch": cfg.micro_batch_size * world, "seq_len": cfg.block_size,
                      "parallelism": (f"dp{world} (bucketed {'RCCL' if cuda else 'gloo'} all-reduce, "
                                      f"{cfg.bucket_cap_mb} MB buckets, overlapped with backward)") if world > 1
                      else ("dp1 over a 1-rank RCCL group: every bucket all-reduce launched from the backward "
                            f"hooks ({cfg.bucket_cap_mb} MB buckets)" if single else
                            "dp1, no collective (one rank: the bucket all-reduces are not launched)")}}
    if cuda:
        res["model_tflops"] = round(fpt * tps / 1e12, 2)
        res["mfu"] = round(fpt * tps / 1e12 / (world * PEAK_BF16_TFLOPS), 4)
        res["flops_per_token"] = fpt
    return res


def main():
    ap = argparse.ArgumentParser()
    for f in dataclasses.fields(TrainingConfig):
        ap.add_argument("--" + f.name.replace("_", "-"), type=type(f.default) if f.default is not None else str,
                        default=f.default)
    cfg = TrainingConfig(**vars(ap.parse_args()))
    train(cfg)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
