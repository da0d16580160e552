"""torch.profiler view of the cfg4 (or cfg3) training step: which ops launch the small
kernels (fills, casts, tiny elementwise) around the GEMMs and attention kernels.

    python tools/train_torchprof.py [--model diff|ndiff] [--steps 2] > out.txt
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from differential_transformer_replication_amd import train as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="diff")
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    base = T.CFG3 if a.model == "ndiff" else T.CFG4
    extra = {"n_terms": 3} if a.model == "ndiff" else {}
    cfg = T.TrainingConfig(**base, **extra, warmup_iters=100, max_iters=10_000, dtype="bf16")
    dev = torch.device("cuda", 0)
    torch.manual_seed(cfg.seed)
    model = T.build_model(cfg).to(dev)
    g = torch.Generator(device="cpu").manual_seed(cfg.seed)
    tokens = torch.randint(0, cfg.vocab_size, (4_000_000,), generator=g).to(dev)
    it = T.ShardedWindows(tokens, cfg.block_size, cfg.micro_batch_size, 0, 1, cfg.seed)
    tr = T.Trainer(cfg, model, 1, 0, dev)
    for _ in range(3):
        tr.step(it.next)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        for _ in range(a.steps):
            tr.step(it.next)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    print(ka.table(sort_by="self_device_time_total", row_limit=70, max_name_column_width=60,
                   max_shapes_column_width=70))
    print(prof.key_averages().table(sort_by="count", row_limit=40, max_name_column_width=60))


if __name__ == "__main__":
    main()
