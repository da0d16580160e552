"""Time model.generate with the KV cache (default) against the reference's
full-recompute loop (DTA_KV_CACHE=0) on the GPU: tokens/s of sampled tokens.
Model: cfg1's DiffTransformer (12000, 384, 6 heads, 6 layers, block 256) and an
AlternatingDiffTransformer (n_terms 3) of the same width, random init, fp32.
Usage: python tools/generate_bench.py  -> one JSON line per model."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from differential_transformer_replication_amd import diff_transformer as D  # noqa: E402
from differential_transformer_replication_amd import Ndiff_transformer as ND  # noqa: E402
from differential_transformer_replication_amd import control as C  # noqa: E402


def timed(model, idx, n, cache):
    os.environ["DTA_KV_CACHE"] = "1" if cache else "0"
    torch.manual_seed(0)
    model.generate(idx, 4)
    torch.cuda.synchronize()
    torch.manual_seed(0)
    t0 = time.perf_counter()
    out = model.generate(idx, n)
    torch.cuda.synchronize()
    return out, time.perf_counter() - t0


def main():
    B, prompt, new = 4, 32, 200
    for name, ctor in [("DiffTransformer cfg1", lambda: D.DiffTransformer(12000, 384, 6, 6, 256, 0.0)),
                       ("AlternatingDiffTransformer N=3", lambda: ND.AlternatingDiffTransformer(
                           12000, 384, 6, 6, 256, 0.0, n_terms=3)),
                       ("StandardTransformer (control, 6 heads of 64)", lambda: C.StandardTransformer(
                           12000, 384, 6, 6, 256, 0.0))]:
        torch.manual_seed(0)
        model = ctor().cuda().eval()
        idx = torch.randint(0, 12000, (B, prompt), device="cuda")
        fast, tf = timed(model, idx, new, True)
        slow, ts = timed(model, idx, new, False)
        print(json.dumps({"model": name, "batch": B, "prompt": prompt, "new_tokens": new,
                          "kv_cache_tok_s": round(B * new / tf, 1), "full_recompute_tok_s": round(B * new / ts, 1),
                          "speedup": round(ts / tf, 2), "tokens_equal": bool(torch.equal(fast, slow))}), flush=True)


if __name__ == "__main__":
    main()
