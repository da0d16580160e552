"""CPU checks of the KV-cache generate host logic (kv_cache.last_logits): which
steps prefill the window and which decode one position, through window slides
past block_size (the reference's crop, diff_transformer.py:177-185).  The model
step is stubbed, so no kernel runs."""
import torch

from differential_transformer_replication_amd import kv_cache


class _Model:
    block_size = 8


def _trace(monkeypatch, prompt, steps, graph="0"):
    monkeypatch.setenv("DTA_DECODE_GRAPH", graph)
    calls = []

    def step(model, idx, cache, pos):
        calls.append((idx.shape[1], pos))
        return torch.zeros(idx.shape[0], 3)

    monkeypatch.setattr(kv_cache, "_model_step", step)
    cache = kv_cache.KVCache()
    idx = torch.zeros(1, prompt, dtype=torch.long)
    for _ in range(steps):
        kv_cache.last_logits(_Model(), idx, cache)
        idx = torch.cat([idx, torch.zeros(1, 1, dtype=torch.long)], dim=1)
    return calls


def test_prefill_then_decode_positions(monkeypatch):
    calls = _trace(monkeypatch, prompt=3, steps=5)
    assert calls == [(3, 0), (1, 3), (1, 4), (1, 5), (1, 6)]


def test_window_slide_falls_back_to_prefill(monkeypatch):
    calls = _trace(monkeypatch, prompt=5, steps=7)
    # lengths 5 (prefill), 6, 7, 8 (decode at 5, 6, 7), then 9, 10, 11 > block 8: re-prefill the crop
    assert calls == [(5, 0), (1, 5), (1, 6), (1, 7), (8, 0), (8, 0), (8, 0)]


def test_full_prompt_window(monkeypatch):
    calls = _trace(monkeypatch, prompt=8, steps=3)
    assert calls == [(8, 0), (8, 0), (8, 0)]


def test_enabled_needs_cuda(monkeypatch):
    assert not kv_cache.enabled(torch.zeros(1, 1, dtype=torch.long))
