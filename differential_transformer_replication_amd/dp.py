"""Data-parallel gradient synchronisation: bucketed all-reduce overlapped with
backward, one process per GPU over RCCL (``torch.distributed`` backend
``"nccl"`` is RCCL on ROCm; xGMI between the GPUs of a node).

The reference imports DDP/DistributedSampler but never uses them
(train.py:7-10, 88, 143-145): this is net-new.

Design
* Parameters are grouped into buckets in reverse registration order (the order
  autograd produces their gradients).  Each bucket owns one flat fp32 buffer;
  every parameter's ``.grad`` is a view into it (gradient-as-bucket-view), so
  autograd accumulates straight into the buffer and no copy is needed.
* A post-accumulate-grad hook counts ready gradients per bucket; the last one
  launches ``all_reduce(SUM, async_op=True)`` on that bucket while backward
  keeps running on the compute stream (RCCL runs on its own stream, ordered
  after the producing kernels).
* ``synchronize()`` (before unscale/clip/step) waits for every bucket and
  scales by 1/world.  ``no_sync()`` skips communication for gradient
  accumulation micro-steps.
* Buffers (``lambda_init``, ``freqs_cis``) are never broadcast per step; the
  reference's T x T ``tril`` does not exist here (SURVEY semantic 8).
* Packed attention projections (``packing.py``): the per-head weights of one
  module are laid out consecutively in pack order inside one bucket and bound
  to it (``packing.bind_grad``), so their backward accumulates the module's whole
  dW with one add and reports the parameters to ``_on_grad`` itself.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import packing


class _Bucket:
    __slots__ = ("params", "flat", "pending", "handle", "size", "seen")

    def __init__(self, params: List[torch.nn.Parameter], flat: torch.Tensor):
        self.params = params
        self.flat = flat
        self.size = len(params)
        self.pending = self.size
        self.handle = None
        self.seen: set = set()          # ids of the parameters reported since the last reset

    def reset(self) -> None:
        self.pending = self.size
        self.handle = None
        self.seen.clear()


class BucketedAllReduce:
    def __init__(self, module: torch.nn.Module, bucket_cap_mb: float = 64.0,
                 process_group: Optional[dist.ProcessGroup] = None, broadcast_init: bool = True,
                 reduce_single: bool = False):
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        # reduce_single: run the collectives even in a 1-rank group (tests of the RCCL path)
        self._reduce = self.world > 1 or (reduce_single and dist.is_initialized())
        self.params = [p for p in module.parameters() if p.requires_grad]
        self._enabled = True
        cap = int(bucket_cap_mb * 1024 * 1024)
        # units of bucket layout: single parameters, or a packed module's per-head
        # weights in pack order (kept together, never split across buckets)
        packs, pack_of = [], {}
        for m in module.modules():
            if hasattr(m, "param_packs"):
                groups_m = m.param_packs()
            elif hasattr(m, "packed_params") and isinstance(getattr(m, "_pack", None), dict):
                groups_m = [(m._pack, m.packed_params())]
            else:
                continue
            for holder, allp in groups_m:
                pp = [p for p in allp if p.requires_grad]
                if (pp and len(pp) == len(allp) and all(p.dtype == torch.float32 for p in pp)
                        and not any(id(p) in pack_of for p in pp)):
                    packs.append((holder, pp))
                    for p in pp:
                        pack_of[id(p)] = len(packs) - 1
        units, seen = [], set()
        for p in reversed(self.params):
            k = pack_of.get(id(p))
            if k is None:
                units.append([p])
            elif k not in seen:
                seen.add(k)
                units.append(packs[k][1])
        groups: List[List[torch.nn.Parameter]] = []
        cur, cur_bytes = [], 0
        for u in units:
            nb = sum(p.numel() for p in u) * 4
            if cur and cur_bytes + nb > cap:
                groups.append(cur)
                cur, cur_bytes = [], 0
            cur.extend(u)
            cur_bytes += nb
        if cur:
            groups.append(cur)
        self.buckets: List[_Bucket] = []
        self._owner: Dict[int, _Bucket] = {}
        for g in groups:
            dev = g[0].device
            flat = torch.zeros(sum(p.numel() for p in g), device=dev, dtype=torch.float32)
            off = 0
            for p in g:
                if p.dtype != torch.float32:
                    raise RuntimeError("bucketed all-reduce expects fp32 master parameters")
                p.grad = flat[off:off + p.numel()].view_as(p)
                off += p.numel()
            b = _Bucket(g, flat)
            self.buckets.append(b)
            for p in g:
                self._owner[id(p)] = b
        # A packed group reports its parameters itself (packing.bind_grad) and returns None
        # gradients to autograd -- whose post-accumulate hooks still fire, with nothing
        # accumulated: hooking those parameters too would count every one of them twice
        # and launch a bucket before the rest of its gradients are in.
        for p in self.params:
            if id(p) not in pack_of:
                p.register_post_accumulate_grad_hook(self._on_grad)
        for holder, pp in packs:
            b = self._owner[id(pp[0])]
            start = pp[0].grad.data_ptr() - b.flat.data_ptr()
            n = sum(p.numel() for p in pp)
            packing.bind_grad(holder, pp, b.flat[start // 4:start // 4 + n], self._on_grad)
        if broadcast_init and self.world > 1:
            # identical initial parameters on every rank (parameters only, once)
            with torch.no_grad():
                for p in self.params:
                    dist.broadcast(p.data, src=0, group=self.pg)

    # ----------------------------------------------------------- hooks ---
    def _is_view(self, p: torch.nn.Parameter) -> bool:
        b = self._owner.get(id(p))
        if b is None or p.grad is None:
            return False
        lo = b.flat.data_ptr()
        return lo <= p.grad.data_ptr() < lo + b.flat.numel() * 4

    def _on_grad(self, p: torch.nn.Parameter) -> None:
        if not self._enabled or not self._reduce:
            return          # (world 1: a replaced .grad falls back to per-parameter grads;
                            # clip_grad_norm_ then checks the views itself)
        if not self._is_view(p):
            raise RuntimeError("parameter gradient is no longer a view of its bucket "
                               "(use BucketedAllReduce.zero_grad, not set_to_none)")
        b = self._owner[id(p)]
        # every parameter reports exactly once per synchronised backward, and a bucket
        # launches only once all of them are in: an early or repeated report (a backward
        # path calling the hook itself) would otherwise all-reduce partial gradients
        if id(p) in b.seen or b.pending <= 0:
            raise RuntimeError("gradient reported twice to its DP bucket in one backward")
        b.seen.add(id(p))
        b.pending -= 1
        if b.pending == 0:
            b.handle = dist.all_reduce(b.flat, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    @contextlib.contextmanager
    def no_sync(self):
        prev, self._enabled = self._enabled, False
        try:
            yield
        finally:
            self._enabled = prev

    def synchronize(self) -> None:
        """Wait for every bucket (launching any whose gradients never all arrived,
        e.g. unused parameters -- identical on every rank) and average."""
        if not self._reduce:
            return
        for b in self.buckets:
            if b.handle is None:
                b.handle = dist.all_reduce(b.flat, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
        inv = 1.0 / self.world
        for b in self.buckets:
            b.handle.wait()
            b.flat.mul_(inv)
            b.reset()

    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """torch.nn.utils.clip_grad_norm_(params, max_norm) (train.py:273) over the flat
        buckets the parameters' gradients are views of: the same L2 norm and scale,
        computed with one norm and one multiply per bucket instead of one per parameter."""
        # the bucket form only while every gradient still is a view of its bucket
        if not all(self._is_view(p) for p in self.params):
            return torch.nn.utils.clip_grad_norm_(self.params, max_norm)
        flats = [b.flat for b in self.buckets]
        total = torch.linalg.vector_norm(torch.stack(torch._foreach_norm(flats, 2.0)), 2.0)
        coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
        torch._foreach_mul_(flats, coef)
        return total

    def zero_grad(self) -> None:
        for b in self.buckets:
            b.flat.zero_()
            b.reset()
