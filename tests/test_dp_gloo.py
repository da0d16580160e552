"""Data-parallel gradient sync (dp.BucketedAllReduce) on CPU with gloo,
world_size 2: DP-averaged gradients equal the single-process full-batch
gradients; no_sync accumulation; multiple buckets; unused parameters."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from differential_transformer_replication_amd.dp import BucketedAllReduce


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(16, 32)
        self.b = torch.nn.Linear(32, 32)
        self.unused = torch.nn.Linear(4, 4)
        self.c = torch.nn.Linear(32, 1)

    def forward(self, x):
        return self.c(torch.tanh(self.b(torch.tanh(self.a(x)))))


def _data():
    g = torch.Generator().manual_seed(0)
    return torch.randn(8, 16, generator=g), torch.randn(8, 1, generator=g)


def _worker(rank, world, port, accum, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(rank + 100)          # different init per rank: broadcast must fix it
    net = Net()
    sync = BucketedAllReduce(net, bucket_cap_mb=0.002)   # tiny cap -> several buckets
    assert len(sync.buckets) >= 3
    x, y = _data()
    xs, ys = x.chunk(world)[rank], y.chunk(world)[rank]
    if accum:
        for i, (xm, ym) in enumerate(zip(xs.chunk(2), ys.chunk(2))):
            ctx = sync.no_sync() if i == 0 else torch.enable_grad()
            with ctx:
                (torch.nn.functional.mse_loss(net(xm), ym) / 2).backward()
    else:
        torch.nn.functional.mse_loss(net(xs), ys).backward()
    sync.synchronize()
    # numpy, not tensors: a tensor in a Queue is shared through a socket of this
    # process, which may have exited by the time the parent unpickles it
    grads = {n: p.grad.clone().numpy() for n, p in net.named_parameters()}
    params = {n: p.detach().clone().numpy() for n, p in net.named_parameters()}
    out.put((rank, grads, params))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("accum", [False, True])
def test_dp_matches_full_batch(accum):
    world = 2
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, accum, out)) for r in range(world)]
    for p in procs:
        p.start()
    res = [out.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    # reference: rank 0's (broadcast) initial weights, full batch, one process
    torch.manual_seed(100)
    ref = Net()
    ref.load_state_dict({k: torch.from_numpy(v) for k, v in res[0][2].items()})
    x, y = _data()
    torch.nn.functional.mse_loss(ref(x), y).backward()
    for _, grads, params in res:
        for n, p in ref.named_parameters():
            assert (params[n] == res[0][2][n]).all(), n
            want = p.grad if p.grad is not None else torch.zeros_like(p)
            assert torch.allclose(torch.from_numpy(grads[n]), want, atol=1e-6, rtol=1e-5), n


# ---- the full Trainer (grad accumulation with no_sync, clip 1.0, AdamW, cosine warmup) ----
def _trainer_cfg(mb):
    from differential_transformer_replication_amd.train import TrainingConfig
    return TrainingConfig(model="control", vocab_size=61, n_embd=32, n_head=2, n_layer=2, block_size=16,
                          dropout=0.0, micro_batch_size=mb, grad_acc_steps=2, device="cpu", dtype="fp32",
                          warmup_iters=2, max_iters=20, learning_rate=1e-2, bucket_cap_mb=0.01)


def _trainer_batches(world, mb, steps=3, acc=2):
    g = torch.Generator().manual_seed(5)
    # [step][micro][rank] -> (X, Y)
    return [[[(torch.randint(0, 61, (mb, 16), generator=g), torch.randint(0, 61, (mb, 16), generator=g))
              for _ in range(world)] for _ in range(acc)] for _ in range(steps)]


def _trainer_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from differential_transformer_replication_amd.train import Trainer, build_model
    cfg = _trainer_cfg(2)
    torch.manual_seed(rank + 7)            # different init per rank: the DP layer broadcasts rank 0's
    model = build_model(cfg)
    tr = Trainer(cfg, model, world, rank, torch.device("cpu"))
    assert len(tr.sync.buckets) >= 2
    batches = _trainer_batches(world, 2)
    losses = []
    for step in batches:
        feed = iter(m[rank] for m in step)
        losses.append(float(tr.step(lambda: next(feed))))
    out.put((rank, {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}, losses))
    dist.barrier()
    dist.destroy_process_group()


def test_trainer_dp_matches_single_process():
    """Two gloo ranks, each with its half of every micro-batch, end at the same
    parameters as one process that sees the whole micro-batch (mean loss over
    equal shards = mean of the shard means)."""
    world = 2
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([out.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from differential_transformer_replication_amd.train import Trainer, build_model
    torch.manual_seed(7)                   # rank 0's initial weights
    cfg = _trainer_cfg(4)
    model = build_model(cfg)
    tr = Trainer(cfg, model, 1, 0, torch.device("cpu"))
    ref_losses = []
    for step in _trainer_batches(world, 2):
        feed = iter((torch.cat([r[0] for r in m]), torch.cat([r[1] for r in m])) for m in step)
        ref_losses.append(float(tr.step(lambda: next(feed))))
    for rank, sd, losses in res:
        for k, v in model.state_dict().items():
            assert torch.allclose(torch.from_numpy(sd[k]), v, atol=2e-5, rtol=1e-4), (rank, k)
    # each rank reports its own shard loss; their mean is the full-batch loss
    for s in range(len(ref_losses)):
        assert abs((res[0][2][s] + res[1][2][s]) / 2 - ref_losses[s]) < 1e-5


def test_bench_cpu_dry_run_two_ranks():
    """bench.py --gpus 2 --device cpu: the launcher spawns two gloo ranks and rank 0
    prints one JSON line for the whole job."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--steps", "2", "--warmup", "1"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["value"] > 0 and rec["config"]["global_batch"] == 8
    bad = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--device", "cpu"],
                         capture_output=True, text=True, timeout=120, env=dict(env, WORLD_SIZE="1"))
    assert bad.returncode == 2                # --gpus disagrees with the launcher's WORLD_SIZE


@pytest.mark.parametrize("scale", [0.01, 100.0])
def test_bucket_clip_matches_torch_clip(scale):
    """BucketedAllReduce.clip_grad_norm_ (one norm / multiply per bucket) gives the
    norm and the clipped gradients of torch.nn.utils.clip_grad_norm_ (train.py:273),
    below and above the max norm, over several buckets."""
    torch.manual_seed(0)
    ref, m = Net(), Net()
    m.load_state_dict(ref.state_dict())
    sync = BucketedAllReduce(m, bucket_cap_mb=0.002)
    assert len(sync.buckets) > 1
    x = torch.randn(8, 16)
    (ref(x).sum() * scale).backward()
    (m(x).sum() * scale).backward()
    for p in ref.parameters():
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    n_ref = torch.nn.utils.clip_grad_norm_(ref.parameters(), 1.0)
    n = sync.clip_grad_norm_(1.0)
    assert torch.allclose(n, n_ref, rtol=1e-6)
    for (k, a), (_, b) in zip(ref.named_parameters(), m.named_parameters()):
        assert torch.allclose(a.grad, b.grad, rtol=1e-6, atol=1e-9), k
