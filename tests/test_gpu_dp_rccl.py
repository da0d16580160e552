"""The DP gradient path over RCCL on the GPU (torch.distributed backend "nccl" is
RCCL on ROCm): a 1-rank process group with BucketedAllReduce forced to launch its
bucket all-reduces from the post-accumulate-grad hooks, overlapped with backward,
then synchronize().  Sum over one rank times 1/world = the gradients themselves, so
they must equal a run without DP bitwise (train.py's step structure)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist


pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bucketed_allreduce_over_rccl_single_rank():
    from differential_transformer_replication_amd import diff_transformer as D
    from differential_transformer_replication_amd.dp import BucketedAllReduce
    dev = torch.device("cuda", 0)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        def build():
            torch.manual_seed(0)
            return D.DiffTransformer(97, 64, 2, 2, 32, 0.0).to(dev)

        ref, m = build(), build()
        sync = BucketedAllReduce(m, bucket_cap_mb=0.05, reduce_single=True)
        assert len(sync.buckets) > 1
        g = torch.Generator().manual_seed(5)
        idx = torch.randint(0, 97, (2, 32), generator=g).to(dev)
        tgt = torch.randint(0, 97, (2, 32), generator=g).to(dev)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lr = ref(idx, tgt)[1]
            lm = m(idx, tgt)[1]
        lr.backward()
        lm.backward()
        launched = sum(b.handle is not None for b in sync.buckets)
        assert launched == len(sync.buckets)          # every bucket reduced from the hooks
        # ... each once all of its parameters had reported, each exactly once (a repeat raises)
        assert all(b.pending == 0 and len(b.seen) == b.size for b in sync.buckets)
        sync.synchronize()
        torch.cuda.synchronize()
        for (n, a), (_, b) in zip(ref.named_parameters(), m.named_parameters()):
            assert torch.equal(a.grad, b.grad), n
        sync.clip_grad_norm_(1.0)
        sync.zero_grad()
        assert all(float(b.flat.abs().max()) == 0.0 for b in sync.buckets)
    finally:
        dist.destroy_process_group()


def test_two_rank_packed_dp_on_one_gpu(tmp_path):
    """World size 2 through the packed DiffTransformer path (packed projection GEMMs,
    lambda packs and LayerNorms reporting to their buckets themselves, packing.bind_grad):
    two child processes share cuda:0 over a gloo group, each with half of the batch.
    Every parameter reports exactly once, every bucket launches from the backward hooks
    with all its gradients in, and the averaged gradients equal one process's on the
    whole batch (train.py:260-281 is the step this DP wraps)."""
    import subprocess
    import sys
    from differential_transformer_replication_amd import diff_transformer as D
    here = os.path.dirname(os.path.abspath(__file__))
    port = _port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    outs = [str(tmp_path / f"rank{r}.pt") for r in range(2)]
    procs = [subprocess.Popen([sys.executable, os.path.join(here, "_dp_worker.py"), str(r), "2", str(port), outs[r]],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), "\n".join(l[-3000:] for l in logs)
    res = [torch.load(o, weights_only=True) for o in outs]
    for r in res:
        assert all(v == 1 for v in r["reports"].values()), {k: v for k, v in r["reports"].items() if v != 1}
        assert all(r["launched"]) and all(r["complete"])
    for n in res[0]["init"]:                       # rank 0's parameters reached rank 1
        assert torch.equal(res[0]["init"][n], res[1]["init"][n]), n
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    ref = D.DiffTransformer(97, 64, 2, 2, 32, 0.0).to(dev)
    with torch.no_grad():
        for n, p in ref.named_parameters():
            if "lambda_" in n:
                p.normal_(0, 0.1, generator=torch.Generator(device=dev).manual_seed(11))
    g = torch.Generator().manual_seed(5)
    idx = torch.randint(0, 97, (4, 32), generator=g)
    tgt = torch.randint(0, 97, (4, 32), generator=g)
    loss = ref(idx.to(dev), tgt.to(dev))[1]
    loss.backward()
    assert abs((res[0]["loss"] + res[1]["loss"]) / 2 - float(loss)) < 1e-5
    for n, p in ref.named_parameters():
        want = p.grad.cpu()
        got = res[0]["grads"][n]
        assert torch.equal(got, res[1]["grads"][n]), n           # both ranks hold the same average
        scale = want.abs().max().item()
        assert (got - want).abs().max().item() <= 1e-4 * max(scale, 1e-12), n
