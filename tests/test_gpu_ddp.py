"""End to end on the north star's path: a torch DistributedDataParallel training step whose gradient
buckets are all-reduced by this engine through a DDP comm hook (nccl_amd.ddp_comm_hook), 2 processes on the
one GPU. After identical steps from identical weights on different data, both ranks must hold identical
parameters, equal to a single-process reference step on the averaged gradient. `eager`: a wider model with
buckets of several MiB and NCCL_AMD_EAGER_REGISTER=-1, so the buckets run eager zero-copy;
`staged`: small buckets on the staged / LL kernels (the defaults)."""
import multiprocessing as mp
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(torch, wide):
    h = 1024 if wide else 256
    return torch.nn.Sequential(torch.nn.Linear(64, h), torch.nn.ReLU(), torch.nn.Linear(h, h), torch.nn.ReLU(),
                               torch.nn.Linear(h, 32)).cuda()


def _worker(rank, world, port, uid, q, wide):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NCCL_AMD_SPIN_TIMEOUT_MS="30000")
        if wide:
            os.environ["NCCL_AMD_EAGER_REGISTER"] = "-1"  # eager zero-copy across processes
            os.environ.update(NCCL_DEBUG="TRACE", NCCL_DEBUG_FILE=f"/tmp/nccl_amd_ddp_{os.getpid()}.log")
        import torch
        import torch.distributed as dist
        import nccl_amd
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        comm = nccl_amd.Communicator.init(world, rank, uid)
        torch.manual_seed(0)
        model = _model(torch, wide)
        # several buckets: 4 MiB ones for the wide model (above the 2 MiB one-shot range at n = 2: eager zero-copy), 10 KB ones otherwise
        ddp = torch.nn.parallel.DistributedDataParallel(model, bucket_cap_mb=4 if wide else 0.01)
        ddp.register_comm_hook(None, nccl_amd.ddp_comm_hook(comm))
        opt = torch.optim.SGD(ddp.parameters(), lr=0.1)
        g = torch.Generator(device="cuda").manual_seed(100 + rank)
        for _ in range(3):
            x = torch.randn(16, 64, device="cuda", generator=g)
            loss = ddp(x).square().mean()
            opt.zero_grad()
            loss.backward()
            opt.step()
        torch.cuda.synchronize()
        flat = torch.cat([p.detach().flatten() for p in model.parameters()]).cpu()
        err = comm.async_error()
        comm.destroy()
        zc = 0
        if wide:
            zc = open(os.environ["NCCL_DEBUG_FILE"]).read().count("AllReduce: registered zero-copy")
        q.put((rank, flat.numpy(), err, zc))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e), -1, 0))


@pytest.mark.parametrize("mode", ["staged", "eager"])
def test_ddp_step_through_engine(built, mode):
    wide = mode == "eager"
    import numpy as np
    import torch
    import nccl_amd
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = nccl_amd.get_unique_id()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, uid, q, wide)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(2):
        r, flat, err, zc = q.get(timeout=240)
        res[r] = (flat, err, zc)
    for p in ps:
        p.join(timeout=60)
    for r in range(2):
        assert not isinstance(res[r][0], str), res[r][0]
        assert res[r][1] == 0
        if wide:  # every step's large buckets ran zero-copy on the ranks' own bucket tensors
            assert res[r][2] >= 3, f"rank {r}: {res[r][2]} zero-copy AllReduces"
    a, b = res[0][0], res[1][0]
    assert np.array_equal(a, b), "ranks diverged"
    # single-process reference: same init, gradient = mean of the two ranks' gradients, same 3 steps
    torch.manual_seed(0)
    model = _model(torch, wide)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    gens = [torch.Generator(device="cuda").manual_seed(100 + r) for r in range(2)]
    for _ in range(3):
        xs = [torch.randn(16, 64, device="cuda", generator=gens[r]) for r in range(2)]
        grads = []
        for x in xs:
            model.zero_grad()
            model(x).square().mean().backward()
            grads.append([p.grad.clone() for p in model.parameters()])
        for p, g0, g1 in zip(model.parameters(), *grads):
            p.grad = (g0 + g1) * 0.5
        opt.step()
    ref = torch.cat([p.detach().flatten() for p in model.parameters()]).cpu().numpy()
    np.testing.assert_allclose(a, ref, rtol=1e-5, atol=1e-6)
