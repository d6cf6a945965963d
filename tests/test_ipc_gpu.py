"""Native xGMI pull collectives (``xdot/utils/ipc.py``, ``csrc/ipc.hip``) on one MI355X.

Two (or three) processes share the box's single GPU: each exports its staging buffer and signal
page with hipIpcGetMemHandle and maps the others' — the same code path as one process per GPU
over xGMI, only the links are local HBM here (bandwidth over xGMI is not measured on a 1-GPU
box).  gloo carries the handle exchange and every fallback route.  Checked:

* all-gather: exact bytes for bf16 / fp32 / fp16, 16-byte and misaligned views, shards from
  16 bytes to 6 MB, many consecutive collectives (both staging slots reused repeatedly);
* reduce-scatter: bitwise equal to the fp32 sum in rank order 0..N-1 rounded once;
* routing: 1-byte dtypes and blocks that are not a multiple of 16 bytes take the wrapped
  communicator and still agree;
* the flash attention module (forward + backward + gradient sync) through IpcComm agrees with
  the same step through the wrapped communicator;
* a peer that skips a collective makes the device waits expire: the kernel drains and the next
  host call raises IpcError instead of hanging.
"""
import pytest
import torch

from _dist import run_gloo

pytestmark = pytest.mark.gpu


def _data(rank, shape, dtype, salt=0):
    g = torch.Generator().manual_seed(1000 * rank + salt)
    return torch.randn(*shape, generator=g).to(dtype)


def _collectives_case(rank, ws):
    import xdot.utils.comm as C
    from xdot.utils.ipc import IpcComm

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = IpcComm(C.get_comm(), capacity_mb=64, timeout_s=20)
    salt = 0
    for rep in range(3):
        for dtype, shape in [(torch.bfloat16, (1000, 768)), (torch.float32, (333, 96)), (torch.float16, (8,)),
                             (torch.bfloat16, (3125, 1024)), (torch.float32, (4,))]:
            salt += 1
            mine = _data(rank, shape, dtype, salt)
            out = torch.empty((ws,) + shape, dtype=dtype, device=dev)
            comm.all_gather_into(out, mine.to(dev))
            exp = torch.stack([_data(r, shape, dtype, salt) for r in range(ws)])
            torch.cuda.synchronize()
            assert torch.equal(out.cpu(), exp), (rep, dtype, shape)
        # in place: the input is this rank's block of the output (the fused module's [q|v]
        # projection writes it there); the kernel skips its own-block copy
        salt += 1
        shape = (1000, 768)
        out = torch.full((ws,) + shape, float("nan"), dtype=torch.bfloat16, device=dev)
        out[rank].copy_(_data(rank, shape, torch.bfloat16, salt).to(dev))
        comm.all_gather_into(out, out[rank])
        exp = torch.stack([_data(r, shape, torch.bfloat16, salt) for r in range(ws)])
        torch.cuda.synchronize()
        assert torch.equal(out.cpu(), exp), (rep, "in place")
        # misaligned input and output views (offset by one element)
        salt += 1
        n = 4096
        buf = torch.zeros(n + 1, dtype=torch.bfloat16, device=dev)
        buf[1:] = _data(rank, (n,), torch.bfloat16, salt).to(dev)
        obuf = torch.zeros(ws * n + 1, dtype=torch.bfloat16, device=dev)
        comm.all_gather_into(obuf[1:], buf[1:])
        exp = torch.cat([_data(r, (n,), torch.bfloat16, salt) for r in range(ws)])
        torch.cuda.synchronize()
        assert torch.equal(obuf[1:].cpu(), exp)
        # reduce-scatter: fp32 sum in rank order, one rounding
        for dtype, blk in [(torch.bfloat16, (3125, 96)), (torch.float32, (100, 8)), (torch.float16, (64,))]:
            salt += 1
            inp = _data(rank, (ws,) + blk, dtype, salt)
            out = torch.empty(blk, dtype=dtype, device=dev)
            comm.reduce_scatter(out, inp.to(dev))
            acc = torch.zeros(blk, dtype=torch.float32)
            for r in range(ws):
                acc += _data(r, (ws,) + blk, dtype, salt)[rank].float()
            torch.cuda.synchronize()
            assert torch.equal(out.cpu(), acc.to(dtype)), (rep, dtype, blk)
    # routed to the wrapped communicator: 1-byte dtype, 6-byte blocks
    salt += 1
    u8 = (_data(rank, (37,), torch.float32, salt) > 0).to(torch.uint8)
    out = torch.empty(ws, 37, dtype=torch.uint8, device=dev)
    comm.all_gather_into(out, u8.to(dev))
    exp = torch.stack([(_data(r, (37,), torch.float32, salt) > 0).to(torch.uint8) for r in range(ws)])
    assert torch.equal(out.cpu(), exp)
    odd = _data(rank, (3,), torch.bfloat16, salt)
    out = torch.empty(ws, 3, dtype=torch.bfloat16, device=dev)
    comm.all_gather_into(out, odd.to(dev))
    assert torch.equal(out.cpu(), torch.stack([_data(r, (3,), torch.bfloat16, salt) for r in range(ws)]))
    comm.check()
    assert comm.epoch >= 20
    comm.close()


@pytest.mark.parametrize("ws", [2, 3])
def test_ipc_collectives(gpu, ws):
    run_gloo(_collectives_case, ws, timeout=300)


def _module_case(rank, ws):
    import xdot
    import xdot.utils.comm as C
    from xdot.parallel import GradSync
    from xdot.utils.ipc import IpcComm

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    base = C.get_comm()
    ipc = IpcComm(base, capacity_mb=32, timeout_s=20)

    def step(comm):
        torch.manual_seed(0)
        m = xdot.DistributedDotProductAttn(256, num_heads=4, impl="flash", comm=comm).to(dev, torch.bfloat16)
        sync = GradSync(m, comm=comm, bucket_mb=0.05)
        g = torch.Generator().manual_seed(7 + rank)
        R = 384
        x = torch.randn(1, R, 256, generator=g).to(dev, torch.bfloat16).requires_grad_(True)
        mask = (torch.rand(1, R, R * ws, generator=torch.Generator().manual_seed(3 + rank)) < 0.2).to(dev)
        mask[..., 0] = False
        out = m(x, x, x, mask)
        out.float().square().sum().backward()
        sync.wait()
        torch.cuda.synchronize()
        return [out.float().cpu(), x.grad.float().cpu()] + [p.grad.float().cpu() for p in m.parameters()]

    ref = step(base)
    got = step(ipc)
    # the forward gathers are exact copies either way: identical outputs
    assert torch.equal(ref[0], got[0])
    for a, b in zip(ref[1:], got[1:]):  # reductions: gloo's vs rank-ordered fp32 sums
        err = (a - b).norm() / (a.norm() + 1e-12)
        assert err < 2e-2, err
    ipc.close()


def test_ipc_module_step(gpu):
    run_gloo(_module_case, 2, timeout=300)


def _timeout_case(rank, ws):
    import xdot.utils.comm as C
    from xdot.utils.ipc import IpcComm, IpcError

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = IpcComm(C.get_comm(), capacity_mb=4, timeout_s=1.5)
    x = torch.ones(4096, dtype=torch.bfloat16, device=dev)
    out = torch.empty(ws, 4096, dtype=torch.bfloat16, device=dev)
    comm.all_gather_into(out, x)  # both ranks
    torch.cuda.synchronize()
    comm.check()
    if rank == 0:  # rank 1 never joins this one: every wait of rank 0 expires, the grid drains
        out.zero_()
        comm.all_gather_into(out, x)
        torch.cuda.synchronize()
        # the missing peer's block is NaN (never stale or zero), our own block is intact
        assert torch.isnan(out[1].float()).all() and torch.equal(out[0], x)
        with pytest.raises(IpcError):
            comm.check()
    C.get_comm().barrier()


def test_ipc_peer_timeout_raises(gpu):
    run_gloo(_timeout_case, 2, timeout=120)


def _async_case(rank, ws):
    """async_op=True returns before the pull completes: the kernel runs on the communication
    stream, the handle's event is pending while the peer has not arrived, and wait() orders
    the caller's stream after it (the data is then exact)."""
    import time

    import xdot.utils.comm as C
    from xdot.utils.ipc import IpcComm

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = IpcComm(C.get_comm(), capacity_mb=8, timeout_s=60)
    x = torch.full((8192,), float(rank + 1), dtype=torch.bfloat16, device=dev)
    out = torch.empty(ws, 8192, dtype=torch.bfloat16, device=dev)
    C.get_comm().barrier()
    if rank == 1:
        time.sleep(3.0)  # rank 0's kernel must still be waiting for us
    h = comm.all_gather_into(out, x, async_op=True)
    if rank == 0:
        time.sleep(0.5)
        assert not h._work.is_completed(), "the pull finished before the peer arrived"
        # the caller's stream is free meanwhile: this runs while the pull kernel waits
        y = (x.float() * 2).sum()
        torch.cuda.current_stream().synchronize()
        assert float(y) == 2.0 * 8192
    got = h.wait()
    torch.cuda.synchronize()
    assert got is out and torch.equal(out[0], torch.full_like(x, 1.0)) and torch.equal(out[1], torch.full_like(x, 2.0))
    comm.close()


def test_ipc_async_handle_overlaps(gpu):
    run_gloo(_async_case, 2, timeout=120)
