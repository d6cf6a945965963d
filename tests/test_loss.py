"""Fused MSE loss (xdot/ops/loss.py, csrc/reduce.hip::mse_fwd_kernel) vs torch.nn.functional.mse_loss."""
import pytest
import torch
import torch.nn.functional as F

import xdot
from xdot.ops.loss import mse_loss


def _check(dev, dt, shape, tol):
    g = torch.Generator(device="cpu").manual_seed(7)
    y0 = torch.randn(*shape, generator=g)
    t0 = torch.randn(*shape, generator=g)
    y = y0.to(dev, dt).requires_grad_()
    t = t0.to(dev, dt).requires_grad_()
    loss = mse_loss(y, t)
    (3.0 * loss).backward()
    yr = y.detach().float().cpu().double().requires_grad_()
    tr = t.detach().float().cpu().double().requires_grad_()
    ref = F.mse_loss(yr, tr)
    (3.0 * ref).backward()
    assert loss.dtype == dt and loss.shape == ()
    assert abs(loss.double().item() - ref.item()) <= tol * ref.item()
    for a, b in ((y.grad, yr.grad), (t.grad, tr.grad)):
        err = (a.double().cpu() - b).abs().max().item()
        assert err <= tol * b.abs().max().item() + 1e-12, err


def test_mse_cpu_matches_torch():
    _check("cpu", torch.float32, (3, 50, 16), 1e-6)
    assert isinstance(xdot.MSELoss()(torch.ones(4), torch.zeros(4)), torch.Tensor)


@pytest.mark.gpu
@pytest.mark.parametrize("dt,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2), (torch.float16, 3e-2)])
@pytest.mark.parametrize("shape", [(1, 3125, 768), (2, 1000, 96), (5, 7)])
def test_mse_gpu_matches_torch(gpu, dt, tol, shape):
    """(5, 7): 35 elements, not a multiple of the 16-byte vector -> torch path; the others run
    the HIP kernel (1024 workgroup partials at the largest shape)"""
    _check(gpu, dt, shape, tol)


@pytest.mark.gpu
def test_mse_gpu_deterministic(gpu):
    y = torch.randn(1, 25000, 768, device=gpu, dtype=torch.bfloat16)
    t = torch.randn(1, 25000, 768, device=gpu, dtype=torch.bfloat16)
    a = mse_loss(y, t)
    b = mse_loss(y, t)
    assert torch.equal(a, b)


def test_unit_grad_seed_matches_default_backward():
    """loss.backward(unit_grad(loss)) == loss.backward() (CPU: torch path; the seed is exact 1)."""
    import xdot
    from xdot.ops.loss import unit_grad

    g = torch.Generator().manual_seed(3)
    y0, t = torch.randn(4, 33, generator=g), torch.randn(4, 33, generator=g)
    a = y0.clone().requires_grad_(True)
    b = y0.clone().requires_grad_(True)
    xdot.MSELoss()(a, t).backward()
    lb = xdot.MSELoss()(b, t)
    lb.backward(unit_grad(lb))
    assert torch.equal(a.grad, b.grad)
    assert unit_grad(lb) is unit_grad(lb)


@pytest.mark.gpu
def test_unit_grad_seed_gpu(gpu):
    """HIP path: the exact-1 seed hands the kernel's saved gradient on unscaled — bitwise equal
    to the default backward (dy * 1)."""
    import xdot
    from xdot.ops.loss import unit_grad

    y0 = torch.randn(1, 3125, 768, device=gpu, dtype=torch.bfloat16)
    t = torch.randn(1, 3125, 768, device=gpu, dtype=torch.bfloat16)
    a = y0.clone().requires_grad_(True)
    b = y0.clone().requires_grad_(True)
    xdot.MSELoss()(a, t).backward()
    lb = xdot.MSELoss()(b, t)
    lb.backward(unit_grad(lb))
    assert torch.equal(a.grad, b.grad)
