"""Numerics of the gfx950 kernels against plain PyTorch references (run with -m gpu)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from rabit_amd import ops  # noqa: E402

INT_TYPES = [torch.int8, torch.uint8, torch.int32, torch.int64]
FLOAT_TYPES = [torch.float32, torch.float64]


def _rand(n, dtype, dev, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    if dtype.is_floating_point:
        return torch.randn(n, generator=g, dtype=torch.float64).to(dtype).to(dev)
    lo, hi = (0, 100) if dtype == torch.uint8 else (-50, 50)
    return torch.randint(lo, hi, (n,), generator=g, dtype=torch.int64).to(dtype).to(dev)


def _ref(op, a, b):
    if op == ops.SUM:
        return (a.double() + b.double()) if a.dtype.is_floating_point else a + b
    if op == ops.MAX:
        return torch.maximum(a, b)
    if op == ops.MIN:
        return torch.minimum(a, b)
    return a | b


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("dtype", FLOAT_TYPES + INT_TYPES)
@pytest.mark.parametrize("op", [ops.SUM, ops.MAX, ops.MIN, ops.BITOR])
@pytest.mark.parametrize("n", [1, 37, 4096 + 3, 1 << 20])
def test_reduce2(dev, dtype, op, n):
    if op == ops.BITOR and dtype.is_floating_point:
        pytest.skip("BitOR undefined for floats")
    a, b = _rand(n, dtype, dev, 1), _rand(n, dtype, dev, 2)
    expect = _ref(op, a, b)
    ops.reduce_(a, b, op)
    torch.cuda.synchronize()
    if dtype.is_floating_point:
        torch.testing.assert_close(a.double(), expect.double(), rtol=1e-6, atol=1e-6)
    else:
        assert torch.equal(a, expect.to(dtype))


def test_reduce2_unaligned(dev):
    base_a, base_b = _rand(1001, torch.float32, dev, 3), _rand(1001, torch.float32, dev, 4)
    a, b = base_a[1:], base_b[1:]  # 4-byte offset: scalar path
    expect = a.double() + b.double()
    ops.reduce_(a, b, ops.SUM)
    torch.cuda.synchronize()
    torch.testing.assert_close(a.double(), expect, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("op", [ops.SUM, ops.MAX, ops.BITOR])
def test_reduce_multi(dev, k, op):
    dtype = torch.int32 if op == ops.BITOR else torch.float32
    n = 3 * 4096 + 5
    srcs = [_rand(n, dtype, dev, 10 + i) for i in range(k)]
    expect = srcs[0].clone()
    for s in srcs[1:]:
        expect = _ref(op, expect, s).to(dtype)
    out = torch.empty_like(srcs[0])
    ops.reduce_multi(out, srcs, op)
    torch.cuda.synchronize()
    if dtype.is_floating_point:
        torch.testing.assert_close(out, expect, rtol=1e-5, atol=1e-5)
    else:
        assert torch.equal(out, expect)


@pytest.mark.parametrize("prep,fn", [(ops.PREP_COPY, lambda x: x), (ops.PREP_SQUARE, lambda x: x * x),
                                     (ops.PREP_SCALE, lambda x: x * 0.5),
                                     (ops.PREP_ABS, lambda x: x.abs())])
def test_prepare(dev, prep, fn):
    src = _rand(1 << 16, torch.float32, dev, 7)
    dst, dst2 = torch.empty_like(src), torch.empty_like(src)
    ops.prepare(dst, src, prep, alpha=0.5, dst2=dst2)
    torch.cuda.synchronize()
    torch.testing.assert_close(dst, fn(src))
    torch.testing.assert_close(dst2, fn(src))


@pytest.mark.parametrize("n", [4, 12344, 1 << 20])
def test_checksum(dev, n):
    x = _rand(n, torch.int32, dev, 9)
    got = ops.checksum(x).cpu().numpy().view(np.uint64)
    w = x.cpu().numpy().view(np.uint32).astype(np.uint64).reshape(-1, 4)
    s1 = np.sum(w, dtype=np.uint64)
    q = w[:, 0] + 2 * w[:, 1] + 3 * w[:, 2] + 4 * w[:, 3]
    s2 = np.sum(q * np.arange(1, w.shape[0] + 1, dtype=np.uint64), dtype=np.uint64)
    assert got[0] == s1 and got[1] == s2


def test_checksum_detects_swap(dev):
    x = _rand(4096, torch.int32, dev, 11)
    y = x.clone()
    y[[0, 4]] = y[[4, 0]]
    if torch.equal(x, y):
        pytest.skip("degenerate data")
    assert not torch.equal(ops.checksum(x), ops.checksum(y))


@pytest.mark.parametrize("nbytes", [16, 1000, (1 << 20) + 8])
def test_copy_kernel(dev, nbytes):
    src = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device=dev)
    dst = torch.zeros_like(src)
    ops.copy(dst, src)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)


def test_fill(dev):
    x = torch.empty(1000, dtype=torch.float64, device=dev)
    ops.fill(x, 2.5)
    torch.cuda.synchronize()
    assert torch.all(x == 2.5)
