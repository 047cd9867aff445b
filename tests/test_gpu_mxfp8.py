"""MX-fp8 quantiser + GEMM (csrc/mxfp8.hip; SURVEY §8(d) configs[3] "fp8 attention and MLP
GEMMs").  The reference has no fp8 path (it runs fp32, ct_clip/attention.py:44-52, :88-181), so
per SURVEY §8(c) this path is compared to (1) a torch restatement of the OCP MX rule, bit-exact,
(2) an f64 matmul of the dequantised operands (rel 1e-4: the scaled MFMA's internal sum of 128
products is not f32-exact — measured 1.4e-5 at K = 128, 20x an f32 dot product's), and
(3) the build's own bf16 GEMM on the same bf16 inputs (quantisation error: rel 0.06, the e4m3
3-bit mantissa's ~2^-4 relative step on every operand)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = 'cuda'


@pytest.fixture(scope='module')
def K():
    from ctclip_mi355x import kernels
    return kernels


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def mx_ref(x, Kp):
    """Torch restatement of the quantiser: per 32-k block X = floor(log2 amax) - 8, q = e4m3
    RNE of clamp(x * 2^-X, +-448), scale byte X + 127; zero blocks get X = 0; k >= K zero."""
    rows, Kx = x.shape
    xf = torch.zeros(rows, Kp, device=x.device, dtype=torch.float32)
    xf[:, :Kx] = x.float()
    blk = xf.view(rows, Kp // 32, 32)
    amax = blk.abs().amax(-1)
    e = ((amax.view(torch.int32) >> 23) & 255)
    X = torch.where(e > 0, e - 127, torch.full_like(e, -127)) - 8
    X = torch.where(amax > 0, X.clamp(-127, 127), torch.zeros_like(X))
    mul = torch.pow(2.0, -X.double()).float()
    q = (blk * mul[..., None]).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8).view(rows, Kp)
    return q, (X + 127).to(torch.uint8)


def dequant(q, s):
    rows, Kp = q.shape
    v = q.view(torch.float8_e4m3fn).double().view(rows, Kp // 32, 32)
    return (v * torch.pow(2.0, s.double() - 127)[..., None]).view(rows, Kp)


@pytest.mark.parametrize('rows,Kx,dtype', [(300, 512, torch.bfloat16), (77, 1365, torch.bfloat16),
                                           (64, 256, torch.float32), (5, 130, torch.float32)])
def test_quant_bit_exact(K, rows, Kx, dtype):
    torch.manual_seed(1)
    x = (torch.randn(rows, Kx, device=dev) * torch.logspace(-6, 4, Kx, device=dev)).to(dtype)
    x[0, :64] = 0                                  # all-zero blocks
    x[1, 5] = 1e30 if dtype == torch.float32 else 3e38   # huge amax
    q, s = K.quant_mxfp8(x)
    Kp = (Kx + 127) // 128 * 128
    qr, sr = mx_ref(x, Kp)
    assert torch.equal(s, sr)
    assert torch.equal(q, qr), (q != qr).sum().item()


@pytest.mark.parametrize('tile', [128, 256])
@pytest.mark.parametrize('M,N,Kx', [(128, 128, 128), (300, 264, 384), (1000, 2730, 512), (257, 512, 1365),
                                    (96, 200, 256)])
def test_gemm_vs_dequantised_matmul(K, M, N, Kx, tile):
    prev = K.gemm_mxfp8_set_tile(tile)
    try:
        _check_gemm(K, M, N, Kx)
    finally:
        K.gemm_mxfp8_set_tile(prev)


def test_gemm_tiles_identical(K):
    torch.manual_seed(4)
    a, b = torch.randn(700, 640, device=dev).bfloat16(), torch.randn(392, 640, device=dev).bfloat16()
    qa, sa = K.quant_mxfp8(a)
    qb, sb = K.quant_mxfp8(b)
    outs = []
    for tile in (128, 256):
        prev = K.gemm_mxfp8_set_tile(tile)
        outs.append(K.gemm_mxfp8(qa, sa, qb, sb, out_f32=True))
        K.gemm_mxfp8_set_tile(prev)
    assert torch.equal(outs[0], outs[1])


def _check_gemm(K, M, N, Kx):
    torch.manual_seed(2)
    a = torch.randn(M, Kx, device=dev).bfloat16()
    b = (torch.randn(N, Kx, device=dev) * 0.05).bfloat16()
    bias = torch.randn(N, device=dev)
    qa, sa = K.quant_mxfp8(a)
    qb, sb = K.quant_mxfp8(b)
    ref = dequant(qa, sa) @ dequant(qb, sb).T
    c = K.gemm_mxfp8(qa, sa, qb, sb, out_f32=True, alpha=0.5)
    assert rel(c, 0.5 * ref) < 1e-4
    cb = K.gemm_mxfp8(qa, sa, qb, sb, bias=bias)
    assert cb.dtype == torch.bfloat16
    assert rel(cb, ref + bias.double()) < 4e-3        # bf16 output rounding


def test_gemm_asymmetric_identity(K):
    """A = I (exact in e4m3), asymmetric B: catches any row / column swap in the C write."""
    n = 256
    a = torch.eye(n, device=dev)
    b = (torch.arange(n * n, device=dev, dtype=torch.float32).view(n, n) % 17 - 8)
    qa, sa = K.quant_mxfp8(a)
    qb, sb = K.quant_mxfp8(b)
    c = K.gemm_mxfp8(qa, sa, qb, sb, out_f32=True)
    assert torch.equal(c, b.T.contiguous())


def test_mxfp8_vs_bf16_path(K):
    """FF1-shaped product (LN output x W1^T): the fp8 path against the bf16 GEMM of the build."""
    torch.manual_seed(3)
    x = torch.randn(2048, 512, device=dev).bfloat16()
    w = (torch.randn(2730, 512, device=dev) * 512 ** -0.5).bfloat16()
    ref = x.float() @ w.float().T
    qx, sx = K.quant_mxfp8(x)
    qw, sw = K.quant_mxfp8(w)
    c = K.gemm_mxfp8(qx, sx, qw, sw, out_f32=True)
    assert rel(c, ref) < 0.06
