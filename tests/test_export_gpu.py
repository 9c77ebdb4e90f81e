"""Packed low-bit export (K15 ssq_pack_encode / K16 ssq_pack_decode, quant/export.py):
the codes are the quantizer's own integer codes in the documented bit layout, decoding
reproduces every quantizer's hard W_hat bit for bit, soft weights are refused, and a
calibrated model restored from the export computes the same outputs bit for bit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from shiftedscalequantization_amd import kernels
    return kernels


def host(t):
    return t.detach().cpu().numpy()


def unpack_host(packed, n, n_bits, qmin):
    """The documented layout restated on the host: code e at bits [e*bs, (e+1)*bs) of a
    little-endian stream, stored as q - qmin."""
    bs = 2 if n_bits <= 2 else (4 if n_bits <= 4 else 8)
    raw = np.unpackbits(host(packed), bitorder="little")
    u = raw[: n * bs].reshape(n, bs) @ (1 << np.arange(bs))
    return u.astype(np.int64) + qmin


@pytest.mark.parametrize("n_bits", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("shape", [(16, 8, 3, 3), (7, 5, 1, 1), (10, 3), (33, 1, 3, 3)])
def test_pack_roundtrip_uaq(K, n_bits, sym, shape):
    g = torch.Generator().manual_seed(n_bits * 10 + sym + len(shape))
    w = (torch.randn(shape, generator=g) * 0.1).cuda()
    d, z, _ = K.scale_init(w, n_bits, sym, True, "max")
    what, codes = K.fake_quant_fwd(w, d, z, n_bits, sym, codes=True)
    qmin, qmax = K.qrange(n_bits, sym)
    Co = shape[0]
    packed, bad = K.pack_encode(what, z.reshape(-1), d.reshape(-1), False, None, n_bits, qmin, qmax)
    assert bad == 0
    q = unpack_host(packed, w.numel(), n_bits, qmin)
    ref = host(codes).astype(np.int64).reshape(-1)
    if sym:
        ref = host(codes.view(torch.int8)).astype(np.int64).reshape(-1)
    np.testing.assert_array_equal(q, ref)
    back = K.pack_decode(packed, shape, z.reshape(-1), d.reshape(-1), False, None, n_bits, qmin)
    np.testing.assert_array_equal(host(back).view(np.int32), host(what).view(np.int32))
    assert packed.numel() == ((w.numel() + 3) // 4) * ({1: 2, 2: 2, 3: 4, 4: 4}.get(n_bits, 8) // 2)
    del Co


def test_pack_refuses_soft_weights(K):
    w = torch.randn(8, 4, 3, 3).cuda()
    d, z, _ = K.scale_init(w, 2, False, True, "max")
    _, bad = K.pack_encode(w, z.reshape(-1), d.reshape(-1), False, None, 2, 0, 3)
    assert bad > 0


def test_pack_per_ci_and_col_scale(K):
    """(q - zp) * d1[co, ci] (* d2[j]) layouts: learned_hard_sigmoid's per-(co,ci) delta
    and ChannelQuantMSE's column scale."""
    g = torch.Generator().manual_seed(4)
    Co, Ci, k = 12, 6, 9
    q = torch.randint(0, 4, (Co, Ci, 3, 3), generator=g).float().cuda()
    zp = torch.randint(0, 4, (Co,), generator=g).float().cuda()
    d1 = (torch.rand(Co, Ci, generator=g) * 0.01 + 1e-3).cuda()
    d2 = (torch.rand(Ci * k, generator=g) + 0.5).cuda()
    what = ((q - zp.view(-1, 1, 1, 1)) * d1.view(Co, Ci, 1, 1)) * d2.view(1, Ci, 3, 3)
    packed, bad = K.pack_encode(what, zp, d1, True, d2, 2, 0, 3)
    assert bad == 0
    np.testing.assert_array_equal(unpack_host(packed, what.numel(), 2, 0), host(q).astype(np.int64).reshape(-1))
    back = K.pack_decode(packed, what.shape, zp, d1, True, d2, 2, 0)
    np.testing.assert_array_equal(host(back).view(np.int32), host(what).view(np.int32))


def test_export_restores_calibrated_model_bit_exactly(K, tmp_path):
    """README flow (shifted-scale weight recon + bias_cal, BRECQ fc, act recon) at a few
    iterations; export -> safetensors -> a fresh random-init QuantModel -> same outputs."""
    import main_imagenet
    from shiftedscalequantization_amd import drivers as D
    from shiftedscalequantization_amd.quant import export_quantized, load_quantized
    qnn = main_imagenet.main(["--arch", "resnet18", "--n_bits_w", "2", "--n_bits_a", "4",
                              "--bias_cal", "True", "--bias_ch_quant", "True", "--num_samples", "64",
                              "--shift_iters", "6", "--iters_w", "6", "--iters_a", "6"])
    qnn.eval()
    path = str(tmp_path / "r18_w2a4.safetensors")
    tensors, meta = export_quantized(qnn, path)
    kinds = {v["kind"] for v in __import__("json").loads(meta["layers"]).values() if "kind" in v}
    assert "channelquant:adaShift" in kinds and any(k.startswith("adaround") for k in kinds)
    n_w = sum(m.weight.numel() for m in qnn.modules() if hasattr(m, "weight_quantizer"))
    n_code_bytes = sum(v.numel() for k, v in tensors.items() if k.endswith(".codes"))
    assert n_code_bytes < n_w * 0.3          # 2-bit body, 8-bit stem/head
    torch.manual_seed(12345)
    fresh = D.build_qnn("resnet18", 2, 4, device="cuda")
    load_quantized(fresh, path)
    fresh.set_quant_state(True, True)
    fresh.eval()
    x = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(9)).cuda()
    with torch.no_grad():
        a, b = qnn(x), fresh(x)
    np.testing.assert_array_equal(host(a).view(np.int32), host(b).view(np.int32))
