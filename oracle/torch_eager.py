"""The reference's q/dq as its own eager PyTorch op sequence, on the CPU (test / baseline
infrastructure only: bench.py's cpu_baseline leg times it; nothing in the package imports
it).  UniformAffineQuantizer.forward, /root/reference/quant/quant_layer.py:92-98:

    x_int = round_ste(x / delta) + zero_point          # round_ste: (t.round() - t).detach() + t
    x_quant = clamp(x_int, 0, n_levels - 1)             # (asymmetric; sym: +-n_levels/2)
    x_dequant = (x_quant - zero_point) * delta

eight elementwise ops (div, round, sub, add | + zp, clamp, - zp, * delta), each a full pass
over the tensor, as the reference runs them (quant_layer.py:18-22 for round_ste)."""
import torch


def uaq_fake_quant(x, delta, zero_point, n_bits, sym=False):
    n_levels = 2 ** n_bits
    t = x / delta
    x_int = ((t.round() - t).detach() + t) + zero_point
    if sym:
        x_quant = torch.clamp(x_int, -n_levels // 2, n_levels // 2 - 1)
    else:
        x_quant = torch.clamp(x_int, 0, n_levels - 1)
    return (x_quant - zero_point) * delta
