"""BRECQ layer reconstruction (reference: quant/layer_recon.py): block_reconstruction's
algorithm on a single QuantModule (first/last layers of a network)."""
import torch

from .block_recon import LinearTempDecay, LossFunction, _reconstruct  # noqa: F401
from .quant_layer import QuantModule
from .quant_model import QuantModel


def layer_reconstruction(model: QuantModel, layer: QuantModule, cali_data: torch.Tensor,
                         batch_size: int = 32, iters: int = 20000, weight: float = 0.001,
                         opt_mode: str = 'mse', asym: bool = False, include_act_func: bool = True,
                         b_range: tuple = (20, 2), warmup: float = 0.0, act_quant: bool = False,
                         lr: float = 4e-5, p: float = 2.0, multi_gpu: bool = False,
                         eval: bool = False, dp_average: bool = False):
    """layer_recon.py:10-104 (its gradient all-reduce is commented out in the reference;
    it is active here when multi_gpu or a process group is initialised)."""
    return _reconstruct(model, layer, [layer], cali_data, batch_size, iters, weight, opt_mode, asym,
                        include_act_func, b_range, warmup, act_quant, lr, p, multi_gpu, eval,
                        dp_average, block_level=False)
