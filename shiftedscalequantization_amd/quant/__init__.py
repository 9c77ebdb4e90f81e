"""Python mirror of the reference's quant/ package (same module, class and function
names).  The arithmetic of every quantizer, loss and regulariser runs in libssq.so."""
from .quant_layer import QuantModule, StraightThrough, UniformAffineQuantizer, lp_loss, round_ste
from .quant_block import (BaseQuantBlock, QuantBasicBlock, QuantBottleneck, QuantInvertedResidual,
                          QuantResBottleneckBlock, specials)
from .quant_model import QuantModel
from .channelQuant import ChannelQuant
from .channelQuantAct import ChannelQuantAct
from .channelQuantMSE import ChannelQuantMSE
from .adaptive_rounding import AdaRoundQuantizer
from .block_recon import block_reconstruction
from .layer_recon import layer_reconstruction
from .layer_recon_fused_shiftedScale import (FusedLinearTempDecayShift, FusedScaleLossFunction,
                                             block_recon_fused_shiftedScale,
                                             layer_recon_fused_shiftedScale, print_ratio)
from .layer_recon_shiftedScale import (LinearTempDecayShift, ScaleLossBlockFunction,
                                       ScaleLossFunction, block_recon_shiftedScale,
                                       layer_recon_shiftedScale)
from .data_utils import save_inp_oup_data, save_grad_data
from .export import PackedWeight, dequant_form, export_quantized, load_quantized
