"""MI355X-native shifted-scale PTQ calibration path (jai1215snu/ShiftedScaleQuantization).

Hot path: hand-written HIP kernels for gfx950 in libssq.so (C ABI: include/ssq.h),
reached through shiftedscalequantization_amd._capi / .kernels, behind a Python mirror
of the reference's quantizer API (shiftedscalequantization_amd.quant).
"""
__version__ = "0.1.0"
