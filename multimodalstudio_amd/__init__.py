"""MMS-AMD: an MI355X-native (gfx950 HIP) implementation of MultimodalStudio's per-ray training hot path.

The hot path (ray generation -> sphere collider -> NeuS sampler -> hash grid -> SDF MLP with
numerical-gradient taps -> radiance MLP -> modality heads -> NeuS alpha + composite) runs in the
C-ABI library ``libmms_hip.so`` (include/mms_hip.h); the Python modules here mirror the reference's
plugin surface (Encoding / FieldComponent / fields / samplers / renderer) and drive those kernels.
"""
__version__ = "0.1.0"
