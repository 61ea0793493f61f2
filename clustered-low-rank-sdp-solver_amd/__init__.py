"""MI355X-native interior-point step for clustered low-rank SDPs (MPMP.jl's hot path).

Public API mirrors MPMP.jl (exports at MPMP.jl:19): ``solverank1sdp``, ``get_block_info``,
``BlockInfo``; plus :class:`DeviceSolver`, the handle over the C ABI in ``include/clrsdp.h``.
"""
from .blockinfo import BlockInfo, block_info, distribute_weights_swapping, get_block_info, \
    partition_clusters
from .instance import SPHERE_PACKING_SHAPE, Cluster, synth, synth_mixed
from .solver import DeviceSolver, initial_point, make_params, solverank1sdp
from . import _lib

__all__ = ["BlockInfo", "block_info", "get_block_info", "distribute_weights_swapping",
           "partition_clusters", "Cluster", "synth", "synth_mixed", "SPHERE_PACKING_SHAPE", "DeviceSolver", "initial_point",
           "make_params", "solverank1sdp"]
