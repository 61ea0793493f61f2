"""MI355X-native interior-point step for clustered low-rank SDPs (MPMP.jl's hot path).

Public API mirrors MPMP.jl (exports at MPMP.jl:19): ``solverank1sdp``, ``get_block_info``,
``BlockInfo``; plus :class:`DeviceSolver`, the handle over the C ABI in ``include/clrsdp.h``.
"""
from .blockinfo import BlockInfo, block_info, distribute_weights_swapping, get_block_info, \
    partition_clusters
from .instance import SPHERE_PACKING_SHAPE, Cluster, synth, synth_C, synth_mixed, synth_start
from .solver import DeviceSolver, compute_step_length, eigmin, initial_point, make_params, solverank1sdp
from .poly import Poly, create_sample_points, create_sample_points_1d, create_sample_points_2d, \
    create_sample_points_3d, create_sample_points_chebyshev, create_sample_points_chebyshev_mod, \
    gegenbauer_basis, jacobi_basis, laguerrebasis, make_monomial_basis, points_X_general
from .prep import prepareabc, solvempmp
from .sdpfiles import read_files, write_files
from .sphere_packing import Nsphere_packing_2point, test_bound_sphere_packing
from . import _lib

__all__ = ["BlockInfo", "block_info", "get_block_info", "distribute_weights_swapping",
           "partition_clusters", "Cluster", "synth", "synth_mixed", "synth_C", "synth_start", "SPHERE_PACKING_SHAPE", "DeviceSolver", "initial_point",
           "make_params", "solverank1sdp", "compute_step_length", "eigmin", "prepareabc", "solvempmp", "Poly", "laguerrebasis",
           "jacobi_basis", "gegenbauer_basis", "make_monomial_basis", "create_sample_points",
           "create_sample_points_1d", "create_sample_points_2d", "create_sample_points_3d",
           "create_sample_points_chebyshev", "create_sample_points_chebyshev_mod", "points_X_general", "write_files", "read_files",
           "Nsphere_packing_2point", "test_bound_sphere_packing"]
