"""The sphere-packing GPU test's exact call (tests/test_gpu_parity.py::test_sphere_packing_bound_qd)
with the iteration log printed: python tools/sp_test_debug.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _clrsdp_pkg  # noqa: E402

pk = _clrsdp_pkg.load()
from clrsdp_amd import sphere_packing as S  # noqa: E402

res = S.Nsphere_packing_2point(3, 8, precision_words=4, duality_gap_threshold=5e-6,
                               primal_error_threshold=1e-15, dual_error_threshold=1e-8,
                               verbose=True, return_info=True)
print("status", res[-1].status, "bound", -res[9])
