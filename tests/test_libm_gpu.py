"""Device side of the libm pin: the glibc-exact tanhf / expm1f / expf restatements
(csrc/libm_glibc.h) evaluated by a HIP kernel (mhppo_libm_eval) on all 2^32 float bit patterns,
compared bit for bit with glibc's own functions (oracle_libm_eval, OpenMP), chunk by chunk.
Any NaN equals any NaN.  This is what makes the policy-driven rollout's discrete outputs
(Categorical draws, and the gap-acceptance decisions downstream of the continuous actions)
independent of device-vs-glibc ulps."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fn", [0, 1, 2], ids=["tanhf", "expm1f", "expf"])
def test_device_libm_matches_glibc_on_all_floats(fn):
    import oracle
    from mhppo import _lib
    L = _lib.lib()
    O = oracle.lib()
    O.oracle_libm_eval.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p]
    oracle.set_threads(16)
    n = 1 << 27
    dev = torch.empty(n, dtype=torch.float32, device="cuda")
    host = np.empty(n, np.float32)
    bad = 0
    first_bad = None
    for c in range((1 << 32) // n):
        _lib.check(L.mhppo_libm_eval(fn, c * n, n, _lib.ptr(dev), _lib.stream_ptr()))
        O.oracle_libm_eval(fn, c * n, n, host.ctypes.data_as(ctypes.c_void_p))
        g = dev.cpu().numpy()
        diff = (g.view(np.uint32) != host.view(np.uint32)) & ~(np.isnan(g) & np.isnan(host))
        k = int(diff.sum())
        if k and first_bad is None:
            i = int(np.nonzero(diff)[0][0])
            first_bad = (hex(c * n + i), hex(int(g.view(np.uint32)[i])), hex(int(host.view(np.uint32)[i])))
        bad += k
    assert bad == 0, (bad, first_bad)
