import ctypes, sys
from pathlib import Path
import numpy as np
sys.path.insert(0, "/root/repo")
import orb_slam_amd as ox
L = ox.lib()
L.orbx_debug_llt_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
nb = 20; n = 6 * nb
rng = np.random.default_rng(nb)
A = rng.standard_normal((n, n)); H = A @ A.T + n * np.eye(n); b = rng.standard_normal(n)
packed = np.concatenate([H[i, :i + 1] for i in range(n)] + [b])
x = np.zeros(n); c = ctypes.c_ulonglong(0)
assert L.orbx_debug_llt_bench(packed.ctypes.data, n, 100, x.ctypes.data, ctypes.byref(c), 0) == 0
print("cycles per solve", c.value / 100)
