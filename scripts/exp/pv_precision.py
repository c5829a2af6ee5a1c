"""Driver of scripts/exp/pv_precision.cpp: per mode (bits: 1 covariance predict, 2 gains, 4 state correct, 8 covariance
correct, 16 state predict in f32; 0 = all f64 = the shipped pv_step), max error vs the reference's f64 golden
run over 28 steps, as the ratio (reference f32 run's error) / (this mode's error).  The GPU test demands >= 100."""
import ctypes, numpy as np, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__)))))
from tests.hip_helpers import pack_sym, unpack_sym
from oracle import quad_oracle as Q
lib = ctypes.CDLL('/tmp/libpvm.so')
V=ctypes.c_void_p
lib.pv_batch.argtypes=[ctypes.c_int, ctypes.c_int, V, V, V, V, ctypes.c_float, V, V, V, V]
g = np.load(__import__('os').path.join(sys.path[0], 'tests', 'golden', 'pvfilter.npz'))
def relerr(a, b):
    a = a.reshape(a.shape[0], -1); b = b.reshape(b.shape[0], -1)
    return float((np.abs(a - b).max(1) / np.maximum(1.0, np.abs(b).max(1))).max())
P = lambda a: a.ctypes.data
import itertools
MODES=[0,1,2,4,8,16,31,2|4|16,1|2|4|16,8|16,1|16]
for seed in range(3):
    res = {}
    for f32 in MODES:
        x = np.ascontiguousarray(g[f"s{seed}_x0"], np.float32); n = x.shape[0]
        Pm = np.ascontiguousarray(pack_sym(np.broadcast_to(np.eye(9) * Q.PV_P0, (n, 9, 9)), 9), np.float32)
        e = [0, 0, 0, 0]
        for step in range(g[f"s{seed}_acc"].shape[0]):
            c = lambda k, dt=np.float32: np.ascontiguousarray(g[f"s{seed}_{k}"][step], dt)
            acc, qw, tp, tv, zp, zv = c("acc"), c("q_wxyz"), c("trig_p", np.uint8), c("trig_v", np.uint8), c("pos"), c("vel")
            lib.pv_batch(f32, n, P(x), P(Pm), P(acc), P(qw), ctypes.c_float(float(g["dt"])), P(tp), P(zp), P(tv), P(zv))
            gx, gP = g[f"s{seed}_x"][step], g[f"s{seed}_P"][step]
            e[0] = max(e[0], relerr(x.astype(np.float64), gx)); e[1] = max(e[1], relerr(unpack_sym(Pm.astype(np.float64), 9), gP))
            e[2] = max(e[2], relerr(g[f"s{seed}_x_f32ref"][step].astype(np.float64), gx)); e[3] = max(e[3], relerr(g[f"s{seed}_P_f32ref"][step].astype(np.float64), gP))
        res[f32] = e
    for m, e in res.items(): print(seed, "mode", m, "x ratio %.0f P ratio %.0f" % (e[2]/max(e[0],1e-30), e[3]/max(e[1],1e-30)))
