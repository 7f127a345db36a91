"""Hit rates of speculation guesses for the path-B latency kernel (tools only; CPU, the C oracle +
libccmi host weight parse): the row above, round(mu) with the true left neighbours, and round(mu)
with the left neighbours guessed from the row above (float ARM on the integer weights).
python tools/guess_stats.py FILE.cool ..."""
import sys, ctypes as C, numpy as np
sys.path.insert(0, '/root/repo/cool-chic_amd'); sys.path.insert(0, '/root/repo/tools')
from ccmi import decode
from pathlib import Path
L = C.CDLL('/root/repo/oracle/_build/libccoracle.so')
class F(C.Structure):
    _fields_ = [("h", C.c_int), ("w", C.c_int), ("fdt", C.c_int), ("bd", C.c_int), ("n_layers", C.c_int),
                ("lh", C.c_int * 8), ("lw", C.c_int * 8), ("lat", C.POINTER(C.c_int32) * 8), ("syn_in", C.c_void_p),
                ("n_out", C.c_int), ("syn_out", C.c_void_p), ("t", C.c_double * 3)]
K16 = [13, 14, 20, 21, 22, 23, 24, 28, 29, 30, 31, 32, 33, 37, 38, 39]
for fn in sys.argv[1:]:
    bs = open(fn, 'rb').read()
    f = F(); assert L.cco_decode_frame_mem(bs, len(bs), C.byref(f)) == 0
    arm, ups, syn = decode.weights_i32(bs)
    d = 16; nh = (len(arm) - 2 * d - 2) // (d * d + d)
    h, w = f.lh[0], f.lw[0]
    q = (np.ctypeslib.as_array(f.lat[0], (h * w,)).reshape(h, w) >> 8).astype(np.float64)
    P = np.zeros((h + 8, w + 8)); P[4:4+h, 4:4+w] = q
    up = np.zeros_like(q); up[1:] = q[:-1]
    def ctx(Pm, same_row=None):
        cols = []
        for k in K16:
            dy, dx = k // 9 - 4, k % 9 - 4
            v = Pm[4+dy:4+dy+h, 4+dx:4+dx+w]
            if dy == 0 and same_row is not None:
                v = same_row[dx]
            cols.append(v)
        return np.stack(cols, -1)
    def mlp(x):
        o = 0
        for l in range(nh):
            W = arm[o:o+d*d].reshape(d, d) / 256.; b = arm[o+d*d:o+d*d+d] / 65536.; o += d*d+d
            x = np.maximum(x @ W.T + b + x, 0)
        Wo = arm[o:o+2*d].reshape(2, d) / 256.; bo = arm[o+2*d:o+2*d+2] / 65536.
        return x @ Wo[0] + bo[0]
    mu = mlp(ctx(P))
    # approx: same-row left neighbours replaced by the latents above them
    Pu = np.zeros_like(P); Pu[4:4+h, 4:4+w] = up
    sr = {dx: Pu[4:4+h, 4+dx:4+dx+w] for dx in (-3, -2, -1)}
    mua = mlp(ctx(P, sr))
    bh, bw = (h + 15) // 16, (w + 15) // 16
    nz = np.zeros((bh, bw), bool)
    for by in range(bh):
        for bx in range(bw):
            nz[by, bx] = (q[by*16:(by+1)*16, bx*16:(bx+1)*16] != 0).any()
    cm = np.kron(nz, np.ones((16, 16), bool))[:h, :w]
    for name, g in (("up", up), ("round(mu)", np.round(mu)), ("round(mu_approx: left=up)", np.round(mua))):
        print(Path(fn).name[:28], "coded %.3f  %-26s hit %.3f" % (cm.mean(), name, (q == g)[cm].mean()))
