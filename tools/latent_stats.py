"""Latent statistics behind the path-B speculation (tools only, runs on the C oracle):
per stream, how often a layer-0 latent equals 0, round(mu), its left / upper neighbour,
overall and on the 16x16 blocks holding a nonzero latent.  python tools/latent_stats.py FILE.cool ..."""
import ctypes as C, numpy as np, sys
L = C.CDLL(str(__import__('pathlib').Path(__file__).resolve().parents[1] / 'oracle' / '_build' / 'libccoracle.so'))
class F(C.Structure):
    _fields_ = [("h", C.c_int), ("w", C.c_int), ("fdt", C.c_int), ("bd", C.c_int), ("n_layers", C.c_int),
                ("lh", C.c_int * 8), ("lw", C.c_int * 8), ("lat", C.POINTER(C.c_int32) * 8), ("syn_in", C.c_void_p),
                ("n_out", C.c_int), ("syn_out", C.c_void_p), ("t", C.c_double * 3)]
for fn in sys.argv[1:]:
    bs = open(fn, 'rb').read()
    f = F()
    assert L.cco_decode_frame_mem(bs, len(bs), C.byref(f)) == 0
    mus = (C.POINTER(C.c_int32) * 8)(); lss = (C.POINTER(C.c_int32) * 8)()
    arrs = []
    for l in range(f.n_layers):
        n = f.lh[l] * f.lw[l]
        m = (C.c_int32 * n)(); s = (C.c_int32 * n)()
        arrs.append((m, s)); mus[l] = C.cast(m, C.POINTER(C.c_int32)); lss[l] = C.cast(s, C.POINTER(C.c_int32))
    L.cco_arm_params(bs, len(bs), C.byref(f), mus, lss)
    h, w = f.lh[0], f.lw[0]
    q = np.ctypeslib.as_array(f.lat[0], (h * w,)).reshape(h, w) >> 8
    mu = np.frombuffer(arrs[0][0], dtype=np.int32).reshape(h, w)
    mr = np.where(mu >= 0, ((mu + 128) >> 8), -((-mu + 128) >> 8))
    print(fn.split('/')[-1][:30], "P(q=0)=%.3f P(q=round(mu))=%.3f P(q=left)=%.3f P(q=up)=%.3f P(round(mu)=0)=%.3f" % (
        (q == 0).mean(), (q == mr).mean(), (q[:, 1:] == q[:, :-1]).mean(), (q[1:] == q[:-1]).mean(), (mr == 0).mean()))
    # coded-ish: 16x16 blocks holding a nonzero latent
    bh, bw = (h + 15) // 16, (w + 15) // 16
    nz = np.zeros((bh, bw), bool)
    for by in range(bh):
        for bx in range(bw):
            nz[by, bx] = (q[by*16:(by+1)*16, bx*16:(bx+1)*16] != 0).any()
    cm = np.kron(nz, np.ones((16, 16), bool))[:h, :w]
    left = np.zeros_like(q); left[:, 1:] = q[:, :-1]
    up = np.zeros_like(q); up[1:] = q[:-1]
    for name, g in (("zero", np.zeros_like(q)), ("left", left), ("up", up), ("round(mu)", mr)):
        hit = (q == g)[cm]
        print("   coded frac %.3f  guess %-9s hit %.3f" % (cm.mean(), name, hit.mean()))
