"""Diagnostic: compare wc_bold_chunk's state planes with a numpy restatement."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import oracle
from nremmodfc_amd import sigchain as wsg
from nremmodfc_amd.filters import bold_band, lfilter_zi
T, C, dec = 6000, 2, 1000
rng = np.random.default_rng(0)
E = 0.2 + 0.05 * rng.standard_normal((T, C))
bs = wsg.BoldStream(C, T, dec=dec)
bs.feed(torch.from_numpy(E).cuda())
torch.cuda.synchronize()
st = bs.state.cpu().numpy()
M = bs.M
o_ring = 4 * C + 4 * C + 16 * C + 16 * C
o_yzs = o_ring + dec * C
o_u = o_yzs + M * C
o_zend = o_u + 4 * M * C
b, a = bold_band(0.04); zi = lfilter_zi(b, a)
def step(z, x):
    y = z[0] + x * b[0]; z[0] = z[1] + x * b[1] - y * a[1]; z[1] = z[2] + x * b[2] - y * a[2]; z[2] = z[3] + x * b[3] - y * a[3]; z[3] = x * b[4] - y * a[4]; return y
bold = oracle.bold(E, 0.04)[2000:]
n = len(bold)
for c in range(C):
    x = bold[:, c]
    zf = zi * (2 * x[0] - x[15])
    for k in range(15, 0, -1): step(zf, 2 * x[0] - x[k])
    yf = np.array([step(zf, v) for v in x])
    yext = [step(zf, 2 * x[-1] - x[n - 2 - k]) for k in range(15)]
    zb = zi * yext[14]
    for k in range(14, -1, -1): step(zb, yext[k])
    print("col", c, "zend gpu", st[o_zend + np.arange(4) * C + c], "np", zb)
    for m in range(M):
        blk = yf[m * dec:(m + 1) * dec]; zs = np.zeros(4)
        for v in blk[::-1]: o = step(zs, v)
        print(" m", m, "yzs", st[o_yzs + m * C + c], o, "u", st[o_u + (m * 4 + np.arange(4)) * C + c], zs)
np.set_printoptions(precision=17)
out = bs.finish().cpu().numpy()
out2 = bs.finish().cpu().numpy()
print("twice equal", np.array_equal(out, out2))
print(out[:, 0])
# numpy longdouble finish on the GPU's planes
LD, CLD = np.longdouble, np.clongdouble
aL = a.astype(LD)
lam = np.roots(a).astype(CLD)
for _ in range(5):
    lam = lam - np.polyval(aL, lam) / np.polyval(np.polyder(aL), lam)
V = np.empty((4, 4), dtype=CLD)
for i, l in enumerate(lam):
    v1 = l + aL[1]; v2 = l * v1 + aL[2]; v3 = l * v2 + aL[3]
    V[:, i] = [CLD(1), v1, v2, v3]
Mx = np.concatenate([V, np.eye(4, dtype=CLD)], axis=1)
for cc in range(4):
    piv = np.argmax(np.abs(Mx[cc:, cc])) + cc; Mx[[cc, piv]] = Mx[[piv, cc]]; Mx[cc] /= Mx[cc, cc]
    for r in range(4):
        if r != cc: Mx[r] -= Mx[r, cc] * Mx[cc]
Vi = Mx[:, 4:]
import oracle.sigchain as osg
want = osg.sim_bold(E, 1000)
for c in range(C):
    w = Vi @ st[o_zend + np.arange(4) * C + c].astype(CLD)
    outs = np.zeros(M)
    for m in range(M - 1, -1, -1):
        outs[m] = float(LD(st[o_yzs + m * C + c]) + np.real(np.sum(lam ** (dec - 1) * w)))
        w = lam ** dec * w + Vi @ st[o_u + (m * 4 + np.arange(4)) * C + c].astype(CLD)
    print("np-on-gpu-planes", outs, "\noracle", want[:, c], "\ngpu", out[:, c] if c == 0 else bs.finish().cpu().numpy()[:, c])
