import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from conftest import golden
from oracle import oracle
from finitedifference_amd.solver import FOMContext
g = golden("ref_ops.npz")
for N in (16,):
    mu = tuple(g[f"n{N}_mu"]); w, r = g[f"n{N}_w"], g[f"n{N}_res"]
    ctx = FOMContext(N, N, tol=0.0); gx = np.linspace(0, 100, N+1)
    ctx.set_problem(gx, gx, 0.05, mu)
    d = ctx.block_solve(w, r)
    P = oracle.Problem(N, mu=mu); do = P.block_solve(w, r)
    bad = np.nonzero(d != do)[0]
    print('N', N, 'nbad', bad.size, 'first', bad[:10])
    n = N*N
    for i in bad[:5]:
        pl, k = divmod(i, n); rr, cc = divmod(k, N)
        print(' plane', pl, 'r', rr, 'c', cc, d[i], do[i], (d[i]-do[i])/do[i])
    # march
    wp = np.ones(2*n)
    for _ in range(3): wp = P.march_step(wp)
    s, st, its, _ = ctx.run(wp, 1)
    m = P.march_step(wp)
    bad = np.nonzero(s[:,1] != m)[0]
    print('march nbad', bad.size, bad[:10])
    for i in bad[:5]:
        pl, k = divmod(i, n); rr, cc = divmod(k, N)
        print(' plane', pl, 'r', rr, 'c', cc, s[i,1], m[i])
